"""Per-phase VALU lane utilisation of the benchmarked kernel.

usage: lane_util.py save OUT.npz    (default library: 4096 lanes x motion02_04, 200 random-action env steps in
                                     launches of k = 32 from a reset, then the physics state + bookkeeping saved)
       lane_util.py run STATE.npz   (ILRL_AMD_LIB = a variant: 4 single-step launches, each from the saved state)
       lane_util.py dump DIR        (DIR/<variant>/**/run_results.db from rocprofv3 --pmc -> DIR/<variant>.json)
       lane_util.py summary DIR     (the per-phase table from DIR/calib.json and DIR/lu*.json)

Variants (tools/build_variant.sh): lu0 .. lu8 = group_f32.hip with -DHUM_STOP_AFTER=k (every substep ends after
phase k), lu9 = the whole substep without the env logic (-DHUM_SKIP_POST), luall = the full kernel.  Phase k's counts
are variant k minus variant k - 1, all stepped from the same saved states (identical work up to the cut); env logic =
luall - lu9.  Lane utilisation = SQ_THREAD_CYCLES_VALU / (64 x VALU instruction cycles), the instruction cycles
calibrated by tools/micro/lane_util.hip (exec masks of 64 / 32 / 16 / 4 / 1 lanes)."""
import glob
import os
import sqlite3
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "imitation-learning-rl_amd"))
N_LANES = 4096
PHASES = ["launch / state load / sincos (substep entry)", "FK", "ABA pass 1", "ABA pass 2", "base + pass 3",
          "geoms + limits", "contacts", "rows", "PGS", "integrate"]
COUNTERS = ["SQ_INSTS_VALU", "SQ_THREAD_CYCLES_VALU", "SQ_ACTIVE_INST_VALU", "SQ_INSTS_VALU_FLOPS_FP32", "SQ_WAVES",
            "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES"]


def save(path):
    import torch
    from ilrl_amd.vec_env import HumanoidVecEnv
    env = HumanoidVecEnv(N_LANES, clips=("motion02_04",), seed=0)
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(11)
    for _ in range(200 // 32 + 1):
        env.step_k(torch.rand(32, N_LANES, 17, device="cuda", generator=g) * 2 - 1, autoreset=True)
    phys, book = env.get_state()
    np.savez(path, phys=phys, book=book)
    print("saved %d lanes to %s" % (N_LANES, path))


def run(path):
    import torch
    from ilrl_amd.vec_env import HumanoidVecEnv
    z = np.load(path)
    env = HumanoidVecEnv(N_LANES, clips=("motion02_04",), seed=0)
    env.reset()
    a = (torch.rand(1, N_LANES, 17, device="cuda", generator=torch.Generator(device="cuda").manual_seed(5)) * 2 - 1)
    for _ in range(4):
        env.set_state(z["phys"], z["book"])
        env.step_k(a, autoreset=True)
    torch.cuda.synchronize()
    print("4 launches from the saved state, flags %#x" % env.error_flags())


def counters(db, kp):
    c = sqlite3.connect(db)
    out = {}
    for name, v, n in c.execute("select counter_name, sum(value), count(distinct dispatch_id) from counters_collection "
                                "where kernel_name like ? group by counter_name", ("%" + kp + "%",)):
        out[name] = v / max(n, 1)   # per launch
    return out


def dump(d):
    """DIR/<variant>/**/run_results.db -> DIR/<variant>.json (the counters this study reads; the database goes)."""
    import json
    import shutil
    for sub in sorted(glob.glob(os.path.join(d, "*", ""))):
        name = os.path.basename(os.path.dirname(sub))
        dbs = glob.glob(os.path.join(sub, "**", "*results.db"), recursive=True)
        if not dbs:
            continue
        if name == "calib":
            out = {str(m): counters(dbs[0], "lanes_active<%d>" % m) or counters(dbs[0], "lanes_activeILi%dE" % m)
                   for m in (64, 32, 16, 4, 1)}
        else:
            out = counters(dbs[0], "step_group_kernel")
        json.dump(out, open(os.path.join(d, name + ".json"), "w"), indent=1)
        shutil.rmtree(sub)


def summary(d):
    import json
    cal = {int(m): c for m, c in json.load(open(os.path.join(d, "calib.json"))).items()}
    lines = ["# VALU counter calibration (tools/micro/lane_util.hip, 1024 waves x 16384 fma per active lane)",
             "# M active lanes: INSTS_VALU/wave, ACTIVE_INST_VALU/wave (quad-cycles), THREAD_CYCLES_VALU/wave, "
             "THREAD_CYCLES / INSTS"]
    tc_per_lane_inst = None
    for m in sorted(cal, reverse=True):
        c = cal[m]
        if not c:
            continue
        w = c.get("SQ_WAVES", 1024) or 1024
        ratio = c["SQ_THREAD_CYCLES_VALU"] / c["SQ_INSTS_VALU"]
        lines.append("  M=%2d  insts %.0f  active %.0f  thread_cycles %.0f  thread_cycles/inst %.2f  FP32 FLOP/wave %.0f" % (
            m, c["SQ_INSTS_VALU"] / w, c["SQ_ACTIVE_INST_VALU"] / w, c["SQ_THREAD_CYCLES_VALU"] / w, ratio,
            c.get("SQ_INSTS_VALU_FLOPS_FP32", 0) / w))
        if m == 64:
            tc_per_lane_inst = ratio / 64
    var = {os.path.basename(f)[:-5]: json.load(open(f)) for f in glob.glob(os.path.join(d, "lu*.json"))}
    lines.append("# per launch of 4096 lanes (1024 waves), one env step; phase k = variant k - variant k-1")
    lines.append("%-46s %12s %8s %14s %8s %10s %10s" % ("phase", "VALU insts", "/wave", "thread-cycles", "lanes",
                                                          "FP32 FLOP", "cyc/wave"))
    prev = None
    rows = []
    order = ["lu%d" % k for k in range(10)] + ["luall"]
    labels = PHASES + ["env logic + outputs (lane 0 per env)"]
    for v, lab in zip(order, labels):
        c = var.get(v)
        if c is None:
            lines.append("%-46s (missing)" % lab)
            prev = None
            continue
        cur = np.array([c.get(k, 0.0) for k in COUNTERS])
        dlt = cur - prev if prev is not None else cur
        prev = cur
        insts, tcyc, flops, waves = dlt[0], dlt[1], dlt[3], c.get("SQ_WAVES", 1024) or 1024
        lanes = tcyc / (insts * tc_per_lane_inst) if insts > 0 and tc_per_lane_inst else float("nan")
        rows.append((lab, insts, tcyc, lanes, flops))
        lines.append("%-46s %12.0f %8.0f %14.0f %8.1f %10.0f %10.0f" % (lab, insts, insts / waves, tcyc, lanes, flops,
                                                                      4 * dlt[7] / waves))
    if "luall" in var:
        c = var["luall"]
        tot_i, tot_t = c["SQ_INSTS_VALU"], c["SQ_THREAD_CYCLES_VALU"]
        lines.append("%-46s %12.0f %8.0f %14.0f %8.1f %10.0f" % (
            "whole step (luall)", tot_i, tot_i / (c.get("SQ_WAVES", 1024) or 1024), tot_t,
            tot_t / (tot_i * tc_per_lane_inst) if tc_per_lane_inst else float("nan"), c.get("SQ_INSTS_VALU_FLOPS_FP32", 0)))
    print("\n".join(lines))


if __name__ == "__main__":
    {"save": save, "run": run, "dump": dump, "summary": summary}[sys.argv[1]](sys.argv[2])
