#!/usr/bin/env python3
"""Benchmark: env steps/s of the HIP humanoid imitation env (BASELINE.json metric).

Workload (BASELINE.json configs[1]): 4096 lanes per GPU, low-level imitation on motion02_04, uniform
random actions in [-1,1] (pre-generated pool, device resident), auto-reset of done lanes inside the
step launch.  A "step" = one hum_step launch advancing every lane one env step (4 physics substeps +
observation + imitation reward + bookkeeping).  Multi-GPU: one process per GPU, lanes sharded by rank
(global lane ids -> identical per-lane streams regardless of N), no data-path collective -> weak scaling;
`--gather-every K` adds the trajectory gather (RCCL all-gather of obs / action / reward / done every K steps,
the only collective the path has), timed separately.

Prints ONE JSON line on rank 0.  Every number in it is measured in this run except `roofline.traffic`
(PMC bytes, profiles/pmc_traffic.json, from a rocprofv3 --pmc pass of this same command) and the static FLOP
count per env-step (profiles/r02_flops_per_env_step.json, tools/flop_count.py).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "imitation-learning-rl_amd"))

# algorithmic HBM bytes per env-step: action 17 x f32 read; physics state 47 x f32 read + write;
# bookkeeping 24 words x 4 B read + write; obs 70 x f32, reward f32, frame i32, done u8 written = 925 B.
BYTES_PER_STEP_ALGO = 17 * 4 + 2 * 47 * 4 + 2 * 24 * 4 + 70 * 4 + 4 + 4 + 1
# the kernel's actual layout per env-step: bookkeeping 23 f64 + 8 i32 instead of 24 words
BYTES_PER_STEP_LAYOUT = 2 * 47 * 4 + 2 * (23 * 8 + 8 * 4) + 17 * 4 + 70 * 4 + 4 + 1 + 4
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E (MI355X_MICROARCH.md)
FP32_PEAK_TFLOPS = 157.3       # MI355X FP32 vector (MI355X_MICROARCH.md)
FP64_PEAK_TFLOPS = 78.6        # MI355X FP64 vector


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--lanes", type=int, default=4096, help="env lanes per GPU")
    ap.add_argument("--clip", default="motion02_04", help="clip name, or 'all' = the four CMU clips round-robin per "
                                                          "lane (BASELINE config 3)")
    ap.add_argument("--precision", default="fp32", choices=["fp32", "fp64"])
    ap.add_argument("--block", type=int, default=64)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget (0 = skip)")
    ap.add_argument("--cpu-workers", type=int, default=0, help="CPU baseline threads (0 = the job's host cores)")
    ap.add_argument("--phys", action="append", default=[], help="physics override k=v (hum_config field), diagnostics")
    ap.add_argument("--hier", action="store_true",
                    help="config 5: HierarchicalHumanoidEnv two-level rollout (hum_hier_step), clip motion09_03")
    ap.add_argument("--gather-every", type=int, default=0, help="multi-GPU: trajectory all-gather every K steps")
    ap.add_argument("--policy", action="store_true",
                    help="closed loop: actions from the on-GPU policy network (random-init weights, exploration "
                         "noise) inside the timed loop, SURVEY 8(f) rank 2")
    ap.add_argument("--no-secondary", action="store_true", help="skip the fp64 / parity side measurements")
    return ap.parse_args()


def host_cores():
    """Host cores this job may use: the box's CPU share (OMP_NUM_THREADS / MAX_JOBS are set to it on the GPU
    box; os.cpu_count() there reports the whole machine), else the affinity mask."""
    for k in ("OMP_NUM_THREADS", "MAX_JOBS"):
        v = os.environ.get(k)
        if v and v.isdigit() and int(v) > 0:
            return int(v)
    try:
        return len(os.sched_getaffinity(0))
    except Exception:
        return os.cpu_count() or 1


def cpu_baseline(seconds, threads):
    """CPU baseline (PyBullet absent -> the build's C restatement with OpenMP over the job's host
    cores): oracle/env_oracle.c (fp64 physics restatement + the env logic, bit-identical to the Python oracle) with
    one lane per thread stepping uniform random actions, reset on done."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import env_oracle as EO
    from ilrl_amd.clips import load_clip
    steps, wall = EO.bench(load_clip("motion02_04"), threads, seconds)
    return {"value": steps / wall, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": "oracle/env_oracle.c (fp64 C restatement of physics + env logic, OpenMP; PyBullet absent) on "
                      "motion02_04, %d threads (the job's host cores) x %.0f s of uniform-random-action steps with "
                      "resets (%d steps)" % (threads, seconds, steps)}


def parity_sample(env, clips, per_clip=64, seed=5, sens_bound=1e-5):
    """CPU checker leg (after the timed region): from the benchmark's own mid-rollout state, step once more on the
    GPU (no auto-reset) with the benchmarked fp32 kernel AND with the fp64 kernel given the identical state, and
    compare a sample of lanes per clip with the fp64 oracle stepped from the same injected state (fp64 C physics +
    the env logic).  Each lane's conditioning is measured too: the oracle stepped again from the state perturbed by
    2^-24 relative (float32 rounding) - a joint limit or contact that switches on within that margin makes the step
    discontinuous, and such lanes are reported apart (the error there is the model's, not the kernel's)."""
    import numpy as np
    import torch
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    from ilrl_amd import _native as N
    from ilrl_amd.clips import load_clip
    from ilrl_amd.vec_env import HumanoidVecEnv
    phys, book = env.get_state()
    n = env.n
    a = np.random.default_rng(seed).uniform(-1, 1, (n, 17)).astype(np.float32)
    at = torch.as_tensor(a, device=env.device)
    obs, rew, done, frame = [x.cpu().numpy() for x in env.step(at)]
    env64 = HumanoidVecEnv(n, clips=clips, seed=0, device=env.device.index, precision="fp64")
    env64.set_state(phys, book)
    obs64, rew64, done64, _ = [x.cpu().numpy() for x in env64.step(at)]
    st64, _ = env64.get_state()
    env64.close()
    prng = np.random.default_rng(seed + 1)
    eo, er, e64, r64, s64, sens, dm, fm, dm64, lanes = [], [], [], [], [], [], 0, 0, 0, 0
    for c, name in enumerate(clips):
        idx = np.nonzero(book[:, N.BK["clip"]].astype(int) == c)[0]
        if name == "motion13_13":   # the reference raises IndexError past the 120-row velocity table
            idx = idx[book[idx, N.BK["frame"]] + 2 < 120]
        clip = load_clip(name)
        for i in idx[np.linspace(0, len(idx) - 1, min(per_clip, len(idx))).astype(int)]:
            o = O.OracleLowLevelEnv.from_lane(clip, phys[i], book[i], N.BK)
            ro, rr, rd, _ = o.step(a[i])
            eo.append(float(np.abs(obs[i] - ro).max()))
            er.append(abs(float(rew[i]) - rr))
            e64.append(float(np.abs(obs64[i] - ro).max()))
            r64.append(abs(float(rew64[i]) - rr))
            s64.append(float(np.abs(st64[i] - o.state).max()))
            dm += int(bool(done[i]) != rd)
            dm64 += int(bool(done64[i]) != rd)
            fm += int(int(frame[i]) != o.frame)
            p = O.OracleLowLevelEnv.from_lane(clip, phys[i] * (1 + 2.0 ** -24 * prng.choice([-1.0, 1.0], 47)), book[i],
                                              N.BK)
            sens.append(float(np.abs(p.step(a[i])[0] - ro).max()))
            lanes += 1
    eo, er, sens = np.array(eo), np.array(er), np.array(sens)
    good = sens <= sens_bound
    return {"vs": "fp64 CPU oracle, one env step from the benchmark's own mid-rollout lane states (PyBullet absent: "
                  "parity vs PyBullet unpinned)", "lanes": lanes,
            "obs_max_abs_err": float(eo.max()), "obs_p99_abs_err": float(np.percentile(eo, 99)),
            "reward_max_abs_err": float(er.max()), "done_mismatches": dm, "frame_mismatches": fm,
            "ill_conditioned_lanes": int((~good).sum()),
            "obs_max_abs_err_conditioned": float(eo[good].max()) if good.any() else None,
            "reward_max_abs_err_conditioned": float(er[good].max()) if good.any() else None,
            "conditioning": "oracle obs change under a 2^-24 relative input perturbation > %g" % sens_bound,
            "fp64_kernel": {"obs_max_abs_err": float(max(e64)), "reward_max_abs_err": float(max(r64)),
                            "state_max_abs_err": float(max(s64)), "done_mismatches": dm64}}


def _load_json(path):
    try:
        return json.load(open(os.path.join(REPO, path)))
    except Exception:
        return None


def run(a, world, rank, dev, n, precision, steps, warmup, phys):
    """Build the env, warm up, time `steps` launches.  Returns (env, wall_max_s, kernel_ms, low_steps)."""
    import torch
    import torch.distributed as dist
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    pool = [(torch.rand(n, 17, device=dev, generator=g) * 2 - 1).contiguous() for _ in range(16)]
    if a.hier:
        from ilrl_amd.hier_env import HierVecEnv
        env = HierVecEnv(n, seed=0, device=dev.index, lane_offset=rank * n, precision=precision, block_size=a.block,
                         **phys)
        hpool = [(torch.rand(n, 2, device=dev, generator=g) * 2 - 1).contiguous() for _ in range(16)]
        step = lambda s: env.step(hpool[s % 16], pool[s % 16], autoreset=True)
    else:
        from ilrl_amd.clips import CLIP_NAMES
        from ilrl_amd.vec_env import HumanoidVecEnv
        clips = tuple(CLIP_NAMES) if a.clip == "all" else (a.clip,)
        env = HumanoidVecEnv(n, clips=clips, seed=0, device=dev.index, lane_offset=rank * n, precision=precision,
                             block_size=a.block, **phys)
        step = lambda s: env.step(pool[s % 16], autoreset=True)
        if a.policy:
            from ilrl_amd.policy import DevicePolicy
            pol = DevicePolicy.random_init(seed=7 + rank, device=dev.index)
            actbuf = torch.zeros(n, 17, device=dev)

            def step(s):
                pol.act(env.obs, env.obs_reset, env.done, explore=True, step=s, out=actbuf)
                return env.step(actbuf, autoreset=True)
    env.reset()
    env.done.zero_()
    for w in range(warmup):
        step(w)
    gather_s = 0.0
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for s in range(steps):
        step(s)
        if a.gather_every and world > 1 and (s + 1) % a.gather_every == 0:
            from ilrl_amd.parallel import gather_trajectories
            tg = time.perf_counter()
            gather_trajectories([env.obs, pool[s % 16], env.reward, env.done], dst=0)
            gather_s += time.perf_counter() - tg
    ev1.record()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / steps   # average launch duration on the launch stream (torch's current)
    t = torch.tensor([wall], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    low_steps = None
    if a.hier:   # physics env-steps in the timed region: replay the same deterministic sequence and count them
        lt = torch.tensor([count_hier_low_steps(a, dev, n, precision, steps, warmup, phys, rank)], dtype=torch.float64,
                          device=dev)
        if world > 1:
            dist.all_reduce(lt)
        low_steps = float(lt.item())   # all ranks
    return env, float(t.item()), kern_ms, low_steps, gather_s


def count_hier_low_steps(a, dev, n, precision, steps, warmup, phys, rank):
    """Lanes that take a low-level (physics) step in each of the timed launches: a lane acts high next iff its
    last outputs carried the high-level obs (level hand-back, or done -> auto-reset)."""
    import torch
    from ilrl_amd import _native as N
    from ilrl_amd.hier_env import HierVecEnv
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    pool = [(torch.rand(n, 17, device=dev, generator=g) * 2 - 1).contiguous() for _ in range(16)]
    hpool = [(torch.rand(n, 2, device=dev, generator=g) * 2 - 1).contiguous() for _ in range(16)]
    env = HierVecEnv(n, seed=0, device=dev.index, lane_offset=rank * n, precision=precision, block_size=a.block, **phys)
    env.reset()
    expect_high = torch.ones(n, dtype=torch.bool, device=dev)
    low = 0
    for s in range(warmup + steps):
        if s >= warmup:
            low += int((~expect_high).sum().item())
        agents, _, _, _, _, done, _ = env.step(hpool[s % 16], pool[s % 16], autoreset=True)
        expect_high = ((agents & N.HUM_AGENT_HIGH) != 0) | (done != 0)
    env.close()
    return low


def main():
    a = parse()
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    n = a.lanes
    phys = {}
    for kv in a.phys:
        k, v = kv.split("=")
        phys[k] = float(v) if "." in v else int(v)
    if a.hier:
        from ilrl_amd.hier_env import HIER_CLIP
        a.clip = HIER_CLIP
    env, wall_max, kern_ms, low_steps, gather_s = run(a, world, rank, dev, n, a.precision, a.steps, a.warmup, phys)
    flags = env.error_flags()
    if rank == 0:
        total = n * world * a.steps
        phys_steps_per_launch = (low_steps / world / a.steps) if a.hier else n   # per GPU
        value = (low_steps if a.hier else total) / wall_max
        flops_j = _load_json("profiles/r02_flops_per_env_step.json")
        flops = flops_j["flops_per_env_step_mean"] if flops_j else None
        achieved = phys_steps_per_launch * BYTES_PER_STEP_ALGO / (kern_ms * 1e-3) / 1e9
        traffic = None
        tj = _load_json("profiles/pmc_traffic.json") or {}
        key = "%s_%d_%s" % ("hier" if a.hier else a.clip, n, a.precision)
        if key in tj:
            traffic = tj[key]["bytes_per_launch"]
        out = {
            "metric": "env steps/sec at N parallel humanoids, 1/2/4/8 MI355X; obs/reward max-abs-err vs PyBullet",
            "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": wall_max / a.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": a.precision.replace("fp", "f"), "data": "synthetic",
            "config": {"workload": ("HumanoidBulletEnv-v0-Hier two-level rollout (high heading every 5 low steps), "
                                    if a.hier else "HumanoidBulletEnv-v0-Low step+reward, ") +
                                   "%s, %d envs/GPU, %s, auto-reset" % (
                                       a.clip, n, "on-GPU policy actions (random-init 70-256-256-17 tanh MLP + "
                                       "Gaussian exploration) in the loop" if a.policy else "uniform random actions"),
                       "envs_per_gpu": n, "clip": a.clip,
                       "parallelism": "lane-sharded x%d" % world, "block": a.block, "physics_overrides": phys},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "bytes_per_env_step": BYTES_PER_STEP_ALGO, "bytes_per_env_step_layout": BYTES_PER_STEP_LAYOUT,
                         "kernel_ms": kern_ms},
            "error_flags": flags,
        }
        if flops:
            peak = FP32_PEAK_TFLOPS if a.precision == "fp32" else FP64_PEAK_TFLOPS
            tf = phys_steps_per_launch * flops / (kern_ms * 1e-3) / 1e12
            out["roofline_valu"] = {"bound": "valu-%s" % a.precision, "achieved": tf, "peak": peak, "unit": "TFLOP/s",
                                    "frac": tf / peak, "flops_per_env_step": flops,
                                    "source": "profiles/r02_flops_per_env_step.json (tools/flop_count.py)"}
        if a.hier:
            out["unit"] = "env-steps/s"
            out["physics_env_steps_per_launch"] = phys_steps_per_launch
            out["agent_transitions_per_s"] = total / wall_max
        if world > 1 and a.gather_every:
            out["gather"] = {"every": a.gather_every, "seconds": gather_s,
                             "bytes_per_rank_per_step": n * (70 * 4 + 17 * 4 + 4 + 1)}
        if world == 1 and not a.no_secondary and not a.hier and not a.policy:
            from ilrl_amd.clips import CLIP_NAMES
            clips = tuple(CLIP_NAMES) if a.clip == "all" else (a.clip,)
            out["parity"] = parity_sample(env, clips)
            other = "fp64" if a.precision == "fp32" else "fp32"
            env2, w2, k2, _, _ = run(a, 1, 0, dev, n, other, 200, 20, phys)
            env2.close()
            out["secondary"] = {other: {"value": n * 200 / w2, "ms_per_step": w2 / 200 * 1e3, "kernel_ms": k2,
                                        "steps": 200, "warmup": 20}}
            if "split_penetration" not in phys:
                # continuity with the bench lines measured before the split-impulse model:
                # the same kernel on the previous workload (every limit / contact violation corrected at ERP)
                prev = dict(phys, split_penetration=-1e30)
                env3, w3, k3, _, _ = run(a, 1, 0, dev, n, a.precision, 200, 20, prev)
                env3.close()
                out["secondary"]["previous_model_split_off"] = {
                    "value": n * 200 / w3, "ms_per_step": w3 / 200 * 1e3, "kernel_ms": k3, "steps": 200, "warmup": 20}
        if world == 1 and a.cpu_seconds > 0 and not a.hier:
            out["cpu_baseline"] = cpu_baseline(a.cpu_seconds, a.cpu_workers or host_cores())
        print(json.dumps(out), flush=True)
    env.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
