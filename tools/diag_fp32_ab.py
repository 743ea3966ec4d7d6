#!/usr/bin/env python3
"""Diagnostic: fp32 step accuracy of two (or more) builds of the library FROM THE SAME STATES.

The full-size parity test samples 64 lanes from a rollout whose states depend on the build (the rollout is
chaotic), so a max over those lanes compares different state samples between builds.  Here one rollout (the
default library) produces the states; every library in LIBS then steps exactly those states once (a fresh process
per library, ILRL_AMD_LIB), and all are compared with the fp64 oracle and the fp32 oracle yardstick on the same
N lanes (the test's per-block statistics: max, p99, p90, p50).

usage: LIBS="base new new@0" [N=512] [STEPS=192] python3 tools/diag_fp32_ab.py   (on a GPU box; writes gpurun_out/fp32ab/)
"""
import json
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "imitation-learning-rl_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))
OUT = os.path.join(REPO, "gpurun_out", "fp32ab")
LIBDIR = os.path.join(REPO, "imitation-learning-rl_amd", "ilrl_amd", "_lib")
N_ENV = 4096
BLOCKS = {"body": np.arange(0, 8), "joint_pos": np.arange(8, 42, 2), "joint_vel": np.arange(9, 42, 2)}


def lib_path(v):   # "name" or "name@K": the library libhumenv_<name>.so ("new": libhumenv.so), kernel K (default 1)
    v = v.split("@")[0]
    return os.path.join(LIBDIR, "libhumenv.so" if v == "new" else "libhumenv_%s.so" % v)


def make_states():
    import torch
    from ilrl_amd.vec_env import HumanoidVecEnv
    env = HumanoidVecEnv(N_ENV, clips=("motion02_04",), seed=21, precision="fp32")
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(4)
    for _ in range(int(os.environ.get("STEPS", "192"))):
        env.step(torch.rand(N_ENV, 17, device="cuda", generator=g) * 2 - 1, autoreset=True)
    phys, book = env.get_state()
    env.close()
    a = np.random.default_rng(5).uniform(-1, 1, (N_ENV, 17)).astype(np.float32)
    np.savez(os.path.join(OUT, "states.npz"), phys=phys, book=book, a=a)


def step_states(tag):
    import torch
    from ilrl_amd.vec_env import HumanoidVecEnv
    z = np.load(os.path.join(OUT, "states.npz"))
    kernel = int(tag.split("@")[1]) if "@" in tag else 1   # 0: the per-lane kernel (physics.h)
    env = HumanoidVecEnv(N_ENV, clips=("motion02_04",), seed=21, precision="fp32", kernel=kernel)
    env.set_state(z["phys"], z["book"])
    obs, rew, done, frame = [x.cpu().numpy() for x in env.step(torch.as_tensor(z["a"], device="cuda"))]
    env.close()
    np.savez(os.path.join(OUT, "step_%s.npz" % tag), obs=obs, rew=rew)


def compare(libs):
    from ilrl_amd.clips import load_clip
    from oracle_inject import oracle_from_lane
    z = np.load(os.path.join(OUT, "states.npz"))
    phys, book, a = z["phys"], z["book"], z["a"]
    outs = {v: np.load(os.path.join(OUT, "step_%s.npz" % v)) for v in libs}
    clip = load_clip("motion02_04")
    n = int(os.environ.get("N", "512"))
    lanes = np.linspace(0, N_ENV - 1, n).astype(int)
    prng, prng32 = np.random.default_rng(6), np.random.default_rng(7)
    err = {v: [] for v in libs}
    o32, o32env, sens = [], [], []
    for i in lanes:
        ro, rr, rd, _ = oracle_from_lane(clip, phys[i], book[i]).step(a[i])
        for v in libs:
            err[v].append(np.abs(outs[v]["obs"][i] - ro))
        env_o = np.zeros(70)
        for rz in range(4):
            pst = phys[i] if rz == 0 else phys[i] * (1 + 2.0 ** -24 * prng32.choice([-1.0, 1.0], 47))
            r32o = oracle_from_lane(clip, pst, book[i], phys_precision="fp32").step(a[i])[0]
            if rz == 0:
                o32.append(np.abs(r32o - ro))
            env_o = np.maximum(env_o, np.abs(r32o - ro))
        o32env.append(env_o)
        p = oracle_from_lane(clip, phys[i] * (1 + 2.0 ** -24 * prng.choice([-1.0, 1.0], 47)), book[i])
        sens.append(np.abs(p.step(a[i])[0] - ro).max())
    good = np.array(sens) <= 1e-5
    res = {"lanes": int(n), "well_conditioned": int(good.sum())}
    rows = {"fp32_oracle": np.array(o32)[good], "fp32_envelope": np.array(o32env)[good]}
    rows.update({v: np.array(err[v])[good] for v in libs})
    for b, ix in BLOCKS.items():
        res[b] = {}
        for name, m in rows.items():
            x = m[:, ix].max(1)
            res[b][name] = {"max": float(x.max()), "p99": float(np.percentile(x, 99)), "p90": float(np.percentile(x, 90)),
                            "p50": float(np.median(x)), "mean": float(x.mean())}
        for v in libs:   # per-lane ratio to the same lane's envelope
            r = rows[v][:, ix].max(1) / np.maximum(rows["fp32_envelope"][:, ix].max(1), 1e-9)
            res[b]["ratio_%s" % v] = {"p50": float(np.median(r)), "p90": float(np.percentile(r, 90)),
                                      "p99": float(np.percentile(r, 99)), "max": float(r.max())}
    json.dump(res, open(os.path.join(OUT, "fp32ab.json"), "w"), indent=1)
    for b in BLOCKS:
        print("== %s" % b)
        for name in rows:
            s = res[b][name]
            print("  %-14s max %.3e  p99 %.3e  p90 %.3e  p50 %.3e  mean %.3e" % (name, s["max"], s["p99"], s["p90"], s["p50"], s["mean"]))
        for v in libs:
            s = res[b]["ratio_%s" % v]
            print("  ratio %-8s (kernel / same-lane envelope) p50 %.2f  p90 %.2f  p99 %.2f  max %.2f" % (v, s["p50"], s["p90"], s["p99"], s["max"]))


def main():
    os.makedirs(OUT, exist_ok=True)
    mode = sys.argv[1] if len(sys.argv) > 1 else "all"
    libs = os.environ.get("LIBS", "base new").split()
    if mode == "states":
        make_states()
    elif mode == "step":
        step_states(sys.argv[2])
    elif mode == "compare":
        compare(libs)
    else:
        env = dict(os.environ, ILRL_AMD_AB="1")
        subprocess.check_call([sys.executable, __file__, "states"], env=env)
        for v in libs:
            subprocess.check_call([sys.executable, __file__, "step", v], env=dict(env, ILRL_AMD_LIB=lib_path(v)))
        compare(libs)


if __name__ == "__main__":
    main()
