#!/usr/bin/env python3
"""Static-algorithm FP32 FLOPs per env-step of the physics (tools/flop_count.cpp) over the benchmark workload's
state distribution: oracle rollouts (oracle/, CPU) of motion02_04 with uniform random actions in [-1, 1] and
auto-reset, the same workload bench.py times.  Prints a JSON summary; --out writes it (profiles/).

The FLOP count is of the per-lane formulation (physics.h); the cooperative kernel runs the same algorithm
(spread over 16 lanes) plus redundant work (padded dofs, zero rows, masked lanes), which is overhead, not
algorithm, and is excluded.  The float64 env logic (obs, reward, bookkeeping, ~1 lane per env) is excluded."""
import argparse
import json
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "oracle"), os.path.join(REPO, "imitation-learning-rl_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lanes", type=int, default=16)
    ap.add_argument("--steps", type=int, default=250)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import oracle as O
    from ilrl_amd.clips import load_clip
    exe = "/tmp/flop_count"
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-o", exe, os.path.join(REPO, "tools", "flop_count.cpp")])
    clip = load_clip("motion02_04")
    recs, ncon = [], []
    for lane in range(a.lanes):
        env = O.OracleLowLevelEnv(clip, seed=1234, lane=lane)
        env.reset()
        rng = np.random.default_rng(lane)
        for _ in range(a.steps):
            act = rng.uniform(-1, 1, 17).astype(np.float32)
            recs.append((env.state.copy(), act))
            ncon.append(len(O.contacts(env.state)))
            _, _, d, _ = env.step(act)
            if d:
                env.reset()
    path = "/tmp/flop_records.bin"
    with open(path, "wb") as f:
        for st, act in recs:
            f.write(np.asarray(st, np.float64).tobytes())
            f.write(np.asarray(act, np.float32).tobytes())
    flops = np.array([int(x) for x in subprocess.check_output([exe, path]).split()])
    ncon = np.array(ncon)
    out = {"flops_per_env_step_mean": float(flops.mean()), "p50": float(np.median(flops)),
           "p99": float(np.percentile(flops, 99)), "min": int(flops.min()), "max": int(flops.max()),
           "samples": int(len(flops)), "contacts_mean": float(ncon.mean()), "contacts_max": int(ncon.max()),
           "by_contacts": {int(c): float(flops[ncon == c].mean()) for c in np.unique(ncon)},
           "workload": "oracle rollouts, motion02_04, uniform random actions, auto-reset (%d lanes x %d steps)"
                       % (a.lanes, a.steps)}
    print(json.dumps(out))
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
