"""Bitwise A/B of two library builds (a change meant to be bitwise-neutral, e.g. the chain-parallel FK).

usage: diag_lib_bitwise.py dump OUT.npz   (ILRL_AMD_LIB = the build: fixed-seed rollouts, every output saved)
       diag_lib_bitwise.py cmp A.npz B.npz
Rollouts: config 2 fp32 (1024 lanes, 64 random-action steps in launches of 32, auto-reset), the same fp64, the
hierarchical env fp32 (512 lanes, 64 transitions), the per-lane kernel fp32 (256 lanes, 16 steps)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "imitation-learning-rl_amd"))


def dump(path):
    import torch
    from ilrl_amd.hier_env import HierVecEnv
    from ilrl_amd.vec_env import HumanoidVecEnv
    out = {}
    g = torch.Generator(device="cuda").manual_seed(21)
    for tag, n, steps, kw in (("c2_fp32", 1024, 64, {}), ("c2_fp64", 1024, 64, {"precision": "fp64"}),
                              ("lane_fp32", 256, 16, {"kernel": 0})):
        env = HumanoidVecEnv(n, clips=("motion02_04",), seed=3, **kw)
        env.reset()
        k = min(32, steps)
        for s in range(steps // k):
            a = torch.rand(k, n, 17, device="cuda", generator=g) * 2 - 1
            o = env.step_k(a, autoreset=True)
            for j, x in enumerate(o):
                out["%s_%d_%d" % (tag, s, j)] = x.cpu().numpy()
        out[tag + "_phys"], out[tag + "_book"] = env.get_state()
        out[tag + "_flags"] = np.array([env.error_flags()])
        env.close()
    env = HierVecEnv(512, seed=5)
    env.reset()
    for s in range(2):
        o = env.step_k(torch.rand(32, 512, 2, device="cuda", generator=g) * 2 - 1,
                       torch.rand(32, 512, 17, device="cuda", generator=g) * 2 - 1, autoreset=True)
        for j, x in enumerate(o):
            out["hier_%d_%d" % (s, j)] = x.cpu().numpy()
    out["hier_phys"], out["hier_book"] = env.get_state()
    env.close()
    np.savez(path, **out)
    print("dumped %d arrays to %s" % (len(out), path))


def cmp(a, b):
    A, B = np.load(a), np.load(b)
    bad = 0
    for k in sorted(A.files):
        x, y = A[k], B[k]
        same = x.shape == y.shape and x.tobytes() == y.tobytes()
        if not same:
            bad += 1
            d = np.abs(x.astype(np.float64) - y.astype(np.float64))
            idx = np.unravel_index(d.argmax(), d.shape)
            nd = np.argwhere(d > 0)
            print("DIFF %-16s max |a-b| %.3g at %s (a %r, b %r); %d entries differ, first at %s" % (
                k, d.max(), idx, x[idx], y[idx], len(nd), tuple(nd[0]) if len(nd) else None))
    print("%d of %d arrays differ" % (bad, len(A.files)))
    return bad


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        sys.exit(1 if cmp(sys.argv[2], sys.argv[3]) else 0)
