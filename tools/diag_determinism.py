#!/usr/bin/env python3
"""Diagnostic: two handles fed identical inputs must stay bitwise identical (hier and low-level, both kernels);
prints the first iteration / lane / bookkeeping column where they diverge."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "imitation-learning-rl_amd"))
from ilrl_amd import _native as N  # noqa: E402
from ilrl_amd.hier_env import HierVecEnv  # noqa: E402
from ilrl_amd.vec_env import HumanoidVecEnv  # noqa: E402

INV = {v: k for k, v in N.BK.items()}


def compare(tag, envs, it):
    p0, b0 = envs[0].get_state()
    p1, b1 = envs[1].get_state()
    dp = np.argwhere(p0 != p1)
    db = np.argwhere(b0 != b1)
    if len(dp) or len(db):
        print("%s: diverged at iteration %d: %d phys, %d book entries" % (tag, it, len(dp), len(db)))
        for i, c in db[:12]:
            print("   lane %d book col %d (%s): %r vs %r" % (i, c, INV.get(c, "?"), b0[i, c], b1[i, c]))
        for i, c in dp[:6]:
            print("   lane %d phys %d: %r vs %r" % (i, c, p0[i, c], p1[i, c]))
        return True
    return False


def hier(kernel, n=32, iters=40, host=False):
    envs = [HierVecEnv(n, seed=3, kernel=kernel) for _ in range(2)]
    for e in envs:
        e.reset()
    rng = np.random.default_rng(4)
    for it in range(iters):
        ah = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        al = rng.uniform(-1, 1, (n, 17)).astype(np.float32)
        for e in envs:
            e.step(ah, al, autoreset=True)
        if compare("hier kernel %d" % kernel, envs, it):
            return
    print("hier kernel %d: identical over %d iterations" % (kernel, iters))


def low(kernel, n=64, iters=40):
    envs = [HumanoidVecEnv(n, seed=21, kernel=kernel) for _ in range(2)]
    for e in envs:
        e.reset()
    rng = np.random.default_rng(2)
    for it in range(iters):
        a = rng.uniform(-1, 1, (n, 17)).astype(np.float32)
        for e in envs:
            e.step(a, autoreset=True)
        if compare("low kernel %d" % kernel, envs, it):
            return
    print("low kernel %d: identical over %d iterations" % (kernel, iters))


if __name__ == "__main__":
    for k in (1, 0):
        hier(k)
        low(k)
