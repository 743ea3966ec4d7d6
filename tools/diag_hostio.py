#!/usr/bin/env python3
"""Diagnostic: hier handle stepped through HUM_STEP_HOST_IO vs one stepped through device buffers (and a control
pair: device vs device with a sync after every step); prints the first diverging iteration / lane / column."""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "imitation-learning-rl_amd"))
from ilrl_amd import _native as N  # noqa: E402
from ilrl_amd.hier_env import HierVecEnv  # noqa: E402

INV = {v: k for k, v in N.BK.items()}
P = lambda x: ctypes.c_void_p(x.ctypes.data) if x is not None else None


def run(mode, rep, n=32, iters=12):
    envs = [HierVecEnv(n, seed=3) for _ in range(2)]
    for e in envs:
        e.reset()
    rng = np.random.default_rng(4)
    for it in range(iters):
        ah = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        al = rng.uniform(-1, 1, (n, 17)).astype(np.float32)
        envs[0].step(ah, al, autoreset=True)
        if mode == "host":
            o = [np.zeros(s, d) for s, d in ((n, np.uint8), ((n, 44), np.float32), ((n, 70), np.float32),
                                             (n, np.float32), (n, np.float32), (n, np.uint8), (n, np.int32))]
            rc = N.lib().hum_hier_step(envs[1].h, P(ah), P(al), None, *[P(x) for x in o],
                                       N.HUM_STEP_AUTORESET | N.HUM_STEP_HOST_IO, None, None)
            assert rc == 0
        else:
            torch.cuda.synchronize()
            envs[1].step(ah, al, autoreset=True)
            torch.cuda.synchronize()
        p0, b0 = envs[0].get_state()
        p1, b1 = envs[1].get_state()
        dp, db = np.argwhere(p0 != p1), np.argwhere(b0 != b1)
        if len(dp) or len(db):
            print("%s rep %d: diverged at iteration %d (%d phys, %d book)" % (mode, rep, it, len(dp), len(db)))
            for i, c in db[:8]:
                print("   lane %d book %s: %r vs %r (expect_high %d, frame %d)" % (
                    i, INV.get(c, c), b0[i, c], b1[i, c], b0[i, N.BK["expect_high"]], b0[i, N.BK["frame"]]))
            for i, c in dp[:4]:
                print("   lane %d phys %d: %r vs %r" % (i, c, p0[i, c], p1[i, c]))
            return False
    print("%s rep %d: identical" % (mode, rep))
    return True


if __name__ == "__main__":
    for rep in range(4):
        run("host", rep)
        run("devsync", rep)
