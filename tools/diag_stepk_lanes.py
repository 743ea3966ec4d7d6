#!/usr/bin/env python3
"""Diagnostic: hum_step_k (k = 2) vs two hum_step launches with the same actions, for a kernel variant (argv[1]:
0 = per-lane, 1 = cooperative) and precision (argv[2]); prints the lanes / obs columns / bookkeeping columns that
differ after each step, and whether those lanes were done (auto-reset) at step 0."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "imitation-learning-rl_amd"))
from ilrl_amd import _native as N  # noqa: E402
from ilrl_amd.vec_env import HumanoidVecEnv  # noqa: E402

kernel = int(sys.argv[1]) if len(sys.argv) > 1 else 0
prec = sys.argv[2] if len(sys.argv) > 2 else "fp32"
n, k = 256, 3
INV = {v: kk for kk, v in N.BK.items()}
envs = [HumanoidVecEnv(n, clips=("motion02_04",), seed=11, precision=prec, kernel=kernel) for _ in range(2)]
for e in envs:
    e.reset()
g = torch.Generator(device="cuda").manual_seed(3)
acts = (torch.rand(k, n, 17, device="cuda", generator=g) * 2 - 1).contiguous()
single, states = [], []
for t in range(k):
    o, r, d, f = envs[0].step(acts[t], autoreset=True)
    single.append([x.clone().cpu().numpy() for x in (o, r, d, f)])
    states.append(envs[0].get_state())
out = [x.cpu().numpy() for x in envs[1].step_k(acts, autoreset=True)]
p1, b1 = envs[1].get_state()
for t in range(k):
    o, r, d, f = single[t]
    bad = np.nonzero((out[0][t] != o).any(1) | (out[1][t] != r) | (out[2][t] != d))[0]
    print("step %d: %d lanes differ %s" % (t, len(bad), bad[:12]))
    for i in bad[:3]:
        cols = np.nonzero(out[0][t][i] != o[i])[0]
        print("   lane %d obs cols %s  done0 %s  max |d| %.3g" % (i, cols[:20], single[0][2][i], np.abs(out[0][t][i] - o[i]).max()))
p0, b0 = states[-1]
dp = np.nonzero((p0 != p1).any(1))[0]
db = np.nonzero((b0 != b1).any(1))[0]
print("final state: %d lanes differ (phys), %d (book)" % (len(dp), len(db)))
for i in db[:3]:
    cols = np.nonzero(b0[i] != b1[i])[0]
    print("   lane %d book cols %s" % (i, [INV.get(c, c) for c in cols]))
for i in dp[:3]:
    print("   lane %d phys cols %s" % (i, np.nonzero(p0[i] != p1[i])[0]))
