#!/usr/bin/env python3
"""Diagnostic: the config-2 fp32 rollout of tests/test_gpu_scale.py (4096 lanes, 200 random-action steps, seed 21),
then one step of the fp64 kernel from its state; saves the states, actions and fp64-kernel results of the given
lanes (default: the sample lanes whose fp64-kernel step differed most from the oracle) to gpurun_out/fp64_lanes.npz
for a CPU comparison with the oracle (tools/diag_fp64_lanes_cpu.py)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "imitation-learning-rl_amd"))
from ilrl_amd.vec_env import HumanoidVecEnv  # noqa: E402

lanes = [int(x) for x in sys.argv[1:]] or [3510, 1430, 4095]
n = 4096
env = HumanoidVecEnv(n, clips=("motion02_04",), seed=21, precision="fp32")
env.reset()
g = torch.Generator(device="cuda").manual_seed(4)
for _ in range(200):
    env.step(torch.rand(n, 17, device="cuda", generator=g) * 2 - 1, autoreset=True)
phys, book = env.get_state()
env.close()
a = np.random.default_rng(5).uniform(-1, 1, (n, 17)).astype(np.float32)
out = {"lanes": np.array(lanes), "phys": phys[lanes], "book": book[lanes], "act": a[lanes]}
for k in (1, 0):
    e = HumanoidVecEnv(n, clips=("motion02_04",), seed=21, precision="fp64", kernel=k)
    e.set_state(phys, book)
    e.step(torch.as_tensor(a, device="cuda"))
    p64, _ = e.get_state()
    e.close()
    out["phys64_k%d" % k] = p64[lanes]
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(REPO, "gpurun_out", "fp64_lanes.npz"), **out)
print("saved", lanes)
