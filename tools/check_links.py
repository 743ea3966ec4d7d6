"""Diagnostic: the wave_log.py workload (4096 envs, motion02_04, seed 0, uniform random actions, auto-reset)
on any library; with a -DHUM_CHECK_LINKS build also prints the PGS link / index check counters."""
import ctypes, os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "imitation-learning-rl_amd"))
import torch
from ilrl_amd import _native as N
from ilrl_amd.vec_env import HumanoidVecEnv
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
env = HumanoidVecEnv(n, clips=("motion02_04",), seed=0)
env.reset()
L = N.lib()
chk = hasattr(L, "hum_debug_check")
buf = (ctypes.c_uint * 8)()
g = torch.Generator(device="cuda").manual_seed(1)
pool = [(torch.rand(n, 17, device="cuda", generator=g) * 2 - 1) for _ in range(8)]
for s in range(steps):
    env.step(pool[s % 8], autoreset=True)
    if chk and s % 10 == 9:
        L.hum_debug_check(buf, 0)
        print("step %d: bad next2 %d, bad next2_ln %d, bad pool %d, env-substeps %d, bad surv %d, bad rdesc %d"
              % (s, buf[0], buf[1], buf[2], buf[3], buf[4], buf[5]), flush=True)
torch.cuda.synchronize()
ef = ctypes.c_uint32(0)
N.lib().hum_get_error_flags(env.h, ctypes.byref(ef))
print("ok: %d steps, eflags %s" % (steps, hex(ef.value)))
