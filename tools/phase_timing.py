"""Diagnostic: per-phase cycle breakdown of the cooperative kernel (needs libhumenv_diag.so built with
-DHUM_PHASE_TIMING; run with ILRL_AMD_LIB pointing at it).  Also prints the PGS row statistics and the
per-launch wave-duration tail (slowest wave vs mean wave: the launch lasts as long as its slowest wave)."""
import ctypes, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "imitation-learning-rl_amd"))
import torch
from ilrl_amd import _native as N
from ilrl_amd.vec_env import HumanoidVecEnv
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
env = HumanoidVecEnv(n, clips=("motion02_04",), seed=0)
env.reset()
L = N.lib()
buf = (ctypes.c_ulonglong * 32)()
g = torch.Generator(device="cuda").manual_seed(1)
pool = [(torch.rand(n, 17, device="cuda", generator=g) * 2 - 1) for _ in range(8)]
for s in range(10):
    env.step(pool[s % 8], autoreset=True)
L.hum_debug_phase_cycles(buf, 1)
steps = 40
acc = [0] * 32
wmax, wmean = [], []
for s in range(steps):
    env.step(pool[s % 8], autoreset=True)
    L.hum_debug_phase_cycles(buf, 1)
    for k in range(32):
        acc[k] += buf[k]
    wmax.append(buf[16])
    wmean.append(buf[17] / max(buf[18], 1))
names = ["-", "fk", "pass1", "pass2", "base+pass3", "nu*/geom/limits", "contacts", "rows", "pgs", "integrate", "post_step"]
blocks = (n + 3) // 4
tot = sum(acc[k] for k in range(1, 11))
print("per block per env-step (cycles, s_memtime):")
for k in range(1, 11):
    print("  %-18s %10.0f  %5.1f%%" % (names[k], acc[k] / blocks / steps, 100.0 * acc[k] / tot))
print("  total %.0f cycles per block-step" % (tot / blocks / steps))
print("rows: slow-path waves %.2f%%, mean rows/env-substep %.2f, envs > 24 rows %.3f%%, > 30 rows %.3f%%" % (
    100.0 * acc[11] / max(acc[12], 1), acc[13] / max(4 * acc[12], 1), 100.0 * acc[14] / max(4 * acc[12], 1),
    100.0 * acc[15] / max(4 * acc[12], 1)))
r = sorted(a / b for a, b in zip(wmax, wmean))
print("wave duration: mean %.0f cycles, slowest/mean per launch: min %.2f median %.2f max %.2f" % (
    sum(wmean) / steps, r[0], r[len(r) // 2], r[-1]))
