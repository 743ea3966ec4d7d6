"""Diagnostic (GPU): bench.py's parity sample over EVERY lane.  Runs the benchmark rollout (4096 lanes,
motion02_04, fp32, the bench's action pool, warm-up + timed steps), then steps once more from the reached
state on the fp32 handle and on an fp64 handle given the identical state, and compares each lane with the fp64
oracle.  Saves the worst lanes (state, book, action, outputs) to gpurun_out/diag_parity.npz for CPU analysis."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("imitation-learning-rl_amd", "oracle"):
    sys.path.insert(0, os.path.join(REPO, p))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as O  # noqa: E402
from ilrl_amd import _native as N  # noqa: E402
from ilrl_amd.clips import load_clip  # noqa: E402
from ilrl_amd.vec_env import HumanoidVecEnv  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1100
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(1234)
pool = [(torch.rand(n, 17, device=dev, generator=g) * 2 - 1).contiguous() for _ in range(16)]
env = HumanoidVecEnv(n, clips=("motion02_04",), seed=0, device=0, precision="fp32")
env.reset()
env.done.zero_()
for s in range(100):
    env.step(pool[s % 16], autoreset=True)
for s in range(steps - 100):
    env.step(pool[s % 16], autoreset=True)
phys, book = env.get_state()
a = np.random.default_rng(5).uniform(-1, 1, (n, 17)).astype(np.float32)
o32, r32, d32, _ = [x.cpu().numpy() for x in env.step(torch.as_tensor(a, device=dev))]
p32, _ = env.get_state()
env64 = HumanoidVecEnv(n, clips=("motion02_04",), seed=0, device=0, precision="fp64")
env64.set_state(phys, book)
o64, r64, d64, _ = [x.cpu().numpy() for x in env64.step(torch.as_tensor(a, device=dev))]
p64, _ = env64.get_state()
clip = load_clip("motion02_04")
eo32, eo64, er32, es32, nco = [], [], [], [], []
for i in range(n):
    o = O.OracleLowLevelEnv.from_lane(clip, phys[i], book[i], N.BK)
    nco.append(len(O.contacts(phys[i])))
    ro, rr, rd, _ = o.step(a[i])
    eo32.append(float(np.abs(o32[i] - ro).max()))
    eo64.append(float(np.abs(o64[i] - ro).max()))
    er32.append(abs(float(r32[i]) - rr))
    es32.append(float(np.abs(p32[i] - o.state).max()))
eo32, eo64, er32, es32, nco = map(np.array, (eo32, eo64, er32, es32, nco))
print("fp32 obs err: p50 %.3g p99 %.3g p99.9 %.3g max %.3g; lanes > 2.5e-4: %d" % (
    np.median(eo32), np.percentile(eo32, 99), np.percentile(eo32, 99.9), eo32.max(), int((eo32 > 2.5e-4).sum())))
print("fp64 obs err: max %.3g   fp32 reward err max %.3g  fp32 state err p50 %.3g max %.3g" % (
    eo64.max(), er32.max(), np.median(es32), es32.max()))
for lo, hi in ((0, 1), (1, 5), (5, 10), (10, 20), (20, 100)):
    m = (nco >= lo) & (nco < hi)
    if m.any():
        print("contacts [%d,%d): lanes %d  fp32 obs err p50 %.3g max %.3g" % (lo, hi, int(m.sum()),
                                                                          np.median(eo32[m]), eo32[m].max()))
worst = np.argsort(-eo32)[:32]
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(REPO, "gpurun_out", "diag_parity.npz"), lanes=worst, phys=phys[worst], book=book[worst],
         action=a[worst], o32=o32[worst], o64=o64[worst], p32=p32[worst], p64=p64[worst], eo32=eo32[worst],
         ncontacts=nco[worst])
print("worst lanes:", [(int(i), round(float(eo32[i]), 5), int(nco[i])) for i in worst[:10]])
