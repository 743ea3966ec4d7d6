"""Diagnostic: step time vs solver iterations (the PGS share of the kernel, measured in place)."""
import os, sys, json
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "imitation-learning-rl_amd"))
import torch
from ilrl_amd.vec_env import HumanoidVecEnv
n = 4096
res = {}
for it in (5, 10, 20):
    env = HumanoidVecEnv(n, clips=("motion02_04",), seed=0, solver_iters=it)
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(1)
    pool = [(torch.rand(n, 17, device="cuda", generator=g) * 2 - 1) for _ in range(8)]
    for s in range(20):
        env.step(pool[s % 8], autoreset=True)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s0 = torch.cuda.current_stream()
    e0.record(s0)
    for s in range(100):
        env.step(pool[s % 8], autoreset=True)
    e1.record(s0)
    torch.cuda.synchronize()
    res[it] = e0.elapsed_time(e1) / 100
    env.close()
print(json.dumps({"lib": os.path.basename(os.environ.get("ILRL_AMD_LIB", "libhumenv.so")), "ms_per_step": res,
                  "ms_per_extra_iter": (res[20] - res[5]) / 15}))
