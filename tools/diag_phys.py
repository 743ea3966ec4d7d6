import os, sys
import numpy as np
REPO = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
for p in ("imitation-learning-rl_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(REPO, p))
import torch
from golden_replay import rec
import test_gpu_hier as TH
import test_gpu_parity as TP
np.set_printoptions(precision=4, suppress=True, linewidth=200)
g = np.load(os.path.join(REPO, "tests/golden/golden_hier.npz"))
r = rec(g, "hier_l0")
for prec in ("fp64", "fp32"):
    for kern in (1, 0):
        o = TH.run_scenario(r, prec, skip_physics=False, kernel=kern)
        e = np.abs(o["phys"] - r["state_post"])
        print(prec, "kernel", kern, "max err", e.max(), "per-row max", e.max(1)[:12])
gl = np.load(os.path.join(REPO, "tests/golden/golden_low.npz"))
rl = rec(gl, "motion02_04_l0")
for kern in (1, 0):
    o = TP.run_scenario(rl, "fp64", skip_physics=False, kernel=kern)
    e = np.abs(o["phys"] - rl["state_post"])
    print("low fp64 kernel", kern, "max err", e.max(), e.max(1)[:10])
