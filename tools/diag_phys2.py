"""Diagnostic: fp32 cooperative-kernel physics error vs the golden state (works with the fast/variant libs)."""
import os, sys
import numpy as np
REPO = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
for p in ("imitation-learning-rl_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(REPO, p))
import torch
from golden_replay import rec
import test_gpu_parity as TP
g = np.load(os.path.join(REPO, "tests/golden/golden_low.npz"))
errs = []
for name in ["motion02_04_l0", "motion08_03_l0", "motion09_03_l1", "teleport_target"]:
    r = rec(g, name)
    o = TP.run_scenario(r, "fp32", skip_physics=False, kernel=1)
    errs.append(np.abs(o["phys"] - r["state_post"]).max())
print(os.environ.get("ILRL_AMD_LIB", "default"), "max errs", ["%.2e" % e for e in errs])
