"""GPU diagnostics: per-element diffs of one golden scenario (kernel vs reference/oracle)."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("imitation-learning-rl_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(REPO, p))
import torch
import oracle as O
from golden_replay import rec
from test_gpu_parity import run_scenario, book_rows
from ilrl_amd import _native as N
np.set_printoptions(precision=5, suppress=True, linewidth=200)
g = np.load(os.path.join(REPO, "tests/golden/golden_low.npz"))
name = sys.argv[1] if len(sys.argv) > 1 else "motion08_03_l0"
r = rec(g, name)
for prec, skip in (("fp64", True), ("fp64", False), ("fp32", False)):
    o = run_scenario(r, prec, skip)
    d = np.abs(o["obs"] - r["obs"])
    print("== %s skip=%s  obs maxerr per element (first 3 steps):" % (prec, skip))
    for t in range(min(3, len(d))):
        bad = np.where(d[t] > 1e-5)[0]
        print("  t=%d bad idx %s" % (t, bad[:20]))
        if len(bad):
            print("    gpu", o["obs"][t][bad[:12]]); print("    ref", r["obs"][t][bad[:12]])
    print("  reward gpu", o["rew"][:5], "ref", r["reward"][:5])
    print("  done gpu", o["done"][:10].astype(int), "ref", r["done"][:10].astype(int))
    if not skip:
        e = np.abs(o["phys"] - r["state_post"])
        print("  state err max per component:", e.max(0))
    print("  book robot_pos gpu", o["book"][:3, 10:13], "ref", r["book_robot_pos"][:3])
