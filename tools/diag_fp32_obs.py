"""Diagnostic (GPU): per-component obs error of the fp32 kernel with injected physics vs the golden fixtures."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("imitation-learning-rl_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(REPO, p))
import numpy as np  # noqa: E402

from conftest import scenarios  # noqa: E402
from golden_replay import rec  # noqa: E402
from test_gpu_parity import run_scenario  # noqa: E402

g = np.load(os.path.join(REPO, "tests", "golden", "golden_low.npz"))
comp = np.zeros(70)
worst = []
for name in scenarios(g):
    r = rec(g, name)
    for kernel in (1, 0):
        o = run_scenario(r, "fp32", skip_physics=True, kernel=kernel)
        d = np.abs(o["obs"] - r["obs"])
        comp = np.maximum(comp, d.max(axis=0))
        t, k = np.unravel_index(d.argmax(), d.shape)
        worst.append((float(d.max()), name, kernel, int(t), int(k), float(o["obs"][t, k]), float(r["obs"][t, k])))
print("per-component max:", " ".join("%d:%.1e" % (k, v) for k, v in enumerate(comp) if v > 1e-6))
for w in sorted(worst, reverse=True)[:10]:
    print(w)
