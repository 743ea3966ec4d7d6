"""Diagnostic (GPU): worst obs components of the fp32 kernel with injected physics vs the golden fixtures."""
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
for name in scenarios(g):
    r = rec(g, name)
    for kernel in (1, 0):
        o = run_scenario(r, "fp32", skip_physics=True, kernel=kernel)
        err = np.abs(o["obs"] - r["obs"])
        excess = err - (1e-6 + 2.0 ** -22 * np.abs(r["obs"]))
        t, k = np.unravel_index(excess.argmax(), excess.shape)
        print("%-20s k%d max excess %.3g at step %d comp %d: got %.9g want %.9g  base xyz %s" % (
            name, kernel, excess.max(), t, k, o["obs"][t, k], r["obs"][t, k], np.round(r["state_pre"][t][:3], 3)))
