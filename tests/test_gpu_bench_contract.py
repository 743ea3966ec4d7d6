"""bench.py's output contract (the driver parses it): one JSON line on stdout with the metric / value / unit /
timing keys, `roofline` for the dominant kernel (achieved / peak = frac, measured from this run's HIP events) and
`cpu_baseline` (the oracle port timed on the host, N = 1) - checked on a short run of the default workload."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("needs a HIP device", allow_module_level=True)

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(300)
def test_bench_line_carries_the_contract_keys():
    r = subprocess.run([sys.executable, "bench.py", "--steps", "40", "--warmup", "8", "--cpu-seconds", "1",
                        "--cpu-workers", "2", "--no-secondary"], cwd=REPO, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 40 and d["warmup"] == 8 and d["higher_is_better"] is True
    assert d["unit"] == "env-steps/s" and d["dtype"] == "f32" and d["scaling"] == "weak" and d["vs_baseline"] is None
    assert "workload" in d["config"] and d["config"]["envs_per_gpu"] == 4096
    # value = every lane's env steps over the timed wall time
    assert abs(d["value"] - 4096 * 40 / (d["ms_per_step"] * 40 * 1e-3)) < 1e-6 * d["value"]
    rf = d["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-12
    # achieved = the algorithmic bytes of an env step of every lane over the kernel's own time per env step
    assert abs(rf["achieved"] - 4096 * rf["bytes_per_env_step"] / (rf["kernel_ms"] * 1e-3) / 1e9) < 1e-6 * rf["achieved"]
    assert 0 < rf["kernel_ms"] <= d["ms_per_step"] * 1.001
    cb = d["cpu_baseline"]
    assert cb["value"] > 0 and cb["unit"] == "env-steps/s" and cb["cores"] == 2 and cb["kind"] in ("port", "reference")
    assert cb["sample"]
    assert d["error_flags"] == 0
