"""Config 4's real benchmark path (BASELINE.json configs[3]: lanes sharded over ranks, trajectory gather to the
learner rank) end to end on the one-GPU box: bench.py under torch.distributed.run with 2 ranks (both on cuda:0,
gloo - RCCL needs one GPU per rank; the 8-GPU RCCL/xGMI run is the driver's), 2048 lanes per rank, 8 env
steps per launch and a gather every 8 env steps.  Rank 0's gathered obs / action / reward / done fragments must
equal those of ONE 4096-lane handle stepped with the same actions, bit for bit (every lane's RNG stream is keyed by
its global id)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("needs a HIP device", allow_module_level=True)

from ilrl_amd.vec_env import HumanoidVecEnv  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LANES, K, EVERY, STEPS = 2048, 8, 8, 16


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(300)
def test_bench_two_ranks_gather_equals_single_handle(tmp_path):
    dump = str(tmp_path / "gather.npz")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2",
           "--backend", "gloo", "--lanes", str(LANES), "--steps", str(STEPS), "--warmup", "0", "--k", str(K),
           "--gather-every", str(EVERY), "--dump-gather", dump, "--cpu-seconds", "0"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=280, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["config"]["steps_per_launch"] == K
    assert line["gather"]["every"] == EVERY and line["gather"]["fragments"] == STEPS // EVERY
    assert line["value"] > 0 and line["error_flags"] == 0
    g = np.load(dump)
    one = HumanoidVecEnv(2 * LANES, clips=("motion02_04",), seed=0)
    one.reset()
    for j in range(STEPS // EVERY):
        acts = g["act_%d" % j]   # [lanes, EVERY, 17] lane-major, rank 0's lanes first
        assert acts.shape == (2 * LANES, EVERY, 17)
        for t in range(EVERY):
            obs, rew, done, _ = one.step(torch.as_tensor(np.ascontiguousarray(acts[:, t]), device="cuda"),
                                         autoreset=True)
            np.testing.assert_array_equal(obs.cpu().numpy(), g["obs_%d" % j][:, t])
            np.testing.assert_array_equal(rew.cpu().numpy(), g["reward_%d" % j][:, t])
            np.testing.assert_array_equal(done.cpu().numpy(), g["done_%d" % j][:, t])
    one.close()
