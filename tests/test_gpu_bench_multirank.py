"""Config 4's real benchmark path (BASELINE.json configs[3]: lanes sharded over ranks, trajectory gather to the
learner rank) end to end on the one-GPU box: bench.py under torch.distributed.run (every rank on cuda:0, gloo -
RCCL needs one GPU per rank; the 8-GPU RCCL/xGMI run is the driver's).  Three runs: 2 ranks x 2048 lanes, 8 env
steps per launch, a gather every 8 env steps; and config 4's own shape, 8 ranks x 4096 lanes = 32,768 lanes, 32 env
steps per launch (the bench default) and a gather every 32 env steps; and the RCCL ("nccl") path itself - RCCL
refuses two ranks on one device ("Duplicate GPU detected", profiles/r04_rccl_probe.txt), so one rank with
--force-dist runs the process group, barriers, the device-tensor timing all-reduce and the all_gather_into_tensor
gather through RCCL.  Rank 0's gathered obs / action / reward /
done fragments must equal those of ONE handle over all the lanes stepped with the same actions, bit for bit (every
lane's RNG stream is keyed by its global id); at 32,768 lanes rank 0 keeps every 61st lane of the
fragment (all eight shards are sampled) to bound host memory."""
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


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(600)
@pytest.mark.parametrize("ranks,lanes,k,every,steps,stride,backend,transport",
                         [(2, 2048, 8, 8, 16, 1, "gloo", "collective"), (8, 4096, 32, 32, 32, 61, "gloo", "collective"),
                          (1, 4096, 32, 32, 64, 7, "nccl", "collective"), (2, 2048, 8, 8, 32, 1, "gloo", "dma"),
                          (8, 4096, 32, 32, 64, 61, "gloo", "dma"), (1, 4096, 32, 32, 64, 7, "nccl", "dma"),
                          (2, 2048, 8, 8, 16, 1, "gloo", "dma_fallback"), (2, 2048, 8, 16, 32, 1, "gloo", "dma")],
                         ids=["2x2048", "config4_8x4096", "rccl_1x4096", "dma_2x2048", "dma_config4_8x4096",
                              "dma_rccl_1x4096", "dma_fallback_2x2048", "dma_2x2048_two_launches_per_fragment"])
def test_bench_ranks_gather_equals_single_handle(tmp_path, ranks, lanes, k, every, steps, stride, backend, transport):
    """transport "dma": the default for N > 1 - IPC-mapped send buffers pulled by rank 0 with the SDMA copy engines
    (parallel.DmaGather; on one GPU the copies are intra-device, between GPUs they cross xGMI)."""
    import types
    sys.path.insert(0, REPO)
    import bench
    dump = str(tmp_path / "gather.npz")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(ranks),
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", str(ranks),
           "--backend", backend, "--lanes", str(lanes), "--steps", str(steps), "--warmup", "0", "--k", str(k),
           "--gather-every", str(every), "--dump-gather", dump, "--dump-lane-stride", str(stride), "--cpu-seconds", "0",
           "--transport", transport]
    if ranks == 1:   # RCCL refuses two ranks on one device: one rank with every collective run through it
        cmd += ["--force-dist", "--no-secondary"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2")
    if transport == "dma_fallback":   # the copy engines refused on one rank: every rank takes the collective path
        env["ILRL_AMD_DMA_PROBE_FAIL"] = "1"
        cmd[cmd.index("--transport") + 1] = "dma"
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=560, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    print("bench line:", json.dumps({x: line[x] for x in ("value", "ms_per_step", "n_gpus", "gather")}))
    # the DMA transport moves every launch's rows while the next launch runs and ends on a short drain launch (the
    # last launch's final fifth, same action rows: bench.launch_plan); the collective transport runs whole launches
    plan = bench.launch_plan(steps, k, drain=transport == "dma")
    assert line["n_gpus"] == ranks and line["config"]["steps_per_launch"] == k
    assert line["config"]["launch_sizes"] == sorted({kk for _, _, kk in plan}, reverse=True)
    assert line["config"]["launches"] == len(plan)
    assert line["gather"]["every"] == every and line["gather"]["fragments"] == steps // every
    if transport == "dma_fallback":
        assert line["gather"]["transport"].startswith("collective (dma unavailable"), line["gather"]["transport"]
    else:
        assert line["gather"]["backend"] == backend and line["gather"]["transport"] == transport
    assert line["value"] > 0 and line["error_flags"] == 0 and 0 < line["ms_per_step"] < 1e3   # a sane clock
    g = np.load(dump)
    total = ranks * lanes
    sel = np.arange(0, total, stride)
    assert len(np.unique(sel // lanes)) == ranks   # every shard sampled
    # the bench's own device-resident action blocks of every rank (bench._pools, seeded by rank), lanes in rank order
    dev = torch.device("cuda", 0)
    pools = [bench._pools(types.SimpleNamespace(hier=False), dev, lanes, k, rr)[0] for rr in range(ranks)]
    one = HumanoidVecEnv(total, clips=("motion02_04",), seed=0)
    one.reset()
    for j in range(steps // every):
        acts = g["act_%d" % j]   # [sampled lanes, every, 17] lane-major, rank 0's lanes first
        assert acts.shape == (len(sel), every, 17)
        for s in range(every // k):
            blk = torch.cat([p[(j * (every // k) + s) % 16] for p in pools], dim=1).contiguous()   # [k, total, 17]
            np.testing.assert_array_equal(blk[:, sel].transpose(0, 1).cpu().numpy(), acts[:, s * k:(s + 1) * k])
            obs, rew, done, _, _ = one.step_k(blk, autoreset=True)
            sl = slice(s * k, (s + 1) * k)
            np.testing.assert_array_equal(obs[:, sel].transpose(0, 1).cpu().numpy(), g["obs_%d" % j][:, sl])
            np.testing.assert_array_equal(rew[:, sel].transpose(0, 1).cpu().numpy(), g["reward_%d" % j][:, sl])
            np.testing.assert_array_equal(done[:, sel].transpose(0, 1).cpu().numpy(), g["done_%d" % j][:, sl])
    one.close()
