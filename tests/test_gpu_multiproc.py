"""Config 4's code path on one GPU: two ranks (gloo, both on cuda:0 - the pool gives us one GPU; the 8-GPU
RCCL run is the driver's) each step their lane shard with hum_config.lane_offset and gather the trajectories;
the gathered obs / reward / done / frame equal those of ONE handle holding all lanes (lane streams are keyed
by the global lane id), bit for bit."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("needs a HIP device", allow_module_level=True)

import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

N_TOTAL, STEPS, EVERY = 1000, 24, 8   # uneven is fine too, but keep the shards equal here: 500 + 500


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _actions(t):
    g = torch.Generator().manual_seed(100 + t)
    return torch.rand(N_TOTAL, 17, generator=g) * 2 - 1


def _rank(rank, world, port, q):
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(repo, "imitation-learning-rl_amd"))
    from ilrl_amd.parallel import gather_trajectories, shard
    from ilrl_amd.vec_env import HumanoidVecEnv
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    off, n = shard(N_TOTAL, world, rank)
    env = HumanoidVecEnv(n, clips=("motion02_04",), seed=17, lane_offset=off)
    env.reset()
    got = []
    for t in range(STEPS):
        a = _actions(t)[off:off + n].cuda()
        obs, rew, done, frame = env.step(a, autoreset=True)
        if (t + 1) % EVERY == 0:
            g = gather_trajectories([obs, rew, done, frame], dst=0)
            if rank == 0:
                got.append([x.cpu().numpy() for x in g])
    env.close()
    if rank == 0:
        q.put(got)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_two_rank_shards_gather_equals_single_handle():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=200)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from ilrl_amd.vec_env import HumanoidVecEnv
    env = HumanoidVecEnv(N_TOTAL, clips=("motion02_04",), seed=17)
    env.reset()
    k = 0
    for t in range(STEPS):
        obs, rew, done, frame = env.step(_actions(t).cuda(), autoreset=True)
        if (t + 1) % EVERY == 0:
            for x, y in zip((obs, rew, done, frame), got[k]):
                np.testing.assert_array_equal(x.cpu().numpy(), y)
            k += 1
    env.close()
    assert k == STEPS // EVERY
