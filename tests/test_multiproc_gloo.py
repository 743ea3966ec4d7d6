"""world_size-2 gloo tests (CPU) for the N>1 layout: lane sharding by global id and the trajectory gather."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle as O
from ilrl_amd.parallel import gather_trajectories, shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_total, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    off, n = shard(n_total, world, rank)
    # per-lane reset draws depend only on the GLOBAL lane id (same as hum_config.lane_offset + i)
    draws = torch.tensor([[O.lane_draw(5, off + i, c, 0, 293) for c in range(3)] for i in range(n)], dtype=torch.float32)
    obs = torch.arange(off * 70, (off + n) * 70, dtype=torch.float32).reshape(n, 70)
    rew = torch.full((n,), float(rank))
    done = torch.zeros(n, dtype=torch.uint8)
    done[0] = 1
    g = gather_trajectories([obs, rew, done, draws], dst=0)
    if rank == 0:
        q.put([t.numpy() for t in g])
    dist.barrier()
    dist.destroy_process_group()


def test_shard_covers_all_lanes():
    for total in (1, 7, 4096, 32768):
        for world in (1, 2, 3, 8):
            spans = [shard(total, world, r) for r in range(world)]
            assert spans[0][0] == 0
            assert sum(n for _, n in spans) == total
            for (o1, n1), (o2, _) in zip(spans, spans[1:]):
                assert o1 + n1 == o2


@pytest.mark.timeout(120)
def test_gloo_world2_gather_and_rng_independent_of_sharding():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    n_total = 10
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_total, q)) for r in range(2)]
    for p in procs:
        p.start()
    obs, rew, done, draws = q.get(timeout=100)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert obs.shape == (n_total, 70)
    np.testing.assert_array_equal(obs.reshape(-1), np.arange(n_total * 70, dtype=np.float32))
    np.testing.assert_array_equal(rew, [0] * 5 + [1] * 5)
    np.testing.assert_array_equal(done, [1, 0, 0, 0, 0, 1, 0, 0, 0, 0])
    single = np.array([[O.lane_draw(5, i, c, 0, 293) for c in range(3)] for i in range(n_total)], dtype=np.float32)
    np.testing.assert_array_equal(draws, single)
