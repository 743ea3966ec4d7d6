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
    big = (torch.arange(off, off + n, dtype=torch.int64) + (1 << 40)).reshape(n, 1).repeat(1, 2)   # > 2**24
    frame = torch.arange(off, off + n, dtype=torch.int32) * 16777217
    f64 = torch.arange(off, off + n, dtype=torch.float64) / 3.0
    g = gather_trajectories([obs, rew, done, draws, big, frame, f64], dst=0)
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
@pytest.mark.parametrize("n_total", [10, 7])   # 7 lanes over 2 ranks: uneven shards (4 + 3)
def test_gloo_world2_gather_and_rng_independent_of_sharding(n_total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_total, q)) for r in range(2)]
    for p in procs:
        p.start()
    obs, rew, done, draws, big, frame, f64 = q.get(timeout=100)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n0 = shard(n_total, 2, 0)[1]
    assert obs.shape == (n_total, 70)
    np.testing.assert_array_equal(obs.reshape(-1), np.arange(n_total * 70, dtype=np.float32))
    np.testing.assert_array_equal(rew, [0] * n0 + [1] * (n_total - n0))
    np.testing.assert_array_equal(done, [1] + [0] * (n0 - 1) + [1] + [0] * (n_total - n0 - 1))
    # lossless for every dtype (the round-1 gather cast through float32)
    assert big.dtype == np.int64 and frame.dtype == np.int32 and f64.dtype == np.float64
    np.testing.assert_array_equal(big[:, 0], np.arange(n_total, dtype=np.int64) + (1 << 40))
    np.testing.assert_array_equal(frame, (np.arange(n_total) * 16777217).astype(np.int32))
    np.testing.assert_array_equal(f64, np.arange(n_total, dtype=np.float64) / 3.0)
    single = np.array([[O.lane_draw(5, i, c, 0, 293) for c in range(3)] for i in range(n_total)], dtype=np.float32)
    np.testing.assert_array_equal(draws, single)


def _tg_worker(rank, world, port, n_total, q):
    """TrajectoryGather (the benchmark's repeated gather): static counts, packed lane-major fragments, two slots,
    launches of k = 4 steps into fragments of G = 8 steps, and a final partial fragment (3 steps)."""
    from ilrl_amd.parallel import TrajectoryGather
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    off, n = shard(n_total, world, rank)
    counts = [shard(n_total, world, r)[1] for r in range(world)]
    G, k = 8, 4
    fields = [("obs", (70,), torch.float32), ("act", (17,), torch.float32), ("reward", (), torch.float32),
              ("done", (), torch.uint8), ("frame", (), torch.int64)]
    tg = TrajectoryGather(fields, counts, G, "cpu")
    got = []
    sizes = [k, k, k, k, 3]   # 19 steps: fragments [0, 8), [8, 16), [16, 19)

    def rows(t0, kk):   # time-major [kk, n, ...] values that name (global lane, step)
        t = torch.arange(t0, t0 + kk, dtype=torch.float64).reshape(kk, 1)
        lane = torch.arange(off, off + n, dtype=torch.float64).reshape(1, n)
        v = lane * 1000 + t
        return {"obs": (v.unsqueeze(-1) + torch.arange(70, dtype=torch.float64) / 100).float(),
                "act": (v.unsqueeze(-1) - torch.arange(17, dtype=torch.float64)).float(),
                "reward": v.float(), "done": ((lane + t) % 2 == 0).to(torch.uint8), "frame": (v * (1 << 33)).long()}
    t = 0
    for s, kk in enumerate(sizes):
        slot = (t // G) % 2
        tg.pack(slot, t % G, rows(t, kk))
        final = (t + kk) % G == 0 or s == len(sizes) - 1
        tg.commit(slot, t % G, t % G + kk, final)   # bench.py's per-launch call: the fragment goes on the final one
        t += kk
        if final:
            tg.wait(slot)
            r = tg.result(slot)
            if r is not None:
                got.append({f: x.clone().numpy() for f, x in r.items()})
    if rank == 0:
        q.put(got)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("n_total", [10, 7])
def test_gloo_world2_trajectory_gather_fragments(n_total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tg_worker, args=(r, 2, port, n_total, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=100)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert len(got) == 3
    lane = np.arange(n_total, dtype=np.float64).reshape(-1, 1)
    for j, nsteps in enumerate((8, 8, 3)):
        f = got[j]
        assert f["obs"].shape == (n_total, 8, 70) and f["done"].dtype == np.uint8 and f["frame"].dtype == np.int64
        t = np.arange(8 * j, 8 * j + nsteps, dtype=np.float64).reshape(1, -1)
        v = lane * 1000 + t
        np.testing.assert_array_equal(f["reward"][:, :nsteps], v.astype(np.float32))
        np.testing.assert_array_equal(f["obs"][:, :nsteps], (v[..., None] + np.arange(70) / 100).astype(np.float32))
        np.testing.assert_array_equal(f["act"][:, :nsteps], (v[..., None] - np.arange(17)).astype(np.float32))
        np.testing.assert_array_equal(f["done"][:, :nsteps], ((lane + t) % 2 == 0).astype(np.uint8))
        np.testing.assert_array_equal(f["frame"][:, :nsteps], (v * (1 << 33)).astype(np.int64))


def test_trajectory_gather_pack_bounds_host():
    """TrajectoryGather.pack refuses a launch that crosses the fragment (host path; the device path is
    tests/test_gpu_traj_pack.py): 0 <= t0, t0 + k <= G, one step count for every field."""
    import torch
    from ilrl_amd.parallel import TrajectoryGather
    n, G = 4, 8
    tg = TrajectoryGather([("obs", (3,), torch.float32), ("done", (), torch.uint8)], [n], G, "cpu")
    mk = lambda k: {"obs": torch.ones(k, n, 3), "done": torch.ones(k, n, dtype=torch.uint8)}
    for t0, k in ((4, 5), (8, 1), (-1, 2)):
        with pytest.raises(ValueError):
            tg.pack(0, t0, mk(k))
    with pytest.raises(ValueError):
        tg.pack(0, 0, {"obs": torch.ones(2, n, 3), "done": torch.ones(3, n, dtype=torch.uint8)})
    assert int(tg.send[0].abs().sum()) == 0
    tg.pack(0, 4, mk(4))
    assert int(tg.send[0].sum()) > 0
