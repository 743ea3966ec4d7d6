"""Multi-GPU layout: one process per GPU, env lanes sharded by rank.

* Rank r owns global lanes [off_r, off_r + n_r) (`shard`); each lane's RNG stream is keyed by its GLOBAL id
  (hum_config.lane_offset), so results are independent of how many GPUs share the job.
* Env stepping needs no collective (weak scaling).  The only exchange is the trajectory gather to the
  learner rank (obs / action / reward / done per step or per rollout fragment), done with ONE collective per
  call over torch.distributed ("nccl" = RCCL over xGMI on MI355X, "gloo" on CPU).  The buffers travel as their
  raw bytes (lossless for every dtype), and uneven shards are padded to the largest one and trimmed on arrival.
"""
import torch
import torch.distributed as dist


def shard(n_total, world, rank):
    """(lane_offset, n_local) of `rank` for n_total lanes split over `world` ranks (contiguous shards)."""
    base, rem = divmod(n_total, world)
    n = base + (1 if rank < rem else 0)
    off = rank * base + min(rank, rem)
    return off, n


def _row_bytes(t):
    return t[0].numel() * t.element_size() if t.dim() > 1 else t.element_size()


def gather_trajectories(tensors, dst=0):
    """Gather per-rank trajectory buffers (same trailing shape and dtype on every rank; leading dim = that
    rank's lanes, may differ between ranks) onto `dst` as one [sum n_r, ...] tensor each, in rank order.

    All buffers are packed, row by row, into ONE uint8 message (their raw bytes: int64 / uint8 / float keep
    their exact values), so RCCL moves one large payload per call: xGMI is point-to-point, so few large
    collectives beat many small ones.  Returns the list on dst, None elsewhere."""
    on = dist.is_initialized()   # one rank with the group initialised still runs the collectives (bench --force-dist)
    world = dist.get_world_size() if on else 1
    rank = dist.get_rank() if on else 0
    n = int(tensors[0].shape[0])
    if any(int(t.shape[0]) != n for t in tensors):
        raise ValueError("every buffer needs the same leading (lane) dimension")
    dev = tensors[0].device
    widths = [_row_bytes(t) for t in tensors]
    flat = torch.cat([t.contiguous().reshape(n, -1).view(torch.uint8).reshape(n, w) for t, w in zip(tensors, widths)],
                     dim=1) if n else torch.zeros((0, sum(widths)), dtype=torch.uint8, device=dev)
    if on and dist.get_backend() == "gloo" and flat.is_cuda:   # gloo gathers host tensors
        flat, dev = flat.cpu(), torch.device("cpu")
    if not on:
        full, counts = flat, [n]
    else:
        cnt = torch.tensor([n], dtype=torch.int64, device=dev)
        counts_t = [torch.zeros_like(cnt) for _ in range(world)]
        dist.all_gather(counts_t, cnt)
        counts = [int(c.item()) for c in counts_t]
        m = max(counts)
        pad = torch.zeros((m, flat.shape[1]), dtype=torch.uint8, device=dev)
        pad[:n] = flat
        if dist.get_backend() == "nccl":   # RCCL all_gather_into_tensor (RCCL emulates gather with it anyway)
            out = torch.empty((world * m, flat.shape[1]), dtype=torch.uint8, device=dev)
            dist.all_gather_into_tensor(out, pad)
            parts = list(out.split(m, dim=0))
        else:
            parts = [torch.empty_like(pad) for _ in range(world)] if rank == dst else None
            dist.gather(pad, gather_list=parts, dst=dst)
        if rank != dst:
            return None
        full = torch.cat([p[:c] for p, c in zip(parts, counts)], dim=0)
    if rank != dst:
        return None
    out, c = [], 0
    for t, w in zip(tensors, widths):
        col = full[:, c:c + w].contiguous()
        out.append(col.view(t.dtype).reshape((full.shape[0],) + tuple(t.shape[1:])))
        c += w
    return out
