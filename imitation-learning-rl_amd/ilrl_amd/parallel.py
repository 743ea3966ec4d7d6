"""Multi-GPU layout: one process per GPU, env lanes sharded by rank.

* Rank r owns global lanes [r*n, (r+1)*n); each lane's RNG stream is keyed by its GLOBAL id
  (hum_config.lane_offset), so results are independent of how many GPUs share the job.
* Env stepping needs no collective (weak scaling).  The only exchange is the trajectory gather to the
  learner rank (obs / action / reward / done per step or per rollout fragment), done with ONE
  collective per buffer over torch.distributed ("nccl" = RCCL over xGMI on MI355X, "gloo" on CPU).
"""
import torch
import torch.distributed as dist


def shard(n_total, world, rank):
    """(lane_offset, n_local) of `rank` for n_total lanes split over `world` ranks (contiguous shards)."""
    base, rem = divmod(n_total, world)
    n = base + (1 if rank < rem else 0)
    off = rank * base + min(rank, rem)
    return off, n


def gather_trajectories(tensors, dst=0):
    """Gather per-rank trajectory buffers (equal shapes per rank) onto `dst` as one [world*n, ...] tensor
    each.  Buffers are packed into a single flat float32 message so RCCL moves one large payload per call
    (xGMI is point-to-point: few large collectives beat many small ones).  Returns a list on dst, None
    elsewhere."""
    world = dist.get_world_size()
    rank = dist.get_rank()
    flat = torch.cat([t.reshape(t.shape[0], -1).to(torch.float32) for t in tensors], dim=1).contiguous()
    if world == 1:
        parts = [flat]
    elif dist.get_backend() == "nccl":   # RCCL: all_gather_into_tensor (gather is emulated by RCCL anyway)
        out = torch.empty((world * flat.shape[0], flat.shape[1]), dtype=flat.dtype, device=flat.device)
        dist.all_gather_into_tensor(out, flat)
        parts = [out]
    else:
        bufs = [torch.empty_like(flat) for _ in range(world)] if rank == dst else None
        dist.gather(flat, gather_list=bufs, dst=dst)
        parts = bufs
    if rank != dst:
        return None
    full = torch.cat(parts, dim=0)
    out, c = [], 0
    for t in tensors:
        w = int(t[0].numel()) if t.shape[0] else 0
        out.append(full[:, c:c + w].reshape((full.shape[0],) + tuple(t.shape[1:])).to(t.dtype))
        c += w
    return out
