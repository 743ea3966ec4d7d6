"""Probe: can two ranks share the one GPU of the box over the nccl (RCCL) backend?  (bench.py's nccl branch for N > 1
otherwise runs only on the driver's 8-GPU node.)  Prints one line per rank; run under torch.distributed.run."""
import os

import torch
import torch.distributed as dist

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
t = torch.full((4,), float(rank + 1), device="cuda:0")
dist.all_reduce(t)
torch.cuda.synchronize()
print("rank %d all_reduce -> %s" % (rank, t.tolist()), flush=True)
dist.destroy_process_group()
