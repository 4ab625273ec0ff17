"""Probe: can two RCCL ranks share one GPU (an all-reduce and a reduce-scatter)? Run under
torch.distributed.run with 2 processes; prints one line per rank. (NCCL refuses duplicate devices.)"""
import os
import sys

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
try:
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    x = torch.full((1024,), float(rank + 1), device="cuda")
    dist.all_reduce(x)
    y = torch.empty(512, device="cuda")
    dist.reduce_scatter_tensor(y, x)
    torch.cuda.synchronize()
    print(f"rank {rank}: all_reduce {x[0].item()} reduce_scatter {y[0].item()}", flush=True)
    dist.destroy_process_group()
except Exception as e:  # noqa: BLE001
    print(f"rank {rank}: {type(e).__name__}: {str(e)[:300]}", flush=True)
    sys.exit(3)
