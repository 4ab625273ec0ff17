"""Which collectives does the gloo backend run on CUDA tensors (two ranks sharing one GPU)?"""
import os
import sys

import torch
import torch.distributed as dist


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    dev = torch.device("cuda", 0)
    x = torch.full((8,), float(rank + 1), device=dev)
    res = {}
    for name, fn in {
        "all_reduce": lambda: dist.all_reduce(x.clone()),
        "all_gather_into_tensor": lambda: dist.all_gather_into_tensor(torch.empty(8 * world, device=dev), x),
        "reduce_scatter_tensor": lambda: dist.reduce_scatter_tensor(torch.empty(8 // world, device=dev), x),
        "all_to_all_single": lambda: dist.all_to_all_single(torch.empty_like(x), x),
        "broadcast": lambda: dist.broadcast(x.clone(), 0),
    }.items():
        try:
            fn()
            torch.cuda.synchronize()
            res[name] = "ok"
        except Exception as e:  # noqa: BLE001
            res[name] = repr(e)[:120]
    if rank == 0:
        print(res, flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
