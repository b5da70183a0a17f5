"""Probe: can two RCCL ranks share one GPU (for testing the column-sharded path on a
1-GPU box)?  Prints one line: 'rccl-same-gpu ok' or the failure."""
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def run(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world)
    x = torch.full((4,), rank + 1, device="cuda", dtype=torch.int64)
    out = [torch.zeros_like(x) for _ in range(world)]
    dist.all_gather(out, x)
    torch.cuda.synchronize()
    if rank == 0:
        print("rccl-same-gpu ok", [int(t[0]) for t in out], flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    try:
        mp.spawn(run, args=(2, 29533), nprocs=2, join=True)
    except Exception as e:  # noqa: BLE001
        print("rccl-same-gpu FAILED:", repr(e)[:400], flush=True)
        sys.exit(0)
