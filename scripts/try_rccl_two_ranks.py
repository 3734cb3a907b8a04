"""Probe: can two RCCL ranks share the one GPU of the test box?  (If so, the nccl path of the PPO update can be
tested there.)  Prints one line per rank."""
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def work(rank, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2")
    torch.cuda.set_device(0)
    try:
        dist.init_process_group("nccl", rank=rank, world_size=2)
        x = torch.full((1024,), float(rank + 1), device="cuda:0")
        dist.all_reduce(x)
        torch.cuda.synchronize()
        print(f"rank {rank}: all_reduce ok, value {float(x[0])}", flush=True)
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        print(f"rank {rank}: failed: {type(e).__name__}: {str(e)[:300]}", flush=True)


if __name__ == "__main__":
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(work, args=(port,), nprocs=2)
