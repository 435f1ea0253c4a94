"""Probe: can two ranks share one GPU under the RCCL ('nccl') backend?
(python tools/probes/rccl_same_gpu.py; spawns 2 ranks on cuda:0)"""
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def run(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    t = torch.full((1 << 20,), float(rank + 1), device=dev)
    dist.broadcast(t, src=0)
    s = torch.tensor([float(rank)], device=dev)
    dist.all_reduce(s, op=dist.ReduceOp.MAX)
    torch.cuda.synchronize()
    print(f"rank {rank}: broadcast {t[0].item()} {t[-1].item()} max {s.item()}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    mp.spawn(run, args=(2, port), nprocs=2, join=True)
