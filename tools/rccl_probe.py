"""Does RCCL run here?  W ranks of backend 'nccl' (RCCL on ROCm), every rank on cuda:0:
an all_reduce of int64 and an all_gather_into_tensor of uint8, checked exactly.

    python tools/rccl_probe.py W
"""
import os
import socket
import sys


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    try:
        t = torch.arange(1000, dtype=torch.int64, device="cuda") * (rank + 1)
        dist.all_reduce(t)
        want = torch.arange(1000, dtype=torch.int64, device="cuda") * (world * (world + 1) // 2)
        g = torch.empty(world * 4096, dtype=torch.uint8, device="cuda")
        mine = torch.full((4096,), rank + 7, dtype=torch.uint8, device="cuda")
        dist.all_gather_into_tensor(g, mine)
        gw = torch.cat([torch.full((4096,), r + 7, dtype=torch.uint8, device="cuda") for r in range(world)])
        torch.cuda.synchronize()
        print(f"rank {rank}/{world}: all_reduce exact {bool(torch.equal(t, want))}, "
              f"all_gather exact {bool(torch.equal(g, gw))}", flush=True)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    import torch.multiprocessing as mp

    W = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    mp.spawn(_rank, args=(W, _free_port()), nprocs=W, join=True)
