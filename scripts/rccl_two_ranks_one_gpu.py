"""Two processes on ONE GPU: does RCCL accept two ranks on the same device, and does the
native communicator set-up (parallel/rccl.make_native_comm) either work or fall back on
every rank together?  Control plane on gloo (CPU).  If the communicator comes up, an
all-reduce and a grouped send/recv pair on the compute stream are checked.

    python scripts/rccl_two_ranks_one_gpu.py      (spawns its own 2 ranks)
"""
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def worker(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from splitlearning_amd.parallel.rccl import make_native_comm
    comm = make_native_comm([0, 1], rank)
    print(f"rank {rank}: native comm {'up' if comm is not None else 'unavailable (fallback)'}", flush=True)
    if comm is not None:
        t = torch.full((1024,), float(rank + 1), device="cuda")
        comm.allreduce_sum(t)
        torch.cuda.synchronize()
        print(f"rank {rank}: allreduce -> {t[0].item()} (expect 3.0)", flush=True)
        x = torch.full((4096,), float(10 + rank), device="cuda")
        y = torch.empty(4096, device="cuda")
        comm.group_start()
        comm.send(x, 1 - rank)
        comm.recv(y, 1 - rank)
        comm.group_end()
        torch.cuda.synchronize()
        print(f"rank {rank}: sendrecv got {y[0].item()} (expect {10 + 1 - rank})", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    mp.spawn(worker, args=(2, 29611), nprocs=2, join=True)
