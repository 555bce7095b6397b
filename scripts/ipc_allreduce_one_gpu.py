"""T processes on ONE GPU exercise the peer-mapped all-reduce (csrc/ipc_ar.h) end to end:
IPC export of the uncached regions, mapping in every peer process, the set-up self-test,
then random fp32 messages checked bitwise against the rank-ordered fp32 sum, on both
parity buffers, and a latency figure.  Control plane on gloo (CPU).  On one device the
"peer" stores stay on-chip, so the latency is not the xGMI figure; the protocol (handles,
flags, generations, parity reuse, bounded waits) is the same code a multi-GPU node runs.

    python scripts/ipc_allreduce_one_gpu.py [T]      (spawns its own T ranks, default 2)
"""
import os
import sys
import time

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def worker(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # SL_RANK_DEVICES=D: rank r on cuda:(r % D) (tests/test_multi_gpu.py: the same protocol across
    # devices, over xGMI); default 1: every rank shares cuda:0
    ndev = int(os.environ.get("SL_RANK_DEVICES", "1"))
    torch.cuda.set_device(rank % ndev)
    dev = torch.device("cuda", rank % ndev)
    from splitlearning_amd.parallel.rccl import make_ipc_allreduce
    ipc = make_ipc_allreduce(list(range(world)), rank)
    print(f"rank {rank}: ipc allreduce {'up' if ipc is not None else 'unavailable'}", flush=True)
    ok = ipc is not None
    if ok:
        for it, n in enumerate((16000, 16000, 64000, 100, 16000, 5000, 200000, 16000)):
            xs = [torch.randn(n, generator=torch.Generator().manual_seed(1000 * it + r)) for r in range(world)]
            want = xs[0].clone()
            for r in range(1, world):
                want += xs[r]
            x = xs[rank].to(dev)
            ipc.allreduce_sum(x)
            torch.cuda.synchronize()
            if not torch.equal(x.cpu(), want):
                ok = False
                print(f"rank {rank}: MISMATCH at iter {it} n={n}: max err "
                      f"{(x.cpu() - want).abs().max().item()}", flush=True)
        x = torch.ones(16000, device=dev)
        dist.barrier()
        for _ in range(20):
            ipc.allreduce_sum(x)
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        iters = 500
        for _ in range(iters):
            ipc.allreduce_sum(x)
        torch.cuda.synchronize()
        us = (time.perf_counter() - t0) / iters * 1e6
        ok = ok and ipc.error() == 0
        print(f"rank {rank}: {iters} x 64 KB all-reduce {us:.1f} us/call", flush=True)
    if ok and os.environ.get("SL_IPC_TIMEOUT_CHECK") == "1":
        # a peer that never arrives: rank 0's waits must give up (bounded) and raise the
        # error word instead of hanging the GPU; the other ranks issue nothing
        dist.barrier()
        if rank == 0:
            ipc.set_timeout_s(0.5)
            y = torch.ones(16000, device=dev)
            t0 = time.perf_counter()
            ipc.allreduce_sum(y)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            print(f"rank 0: lone all-reduce returned after {dt:.2f} s, error word {ipc.error()}", flush=True)
            ok = ipc.error() == 1 and dt < 10.0
        dist.barrier()
    print(f"rank {rank}: {'PASS' if ok else 'FAIL'}", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    mp.spawn(worker, args=(T, 29613 + T), nprocs=T, join=True)
