"""Tensor-parallel Bob as T real processes on ONE GPU: each rank runs its shard of the
production native executor (`_C.ServerEpoch`, csrc/engine.cpp) with the peer-mapped
all-reduce (csrc/ipc_ar.h) between the processes — the multi-GPU code path minus xGMI
(RCCL refuses two ranks on one device; the peer-mapped regions do not).  Every rank also
runs the single-process emulation of the same T-way epoch (`_C.tp_emulate_epoch`, whose
stand-in all-reduce sums the shards in the same rank order) and checks that its own
shard's weights and losses are BITWISE the emulation's shard.

    python scripts/tp_processes_one_gpu.py [T] [epochs]      (spawns its own T ranks)
"""
import copy
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def worker(rank, world, port, epochs):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    from splitlearning_amd import ops
    from splitlearning_amd.engine import OptSlot, TailEngine, adam
    from splitlearning_amd.models import ServerTailSisa, sisa_server_spec
    from splitlearning_amd.parallel.rccl import ipc_allreduce, make_ipc_allreduce
    ops.set_backend("hip")
    ipc = make_ipc_allreduce(list(range(world)), rank)
    print(f"rank {rank}: ipc allreduce {'up' if ipc is not None else 'unavailable'}", flush=True)
    ok = ipc is not None
    if ok:
        B, n = 16, 16 * 12 + 5
        g = torch.Generator().manual_seed(11)
        acts = (torch.rand(n, 5408, generator=g) * 30).to(dev)
        labels = torch.randint(0, 10, (n,), generator=g).to(dev)
        torch.manual_seed(0)
        base = ServerTailSisa()
        mine = TailEngine(copy.deepcopy(base), sisa_server_spec(), dev, tp_rank=rank, tp_size=world,
                          allreduce=ipc_allreduce(ipc), seed_base=777)
        slot = OptSlot(adam(1e-3, 1e-5))
        shards = [TailEngine(copy.deepcopy(base), sisa_server_spec(), dev, tp_rank=r, tp_size=world,
                             allreduce=None, seed_base=777, ws_tag=f"#emu{world}.{r}") for r in range(world)]
        slots = [OptSlot(adam(1e-3, 1e-5)) for _ in range(world)]
        assert mine.native_epoch_ok(B)
        for ep in range(epochs):
            mine.lookahead_prologue(acts[:B])
            loss = mine.run_native_epoch(acts, labels, slot, B, True)
            loss_e = TailEngine.emulate_tp_epoch(shards, slots, acts, labels, B)
            torch.cuda.synchronize()
            same = torch.equal(loss, loss_e) and all(
                torch.equal(a.W, b.W) and torch.equal(a.b, b.b) for a, b in zip(mine.layers, shards[rank].layers))
            same = same and (mine.fwd_count, slot.t) == (shards[rank].fwd_count, slots[rank].t)
            print(f"rank {rank}: epoch {ep} loss {loss.mean().item():.6f} bitwise-emulation {same}", flush=True)
            ok = ok and same
        ok = ok and ipc.error() == 0
    print(f"rank {rank}: {'PASS' if ok else 'FAIL'}", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    E = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    mp.spawn(worker, args=(T, 29633 + T, E), nprocs=T, join=True)
