"""The resident executor's adoption probe, tensor-parallel across T REAL processes on ONE GPU,
with and without an injected failure (engine/resident.py decide).

    python scripts/resident_probe_fault_one_gpu.py T fault_rank     (fault_rank -1: no fault)

Every rank builds its shard of a narrow tail (fits the resident executor at 256 / T workgroups
per rank, so the T persistent launches are resident together) with the peer-mapped region
between the ranks, then calls `decide`:
  * no fault: every rank adopts the resident executor;
  * fault_rank r: rank r skips its probe launch, so every other rank's in-launch fc2 exchange
    times out (5 s) and raises the region's error word; every rank must agree "no", re-arm the
    region, and then train a server epoch on the launch-per-stage executor (fused peer-mapped
    all-reduce in the head) without any wait giving up, with the replicated fc3 and fc2 bias
    bitwise equal across ranks.
Each rank prints PASS.  Reference: split_nn.py:183-186 (a failing child must not leave the
survivors inconsistent), data_entities_vanilla_sisa.py:298-313 (the server loop).
"""
import copy
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def worker(rank, world, port, fault):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    if fault >= 0:
        os.environ["SL_FAULT_RESIDENT_PROBE"] = str(fault)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    from splitlearning_amd import ops
    from splitlearning_amd.engine import OptSlot, TailEngine, adam, resident
    from splitlearning_amd.models.zoo import LinearSpec, TailSpec, _MLP
    from splitlearning_amd.parallel.rccl import ipc_allreduce, make_ipc_allreduce
    ops.set_backend("hip")
    ipc = make_ipc_allreduce(list(range(world)), rank)
    ok = ipc is not None
    print(f"rank {rank}: ipc {'up' if ok else 'unavailable'}", flush=True)
    if ok:
        spec = TailSpec([LinearSpec("fc1", 1024, 96 * world, True, 0.25), LinearSpec("fc2", 96 * world, 256, True, 0.25),
                         LinearSpec("fc3", 256, 10, False, 0.0)])
        B, n = 16, 16 * 40
        g = torch.Generator().manual_seed(3)
        acts = (torch.rand(n, 1024, generator=g) * 4).to(dev)
        labels = torch.randint(0, 10, (n,), generator=g).to(dev)
        torch.manual_seed(9)
        tail = TailEngine(_MLP(spec), spec, dev, tp_rank=rank, tp_size=world, allreduce=ipc_allreduce(ipc), seed_base=5)
        tail.resident_workgroups = 256 // world
        slot = OptSlot(adam(1e-3, 1e-5))
        kind, why = resident.decide(tail, slot, B, distributed=True)
        adopted = kind == "resident"
        print(f"rank {rank}: adopted {adopted} ({kind}: {why})", flush=True)
        ok = adopted == (fault < 0)
        if fault >= 0:
            ok = ok and ipc.error() == 0 and ipc.host_error() == 0
            print(f"rank {rank}: error word clear after re-arm {ok}", flush=True)
        if ok:
            try:
                if adopted:
                    tail.run_resident_epoch(acts, labels, slot, B)
                else:
                    tail.lookahead_prologue(acts[:B])
                    tail.run_native_epoch(acts, labels, slot, B, True)
                torch.cuda.synchronize()
                ok = ipc.error() == 0
                print(f"rank {rank}: server epoch on the {'resident' if adopted else 'launch-per-stage'} executor "
                      f"finished, error word {ipc.error()}", flush=True)
            except RuntimeError as e:
                print(f"rank {rank}: server epoch failed: {e}", flush=True)
                ok = False
        if ok:
            rep = torch.cat([tail.layers[1].b, tail.layers[2].W.reshape(-1), tail.layers[2].b]).cpu()
            outs = [torch.empty_like(rep) for _ in range(world)]
            dist.all_gather(outs, rep)
            same = all(torch.equal(o, rep) for o in outs) and bool(torch.isfinite(rep).all())
            print(f"rank {rank}: replicated fc2 bias / fc3 bitwise equal across ranks {same}", flush=True)
            ok = same
    flags = [None] * world
    dist.all_gather_object(flags, bool(ok))
    dist.destroy_process_group()
    if not all(flags):
        sys.exit(1)
    print(f"rank {rank}: PASS", flush=True)


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    fault = int(sys.argv[2]) if len(sys.argv) > 2 else -1
    port = 29600 + (os.getpid() % 1000)
    mp.spawn(worker, args=(T, port, fault), nprocs=T, join=True)


if __name__ == "__main__":
    main()
