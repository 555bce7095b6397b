"""The register-resident server epoch tensor-parallel across REAL processes on ONE GPU: T
ranks each run their shard's persistent launch (csrc/resident.hip) with 256 / T workgroups,
so all T launches are resident on the device together, and exchange their fc2 product rows
through the peer-mapped region in-launch (8-byte tagged granules, system scope) — the
multi-GPU code path minus the xGMI links.  Checks on every rank: no wait gave up, the
replicated parameters (fc2 bias, fc3) and the per-row losses are bitwise identical across
ranks, and the losses match an fp32 torch run of the whole (unsharded) tail.

    python scripts/resident_tp_one_gpu.py [T] [resident|hybrid]     (spawns its own T ranks)

`hybrid` runs the same check on the hybrid persistent executor (csrc/hybrid.hip: fc2 tiles
on-chip, fc1 streamed, the fc2 product exchanged by the same granule protocol).
"""
import copy
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def worker(rank, world, port, kind):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # SL_RANK_DEVICES=D: rank r on cuda:(r % D) (tests/test_multi_gpu.py: the same protocol across
    # devices, over xGMI); default 1: every rank shares cuda:0
    ndev = int(os.environ.get("SL_RANK_DEVICES", "1"))
    torch.cuda.set_device(rank % ndev)
    dev = torch.device("cuda", rank % ndev)
    from splitlearning_amd import ops
    from splitlearning_amd.engine import OptSlot, TailEngine, adam
    from splitlearning_amd.models.zoo import LinearSpec, TailSpec, _MLP
    from splitlearning_amd.ops import rng
    from splitlearning_amd.parallel.rccl import ipc_allreduce, make_ipc_allreduce
    ops.set_backend("hip")
    ipc = make_ipc_allreduce(list(range(world)), rank)
    print(f"rank {rank}: ipc {'up' if ipc is not None else 'unavailable'}", flush=True)
    ok = ipc is not None
    if ok:
        # fc2 width: the resident executor holds <= 4 fc2 rows per workgroup (256 / T workgroups)
        n2 = min(256, 4 * (256 // world))
        spec = TailSpec([LinearSpec("fc1", 1024, 96 * world, True, 0.25), LinearSpec("fc2", 96 * world, n2, True, 0.25),
                         LinearSpec("fc3", n2, 10, False, 0.0)])
        B, n, seed_base = 16, 16 * 6, 5
        g = torch.Generator().manual_seed(3)
        acts = (torch.rand(n, 1024, generator=g) * 4).to(dev)
        labels = torch.randint(0, 10, (n,), generator=g).to(dev)
        torch.manual_seed(9)
        base = _MLP(spec)
        mine = TailEngine(copy.deepcopy(base), spec, dev, tp_rank=rank, tp_size=world, allreduce=ipc_allreduce(ipc),
                          seed_base=seed_base)
        mine.resident_workgroups = 256 // world if ndev == 1 else 0
        mine.resident_timeout_s = 5.0
        slot = OptSlot(adam(1e-3, 1e-5))
        ok = mine.hybrid_ok(slot, B) if kind == "hybrid" else mine.resident_ok(slot, B)
        print(f"rank {rank}: {kind} fits {ok}", flush=True)
        if ok:
            try:
                run = mine.run_hybrid_epoch if kind == "hybrid" else mine.run_resident_epoch
                loss = run(acts, labels, slot, B)
                torch.cuda.synchronize()
            except RuntimeError as e:
                print(f"rank {rank}: {kind} epoch failed: {e}", flush=True)
                ok = False
        if ok:
            rep = torch.cat([loss, mine.layers[1].b, mine.layers[2].W.reshape(-1), mine.layers[2].b]).cpu()
            outs = [torch.empty_like(rep) for _ in range(world)]
            dist.all_gather(outs, rep)
            same = all(torch.equal(o, rep) for o in outs)
            print(f"rank {rank}: replicated state and losses bitwise equal across ranks {same}", flush=True)
            ref = copy.deepcopy(base).to(dev)
            opt = torch.optim.Adam(ref.parameters(), lr=1e-3, weight_decay=1e-5)
            losses = []
            for i in range(n // B):
                x, y = acts[i * B:(i + 1) * B], labels[i * B:(i + 1) * B]
                h = x
                for li, lin in enumerate(ref.linears()):
                    ls = spec.layers[li]
                    h = F.linear(h, lin.weight, lin.bias)
                    if ls.relu:
                        h = F.relu(h)
                    if ls.dropout:
                        keep = rng.keep_mask(rng.step_seed(seed_base, li, i + 1), h.shape[0], h.shape[1], ls.dropout,
                                             device=dev)
                        h = h * keep / (1 - ls.dropout)
                opt.zero_grad()
                lr_ = F.cross_entropy(h, y, reduction="none")
                lr_.mean().backward()
                opt.step()
                losses.append(lr_.detach())
            close = torch.allclose(loss, torch.cat(losses), rtol=1e-3, atol=1e-3)
            print(f"rank {rank}: losses close to torch {close} (max diff "
                  f"{(loss - torch.cat(losses)).abs().max().item():.2e})", flush=True)
            ok = same and close
    flags = [None] * world
    dist.all_gather_object(flags, bool(ok))
    dist.destroy_process_group()
    if not all(flags):
        sys.exit(1)
    print(f"rank {rank}: PASS", flush=True)


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    kind = sys.argv[2] if len(sys.argv) > 2 else "resident"
    port = 29500 + (os.getpid() % 1000)
    mp.spawn(worker, args=(T, port, kind), nprocs=T, join=True)


if __name__ == "__main__":
    main()
