"""The persistent chain launch (csrc/chain.hip) tensor-parallel across REAL processes on ONE
GPU: T ranks each run their shard's launch-per-stage epoch (`_C.ServerEpoch`) with the chain
on and 256 / T workgroups per chain launch, so the T ranks' launches of a step are resident on
the device together, and exchange their fc2 partial products through the peer-mapped region
in-launch (8-byte tagged granules, system scope) — the multi-GPU code path minus the xGMI
links.  The epoch's trailing partial batch runs on the six kernels, whose fused head uses the
same region with flags, so the two protocols alternate on it.  Checks on every rank: the chain
was set up, no wait gave up, the replicated parameters (fc2 bias, fc3) and the per-row losses
are bitwise identical across ranks, and the losses match an fp32 torch run of the whole
(unsharded) tail.

    python scripts/chain_tp_one_gpu.py [T]      (spawns its own T ranks)
"""
import copy
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def worker(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
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
        spec = TailSpec([LinearSpec("fc1", 1024, 96 * world, True, 0.25), LinearSpec("fc2", 96 * world, 256, True, 0.25),
                         LinearSpec("fc3", 256, 10, False, 0.0)])
        B, n, seed_base = 16, 16 * 6 + 5, 5
        g = torch.Generator().manual_seed(3)
        acts = (torch.rand(n, 1024, generator=g) * 4).to(dev)
        labels = torch.randint(0, 10, (n,), generator=g).to(dev)
        torch.manual_seed(9)
        base = _MLP(spec)
        mine = TailEngine(copy.deepcopy(base), spec, dev, tp_rank=rank, tp_size=world, allreduce=ipc_allreduce(ipc),
                          seed_base=seed_base)
        mine.server_chain = True
        mine.chain_workgroups = 256 // world
        mine.chain_timeout_s = 5.0
        slot = OptSlot(adam(1e-3, 1e-5))
        ok = mine.native_epoch_ok(B)
        if ok:
            try:
                mine.lookahead_prologue(acts[:B])
                loss = mine.run_native_epoch(acts, labels, slot, B, True)
                torch.cuda.synchronize()
                ex = mine._native[2]
                ok = ex.chain_enabled()
                print(f"rank {rank}: chain {ok} ({ex.chain_why() or 'set up'})", flush=True)
            except RuntimeError as e:
                print(f"rank {rank}: epoch failed: {e}", flush=True)
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
            for i in range(-(-n // B)):
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
    port = 29500 + (os.getpid() % 1000)
    mp.spawn(worker, args=(T, port), nprocs=T, join=True)


if __name__ == "__main__":
    main()
