"""Diagnostic: T=2 resident epochs on one GPU, no fault, several epochs, each epoch's losses vs torch."""
import copy, os, sys
import torch, torch.distributed as dist, torch.multiprocessing as mp, torch.nn.functional as F
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))

def worker(rank, world, port, kind, n_eng, epochs):
    os.environ["MASTER_ADDR"] = "127.0.0.1"; os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0); dev = torch.device("cuda", 0)
    from splitlearning_amd import ops
    from splitlearning_amd.engine import OptSlot, TailEngine, adam
    from splitlearning_amd.models.zoo import LinearSpec, TailSpec, _MLP
    from splitlearning_amd.ops import rng
    from splitlearning_amd.parallel.rccl import ipc_allreduce, make_ipc_allreduce
    ops.set_backend("hip")
    ipc = make_ipc_allreduce(list(range(world)), rank)
    n2 = min(256, 4 * (256 // world))
    spec = TailSpec([LinearSpec("fc1", 1024, 96 * world, True, 0.25), LinearSpec("fc2", 96 * world, n2, True, 0.25),
                     LinearSpec("fc3", n2, 10, False, 0.0)])
    B, n, seed_base = 16, 16 * 8, 5
    g = torch.Generator().manual_seed(3)
    acts = (torch.rand(n, 1024, generator=g) * 4).to(dev)
    labels = torch.randint(0, 10, (n,), generator=g).to(dev)
    torch.manual_seed(9)
    base = _MLP(spec)
    engs = []
    for k in range(n_eng):
        t = TailEngine(copy.deepcopy(base), spec, dev, tp_rank=rank, tp_size=world, allreduce=ipc_allreduce(ipc),
                       seed_base=seed_base, ws_tag=f"#d{k}")
        t.resident_workgroups = 256 // world
        s = OptSlot(adam(1e-3, 1e-5))
        ok = t.hybrid_ok(s, B) if kind == "hybrid" else t.resident_ok(s, B)
        engs.append((t, s))
    ref = copy.deepcopy(base).to(dev)
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3, weight_decay=1e-5)
    step = 0
    for e in range(epochs):
        last = []
        for i in range(n // B):
            step += 1
            x, y = acts[i * B:(i + 1) * B], labels[i * B:(i + 1) * B]
            h = x
            for li, lin in enumerate(ref.linears()):
                ls = spec.layers[li]
                h = F.linear(h, lin.weight, lin.bias)
                if ls.relu: h = F.relu(h)
                if ls.dropout:
                    keep = rng.keep_mask(rng.step_seed(seed_base, li, step), h.shape[0], h.shape[1], ls.dropout, device=dev)
                    h = h * keep / (1 - ls.dropout)
            opt.zero_grad(); lr_ = F.cross_entropy(h, y, reduction="none"); lr_.mean().backward(); opt.step()
            last.append(lr_.detach())
        ref_l = torch.cat(last)
        for k, (t, s) in enumerate(engs):
            run = t.run_hybrid_epoch if kind == "hybrid" else t.run_resident_epoch
            if os.environ.get("ALT") and e % 2 == 1:
                from splitlearning_amd.engine.resident import _launch_per_stage_epoch
                l = _launch_per_stage_epoch(t, s, acts, labels, B)
            else:
                l = run(acts, labels, s, B)
            torch.cuda.synchronize()
            nanw = sum(int(torch.isnan(L.W).sum().item()) for L in t.layers)
            print(f"rank {rank}: {kind} engine {k} epoch {e} ({'lps' if os.environ.get('ALT') and e % 2 else kind}): losses vs torch max |d| {(l - ref_l).abs().max().item():.3g}; NaN in W {nanw}", flush=True)
    dist.barrier(); dist.destroy_process_group()

if __name__ == "__main__":
    kind = sys.argv[1]; n_eng = int(sys.argv[2]); epochs = int(sys.argv[3])
    mp.spawn(worker, args=(2, 29500 + os.getpid() % 1000, kind, n_eng, epochs), nprocs=2, join=True)
