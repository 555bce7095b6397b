"""Mid-epoch failure of a tensor-parallel persistent server epoch, survived: T real processes on
ONE GPU, each a Bob shard on the hybrid (or register-resident) executor with the fc2 product
exchanged in-launch through the peer-mapped region; rank 0's launch is made to stop at step
STEP of its second client epoch (SL_FAULT_PERSIST_EPOCH, the kernels' fault_step), so rank 1's
in-launch exchange times out as it would if a peer GPU died or the xGMI exchange hung.

Per rank, engine A runs three client epochs through `engine.resident.Failsafe` (the path
`SisaSession.server_epoch` takes): epoch 0 persistent, epoch 1 fails on every rank -> every
rank restores its shard, re-arms the region, re-runs the epoch on the launch-per-stage
executor, and epoch 2 stays there.  Engine B (same init) runs epoch 0 persistent and epochs
1-2 launch-per-stage with no failure.  Checks on every rank: nothing raised, A's fallback
record names epoch 1, A's parameters, optimizer state and counters are BITWISE B's, and both
are close to an fp32 torch run of the unsharded tail.

    python scripts/persist_fallback_one_gpu.py [T] [hybrid|resident]     (spawns its own T ranks)

Reference failure rule: split_nn.py:183-186 (mp.spawn join=True: one child's exception ends
the job); here the job continues with consistent state instead.
"""
import copy
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

FAULT_STEP = 3


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
    from splitlearning_amd.engine.resident import FAULT_EPOCH_ENV, Failsafe, _launch_per_stage_epoch
    from splitlearning_amd.models.zoo import LinearSpec, TailSpec, _MLP
    from splitlearning_amd.ops import rng
    from splitlearning_amd.parallel.rccl import ipc_allreduce, make_ipc_allreduce
    ops.set_backend("hip")
    ipc = make_ipc_allreduce(list(range(world)), rank)
    print(f"rank {rank}: ipc {'up' if ipc is not None else 'unavailable'}", flush=True)
    ok = ipc is not None
    if ok:
        ipc.set_timeout_s(2.0)            # rank 1's exchange gives up 2 s after rank 0 stopped
    n2 = min(256, 4 * (256 // world))
    spec = TailSpec([LinearSpec("fc1", 1024, 96 * world, True, 0.25), LinearSpec("fc2", 96 * world, n2, True, 0.25),
                     LinearSpec("fc3", n2, 10, False, 0.0)])
    B, n, seed_base, epochs = 16, 16 * 8, 5, 3
    g = torch.Generator().manual_seed(3)
    acts = (torch.rand(n, 1024, generator=g) * 4).to(dev)
    labels = torch.randint(0, 10, (n,), generator=g).to(dev)
    torch.manual_seed(9)
    base = _MLP(spec)

    def engine(tag):
        t = TailEngine(copy.deepcopy(base), spec, dev, tp_rank=rank, tp_size=world, allreduce=ipc_allreduce(ipc),
                       seed_base=seed_base, ws_tag=tag)
        t.resident_workgroups = 256 // world if ndev == 1 else 0
        t.resident_timeout_s = 2.0
        s = OptSlot(adam(1e-3, 1e-5))
        for L in t.layers:
            s.state(f"{L.spec.name}.weight", L.W)
            s.state(f"{L.spec.name}.bias", L.b)
        return t, s

    if ok:
        ta, sa = engine("#fa")
        tb, sb = engine("#fb")
        fits = ta.hybrid_ok(sa, B) if kind == "hybrid" else ta.resident_ok(sa, B)
        fits = fits and (tb.hybrid_ok(sb, B) if kind == "hybrid" else tb.resident_ok(sb, B))
        print(f"rank {rank}: {kind} fits {fits}", flush=True)
        ok = fits
    raised = None
    if ok:
        try:
            os.environ[FAULT_EPOCH_ENV] = f"0:1:{FAULT_STEP}"
            fs = Failsafe(ta, sa, B, group=None)
            ex_a = kind
            la = []
            la_all = []
            canary = (acts.clone(), labels.clone())

            def intact(where):
                ok_a, ok_y = torch.equal(acts, canary[0]), torch.equal(labels, canary[1])
                if not (ok_a and ok_y):
                    print(f"rank {rank}: INPUTS CORRUPTED {where}: acts {ok_a} labels {ok_y}; "
                          f"{int((acts != canary[0]).sum().item())} act elements differ", flush=True)
            for e in range(epochs):
                intact(f"before A epoch {e}")
                if ex_a != "launch_per_stage" and fs.run(ex_a, acts, labels):
                    la_all.append(fs.loss)
                    continue
                ex_a = "launch_per_stage"
                la.append(_launch_per_stage_epoch(ta, sa, acts, labels, B))
                la_all.append(la[-1])
                print(f"rank {rank}: A epoch {e} on launch-per-stage; ipc error word {ipc.error()}", flush=True)
            os.environ.pop(FAULT_EPOCH_ENV)
            print(f"rank {rank}: engine A fallback {fs.fallback}", flush=True)
            intact("after A")
            run_b = tb.run_hybrid_epoch if kind == "hybrid" else tb.run_resident_epoch
            lb_all = [run_b(acts, labels, sb, B)]
            intact("after B epoch 0")
            lb = [_launch_per_stage_epoch(tb, sb, acts, labels, B) for _ in range(epochs - 1)]
            lb_all += lb
            torch.cuda.synchronize()
            for e, (x, y) in enumerate(zip(la_all, lb_all)):
                print(f"rank {rank}: epoch {e} losses A vs B max |d| {(x - y).abs().max().item():.3g}", flush=True)
            for nm, (La, Lb) in zip(("fc1", "fc2", "fc3"), zip(ta.layers, tb.layers)):
                print(f"rank {rank}: {nm} W A vs B max |d| {(La.W - Lb.W).abs().max().item():.3g}", flush=True)
        except Exception as e:                          # the test's point: nothing raises
            raised = e
            print(f"rank {rank}: raised {type(e).__name__}: {e}", flush=True)
            ok = False
    if ok:
        fb_ok = fs.fallback is not None and fs.fallback["epoch"] == 1 and ex_a == "launch_per_stage"
        same = all(torch.equal(La.W, Lb.W) and torch.equal(La.b, Lb.b) for La, Lb in zip(ta.layers, tb.layers))
        for k in sa.states:
            for kk in sa.states[k]:
                same = same and torch.equal(sa.states[k][kk], sb.states[k][kk])
        same = same and (ta.fwd_count, sa.t) == (tb.fwd_count, sb.t) == (epochs * n // B, epochs * n // B)
        same = same and all(torch.equal(x, y) for x, y in zip(la, lb))
        print(f"rank {rank}: fallback at epoch 1 {fb_ok}; state bitwise the clean switch {same}", flush=True)
        # fp32 torch of the whole tail over the same three epochs
        ref = copy.deepcopy(base).to(dev)
        opt = torch.optim.Adam(ref.parameters(), lr=1e-3, weight_decay=1e-5)
        step = 0
        last = []
        for e in range(epochs):
            ep = []
            for i in range(n // B):
                step += 1
                x, y = acts[i * B:(i + 1) * B], labels[i * B:(i + 1) * B]
                h = x
                for li, lin in enumerate(ref.linears()):
                    ls = spec.layers[li]
                    h = F.linear(h, lin.weight, lin.bias)
                    if ls.relu:
                        h = F.relu(h)
                    if ls.dropout:
                        keep = rng.keep_mask(rng.step_seed(seed_base, li, step), h.shape[0], h.shape[1], ls.dropout,
                                             device=dev)
                        h = h * keep / (1 - ls.dropout)
                opt.zero_grad()
                lr_ = F.cross_entropy(h, y, reduction="none")
                lr_.mean().backward()
                opt.step()
                ep.append(lr_.detach())
                if e == epochs - 1:
                    last.append(lr_.detach())
            ep = torch.cat(ep)
            print(f"rank {rank}: epoch {e} vs torch max |d|: A {(la_all[e] - ep).abs().max().item():.3g} "
                  f"B {(lb_all[e] - ep).abs().max().item():.3g}", flush=True)
        nan_a = sum(int(torch.isnan(L.W).sum().item()) for L in ta.layers)
        nan_b = sum(int(torch.isnan(L.W).sum().item()) for L in tb.layers)
        print(f"rank {rank}: NaN in W: A {nan_a} B {nan_b}", flush=True)
        close = torch.allclose(la[-1], torch.cat(last), rtol=2e-3, atol=2e-3)
        print(f"rank {rank}: last epoch's losses close to torch {close} (max diff "
              f"{(la[-1] - torch.cat(last)).abs().max().item():.2e})", flush=True)
        ok = fb_ok and same and close
    flags = [None] * world
    dist.all_gather_object(flags, bool(ok))
    dist.destroy_process_group()
    if not all(flags) or raised is not None:
        sys.exit(1)
    print(f"rank {rank}: PASS", flush=True)


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    kind = sys.argv[2] if len(sys.argv) > 2 else "hybrid"
    port = 29500 + (os.getpid() % 1000)
    mp.spawn(worker, args=(T, port, kind), nprocs=T, join=True)


if __name__ == "__main__":
    main()
