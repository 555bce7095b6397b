"""Server step time of the hybrid persistent epoch (`_C.HybridEpoch`, csrc/hybrid.hip) against
the launch-per-stage native executor (`_C.ServerEpoch`, csrc/engine.cpp) on the same shard of
model2_sisa, one MI355X.

TP > 1 runs shard 0 of the full model with a 1-rank peer-mapped region standing in for the
other ranks (the exchange's stores and tag polls run, there is no peer to wait for).
Interleaved rounds, us per server step over one client epoch of `--steps` batches of 16 (a
ws = 2 SISA client holds 3,500 batches).  `--trace` prints the hybrid launch's phase stamps.

    python scripts/hybrid_ab.py --tp 1 2 4 --steps 500 --rounds 3
"""
import argparse
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from splitlearning_amd import ops  # noqa: E402
from splitlearning_amd.engine import OptSlot, TailEngine, adam  # noqa: E402
from splitlearning_amd.models import ServerTailSisa, sisa_server_spec  # noqa: E402
from splitlearning_amd.ops import hip_ops as H  # noqa: E402

PHASES = ["F wait", "F h1 load+mma", "H wait", "H+L", "S wait", "S", "H2 wait", "H2", "B wait", "B dgrad",
          "W2 update", "U wait P", "U dz1+stream", "flush", "end"]


# stamps of csrc/hybrid.hip HY_MARK: (index, label, who runs it)
STAMPS = [(14, "flush end", "all"), (1, "F wait end (h1 published)", "all"), (2, "F arrive", "all"),
          (3, "H wait end", "head"), (4, "H arrive", "head"), (5, "S wait end", "rows"), (6, "S arrive", "rows"),
          (7, "H2 wait end", "head"), (8, "H2 arrive", "head"), (9, "B wait end", "all"), (10, "B arrive", "all"),
          (11, "W2 update end", "all"), (12, "P wait end (stream start)", "all"), (13, "stream end", "all")]


def critical_path(tp, ta, G):
    """Per-seam latency table of one launch: every workgroup's phase stamps for consecutive
    steps, each boundary as min / median / max over the workgroups that run it, in us after the
    previous step's LAST stream end (T0), averaged over the step pairs.  A seam's latency is the
    gap between the last producer's arrival (max of the arrive row) and the first consumer's
    release (min of the next wait-end row)."""
    NS = ta.shape[0]
    rows = {k: [] for k, _, _ in STAMPS}
    slen, spread = [], []
    for s in range(NS - 1):
        t0 = ta[s, :, 13].max()
        for k, _, _ in STAMPS:
            src = ta[s] if k == 14 else ta[s + 1]
            v = src[:, k]
            v = v[v > 0] - t0
            if v.numel():
                rows[k].append((v.min().item(), v.median().item(), v.max().item()))
        d = ta[s, :, 13] - ta[s, :, 12]
        slen.append((d.min().item(), d.median().item(), d.max().item()))
        spread.append((ta[s + 1, :, 13].max() - t0).item())
    print(f"tp={tp} critical path (us after the previous step's last stream end; min / median / max over "
          f"workgroups, mean of {NS - 1} step pairs):", flush=True)
    prev_max = None
    for k, label, who in STAMPS:
        if not rows[k]:
            continue
        mn, md, mx = (statistics.mean(r[i] for r in rows[k]) for i in range(3))
        gap = f"  (+{mn - prev_max:5.2f} from the last arrival above)" if prev_max is not None and "wait" in label else ""
        print(f"tp={tp}   {label:28s} [{who:4s}] {mn:7.2f} {md:7.2f} {mx:7.2f}{gap}", flush=True)
        prev_max = mx
    mn, md, mx = (statistics.mean(r[i] for r in slen) for i in range(3))
    print(f"tp={tp}   stream length min / median / max {mn:.2f} / {md:.2f} / {mx:.2f}; step (last stream end to "
          f"last stream end) {statistics.mean(spread):.2f}", flush=True)
    # where the slow streams are: by w % 8 (the XCD under round-robin dispatch) and by w // 32
    d = (ta[:-1, :, 13] - ta[:-1, :, 12]).mean(0)
    e = (ta[:-1, :, 13] - ta[:-1, :, 13].max(1, keepdim=True).values).mean(0)
    print(f"tp={tp}   stream length by w % 8: " + " ".join(f"{d[x::8].mean().item():6.2f}" for x in range(8)), flush=True)
    print(f"tp={tp}   stream length by w // 32: " + " ".join(f"{d[32 * x:32 * x + 32].mean().item():6.2f}"
                                                       for x in range((G + 31) // 32)), flush=True)
    print(f"tp={tp}   stream end - last end by w % 8: " + " ".join(f"{e[x::8].mean().item():6.2f}" for x in range(8)), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    torch.save(ta - ta[ta > 0].min(), f"gpurun_out/hybrid_tall_tp{tp}.pt")   # relative, float64


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tp", type=int, nargs="+", default=[1])
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--trace", action="store_true")
    ap.add_argument("--only", choices=("both", "hybrid", "native"), default="both")
    ap.add_argument("--nt", type=int, nargs="+", default=[-1],
                    help="hybrid fc1 state stores to A/B: 1 non-temporal, 0 write-through, -1 the default rule")
    a = ap.parse_args()
    C = H.C()
    dev = torch.device("cuda", 0)
    ops.set_backend("hip")
    B = 16
    for tp in a.tp:
        torch.manual_seed(0)
        n = B * a.steps
        acts = torch.rand(n, 5408, device=dev) * 20
        labels = torch.randint(0, 100, (n,), device=dev)
        ar = None
        if tp > 1:
            from splitlearning_amd.parallel.rccl import ipc_allreduce
            ipc = C.IpcAllReduce(1, 0, 64 * 1024)
            ipc.open([ipc.handle()])
            ar = ipc_allreduce(ipc)
        hyk = [f"hybrid{'' if len(a.nt) == 1 else f'_nt{v}'}" for v in a.nt]
        kinds = (["native"] if a.only != "hybrid" else []) + (hyk if a.only != "native" else [])
        mods = {}
        for kind in kinds:
            torch.manual_seed(1)
            tail = TailEngine(ServerTailSisa(), sisa_server_spec(), dev, tp_rank=0, tp_size=tp, allreduce=ar,
                              ws_tag="#" + kind)
            ntv = int(kind.split("_nt")[1]) if "_nt" in kind else a.nt[0]
            tail.hybrid_nt_stores = None if ntv < 0 else ntv
            slot = OptSlot(adam(1e-3, 1e-5))
            mods[kind] = (tail, slot)
        hk = [k for k in mods if k.startswith("hybrid")]
        bad = [k for k in hk if not mods[k][0].hybrid_ok(mods[k][1], B)]
        if bad:
            t0, s0 = mods[bad[0]]
            print(f"tp={tp}: hybrid epoch does not fit: {t0._hybrid_executor(s0, B).why()}", flush=True)
            continue

        def run(kind, k):
            tail, slot = mods[kind]
            for _ in range(k):
                if kind == "native":
                    tail.lookahead_prologue(acts[:B])
                    tail.run_native_epoch(acts, labels, slot, B, True)
                else:
                    tail.run_hybrid_epoch(acts, labels, slot, B)

        res = {k: [] for k in mods}
        for _ in range(a.rounds):
            for kind in mods:
                run(kind, 1)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                run(kind, a.epochs)
                torch.cuda.synchronize()
                res[kind].append((time.perf_counter() - t0) / (a.epochs * a.steps) * 1e6)
        for kind, xs in res.items():
            print(f"tp={tp} {kind:8s} median {statistics.median(xs):7.2f} us/step  min {min(xs):7.2f}  "
                  f"({' '.join(f'{x:.1f}' for x in xs)})", flush=True)
        if a.trace and hk:
            tail, slot = mods[hk[-1]]
            ex = tail._hybrid_executor(slot, B)
            ts = 64
            tr = torch.zeros(2, ts, 16, dtype=torch.int64, device=dev)
            loss = torch.empty(n, device=dev)
            G = ex.workgroups()
            NS = 8
            tall = torch.zeros(NS, G, 16, dtype=torch.int64, device=dev)
            ex.run(acts, labels, loss, tail.seed_base, tail.fwd_count, slot.t, tr, tall, 40)
            torch.cuda.synchronize()
            critical_path(tp, tall.cpu().double() / 100.0, G)   # us (100 MHz wall clock)
            khz = 100000.0
            t = tr.cpu().double()
            for wgi, name in ((0, "wg 0"), (1, "wg G-1")):
                d = (t[wgi, 8:ts - 1, 1:] - t[wgi, 8:ts - 1, :-1]) / khz * 1e3
                valid = (t[wgi, 8:ts - 1, 1:] > 0) & (t[wgi, 8:ts - 1, :-1] > 0)
                parts = []
                for k in range(14):
                    v = d[:, k][valid[:, k]]
                    if v.numel():
                        parts.append(f"{PHASES[k]} {v.mean().item():.2f}")
                fl = t[wgi, 8:ts - 1]
                okf = (fl[:, 15] > 0) & (fl[:, 13] > 0) & (fl[:, 14] > 0)
                if okf.any():
                    dr = ((fl[:, 15] - fl[:, 13]) / khz * 1e3)[okf].mean().item()
                    rest = ((fl[:, 14] - fl[:, 15]) / khz * 1e3)[okf].mean().item()
                    parts.append(f"(flush: drain {dr:.2f} + publish {rest:.2f})")
                step = (t[wgi, 9:ts - 1, 0] - t[wgi, 8:ts - 2, 0]) / khz * 1e3
                print(f"tp={tp} trace {name}: step {step.mean().item():.2f} us | " + ", ".join(parts), flush=True)
        del mods, acts
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
