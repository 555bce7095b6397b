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
            tall = torch.zeros(G, 4, dtype=torch.int64, device=dev)
            ex.run(acts, labels, loss, tail.seed_base, tail.fwd_count, slot.t, tr, tall, 40)
            torch.cuda.synchronize()
            ta = tall.cpu().double() / 100.0   # us (100 MHz wall clock)
            s0 = ta[:, 0].min()
            st, en, fl, nx = ta[:, 0] - s0, ta[:, 1] - s0, ta[:, 2] - s0, ta[:, 3] - s0
            dur = en - st
            print(f"tp={tp} per-workgroup (step 40, us from the first stream start): stream start "
                  f"min/med/max {st.min():.1f}/{st.median():.1f}/{st.max():.1f}; stream length "
                  f"{dur.min():.1f}/{dur.median():.1f}/{dur.max():.1f}; stream end {en.min():.1f}/{en.median():.1f}/"
                  f"{en.max():.1f}; flush end {fl.min():.1f}/{fl.median():.1f}/{fl.max():.1f}; next F released "
                  f"{nx.min():.1f}/{nx.median():.1f}/{nx.max():.1f}", flush=True)
            # is a workgroup's stream length a property of the workgroup within a launch (the same
            # slow ones every step) or of the step?  correlation between steps of one launch
            tall4 = torch.zeros(8, G, 4, dtype=torch.int64, device=dev)
            ex.run(acts, labels, loss, tail.seed_base, tail.fwd_count, slot.t, None, tall4, 40)
            torch.cuda.synchronize()
            t4s = tall4.cpu().double() / 100.0
            d4 = t4s[:, :, 1] - t4s[:, :, 0]
            cc = [torch.corrcoef(torch.stack([d4[0], d4[k]]))[0, 1].item() for k in range(1, 8)]
            slow = [set(torch.argsort(d4[k], descending=True)[:16].tolist()) for k in range(8)]
            common = len(set.intersection(*slow[:4]))
            print(f"tp={tp} per-workgroup stream length, steps 40..47 of one launch: correlation with step 40 "
                  + " ".join(f"{c:.2f}" for c in cc) + f"; workgroups among the 16 slowest in all of steps 40-43: "
                  f"{common}", flush=True)
            xcd = [dur[x::8].mean().item() for x in range(8)]
            print(f"tp={tp} stream length by w % 8: " + " ".join(f"{v:.1f}" for v in xcd), flush=True)
            order = torch.argsort(dur, descending=True)[:8].tolist()
            print(f"tp={tp} slowest workgroups: " + " ".join(f"{w}:{dur[w]:.1f}" for w in order), flush=True)
            blk = [dur[i:i + 32].mean().item() for i in range(0, G, 32)]
            print(f"tp={tp} stream length by w // 32: " + " ".join(f"{v:.1f}" for v in blk), flush=True)
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
