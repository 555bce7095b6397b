"""Interleaved kernel-variant A/B of Bob's server step issued by the native executor.

`scripts/cache_ab.py` issues each step from Python; at a TP = 8 shard the GPU finishes a
step in ~50 us, the same order as Python's issue cost, so host jitter there can swamp a
few-us kernel change.  This script drives `TailEngine.run_native_epoch` (`_C.ServerEpoch`,
csrc/engine.cpp) instead — the path `bench.py` / the SISA protocol use — with a 1-rank
RCCL communicator standing in for the tensor-parallel all-reduce.

    python scripts/native_ab.py --tp 1 2 4 8 --variants 5=0 5=99 [--rounds 5 --epochs 4]

Each variant is `SLOT=VALUE[,SLOT=VALUE]` (`_C.set_variant`); all variants run in one
process in interleaved rounds and the median / min us per step are printed.
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


def parse(v):
    """`SLOT=VALUE[,...]`; the key `fences` (0 / 1) toggles the peer-mapped all-reduce's
    release / acquire fences (`--allreduce ipc`) instead of a kernel-variant slot, the key
    `chain` (0 / 1) the executor's persistent chain launch (csrc/chain.hip)."""
    return {(a if a in ("fences", "chain") else int(a)): int(b) for a, b in (kv.split("=") for kv in v.split(","))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tp", type=int, nargs="+", default=[1, 8])
    ap.add_argument("--variants", nargs="+", default=["5=0", "5=99"])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--epochs", type=int, default=4, help="timed epochs (64 steps each) per variant per round")
    ap.add_argument("--allreduce", choices=("rccl", "ipc"), default="rccl",
                    help="TP > 1 stand-in all-reduce: a 1-rank RCCL communicator or a 1-rank peer-mapped "
                         "all-reduce (csrc/ipc_ar.h: its kernel runs, with no peer to wait for)")
    ap.add_argument("--trace", action="store_true", help="print the last chain launch's phase stamps")
    a = ap.parse_args()
    C = H.C()
    dev = torch.device("cuda", 0)
    ops.set_backend("hip")
    B, nb = 16, 64
    slots = sorted({s for v in a.variants for s in parse(v) if s not in ("fences", "chain")})
    for tp in a.tp:
        torch.manual_seed(0)
        acts = torch.rand(B * nb, 5408, device=dev) * 20
        labels = torch.randint(0, 10, (B * nb,), device=dev)
        ar = ipc = None
        if tp > 1:
            from splitlearning_amd.parallel.rccl import ipc_allreduce, native_allreduce, self_comm
            if a.allreduce == "ipc":
                ipc = C.IpcAllReduce(1, 0, 64 * 1024)
                ipc.open([ipc.handle()])
                ar = ipc_allreduce(ipc)
            else:
                ar = native_allreduce(self_comm())
        tail = TailEngine(ServerTailSisa(), sisa_server_spec(), dev, tp_rank=0, tp_size=tp, allreduce=ar)
        tail.chain_trace = a.trace
        slot = OptSlot(adam(1e-3, 1e-5))
        assert tail.native_epoch_ok(B)
        tail.lookahead_prologue(acts[:B])
        pre = True

        def epochs(k):
            nonlocal pre
            for _ in range(k):
                tail.run_native_epoch(acts, labels, slot, B, pre)
                pre = tail._pre is not None
                if not pre:
                    tail.lookahead_prologue(acts[:B])
                    pre = True

        res = {v: [] for v in a.variants}
        for _ in range(a.rounds):
            for v in a.variants:
                for s in slots:
                    C.set_variant(s, 0)
                if getattr(tail, "_native", None) is None:
                    pre = False
                for s, val in parse(v).items():
                    if s == "fences":
                        if ipc is not None:
                            ipc.set_fences(bool(val))
                    else:
                        C.set_variant(s, val)
                epochs(1)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                epochs(a.epochs)
                torch.cuda.synchronize()
                res[v].append((time.perf_counter() - t0) / (a.epochs * nb) * 1e6)
                if a.trace and ch:
                    tr = tail._native[2].chain_trace().cpu()
                    t0w = int(tr[0])
                    print(f"tp={tp} chain phases (us after wg 0 start) wg0: "
                          + " ".join(f"{(int(x) - t0w) / 100:.2f}" for x in tr[:15])
                          + " | wg last: " + " ".join(f"{(int(x) - t0w) / 100:.2f}" for x in tr[16:31]), flush=True)
        for s in slots:
            C.set_variant(s, 0)
        for v, xs in res.items():
            print(f"tp={tp} {v:10s} median {statistics.median(xs):7.2f} us/step  min {min(xs):7.2f}  "
                  f"({' '.join(f'{x:.1f}' for x in xs)})", flush=True)
        del tail, slot, acts
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
