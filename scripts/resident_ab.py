"""Server step time of the register-resident epoch (`_C.ResidentEpoch`, csrc/resident.hip)
against the launch-per-stage native executor (`_C.ServerEpoch`, csrc/engine.cpp) on the same
tensor-parallel shard of model2_sisa, one MI355X.

TP > 1 runs shard 0 of the full model with a 1-rank peer-mapped region standing in for the
other ranks (as scripts/native_ab.py --allreduce ipc): the exchange's stores, flags and slot
reads run, there is no peer to wait for.  Interleaved rounds, us per server step over one
client epoch of `--steps` batches of 16 (an 8-Alice SISA client holds ~437 batches).

    python scripts/resident_ab.py --tp 8 --steps 437 --rounds 5
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tp", type=int, nargs="+", default=[8])
    ap.add_argument("--steps", type=int, default=437)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--no_ipc", action="store_true", help="shard without the exchange (T = 0)")
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
        mods = {}
        for kind in ("native", "resident"):
            torch.manual_seed(1)
            tail = TailEngine(ServerTailSisa(), sisa_server_spec(), dev, tp_rank=0, tp_size=tp, allreduce=ar,
                              ws_tag="#" + kind)
            slot = OptSlot(adam(1e-3, 1e-5))
            mods[kind] = (tail, slot)
        tail, slot = mods["resident"]
        if not tail.resident_ok(slot, B):
            print(f"tp={tp}: resident epoch does not fit: {tail._resident_executor(slot, B).why()}", flush=True)
            continue

        def run(kind, k):
            tail, slot = mods[kind]
            for _ in range(k):
                if kind == "native":
                    tail.lookahead_prologue(acts[:B])
                    tail.run_native_epoch(acts, labels, slot, B, True)
                else:
                    tail.run_resident_epoch(acts, labels, slot, B)

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
            print(f"tp={tp} {kind:9s} median {statistics.median(xs):7.2f} us/step  min {min(xs):7.2f}  "
                  f"({' '.join(f'{x:.1f}' for x in xs)})", flush=True)
        l1 = mods["native"][0]
        l2 = mods["resident"][0]
        print(f"tp={tp} final loss-free check: native fc1 |W| {l1.layers[0].W.abs().mean().item():.6f} "
              f"resident {l2.layers[0].W.abs().mean().item():.6f}", flush=True)
        del mods, acts
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
