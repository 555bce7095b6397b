"""Drive Bob's server step for rocprofv3 (per-kernel device times):

    rocprofv3 --kernel-trace --stats --output-format csv -d OUT -o step -- \
        python3 scripts/prof_step.py --path fused --steps 200

--path generic|fused|lookahead|graph|native|local (local = the SISA client step).
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from splitlearning_amd import ops  # noqa: E402
from splitlearning_amd.engine import OptSlot, TailEngine, adam  # noqa: E402
from splitlearning_amd.models import ServerTailSisa, sisa_server_spec  # noqa: E402
from splitlearning_amd.ops import hip_ops as H  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--path", default="fused")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--tp", type=int, default=1, help="simulate a TP shard (rank 0 of tp, 1-rank all-reduce)")
    ap.add_argument("--time", action="store_true", help="print wall-clock us/step (second half of the run)")
    ap.add_argument("--variant", action="append", default=[], help="slot=value kernel variant (A/B)")
    ap.add_argument("--allreduce", choices=("rccl", "ipc"), default="rccl",
                    help="TP shard's all-reduce stand-in: 1-rank RCCL or the 1-rank peer-mapped kernel")
    a = ap.parse_args()
    for kv in a.variant:
        slot, val = (int(v) for v in kv.split("="))
        H.C().set_variant(slot, val)
    dev = torch.device("cuda", 0)
    ops.set_backend("hip")
    torch.manual_seed(0)
    n = 16 * 64
    acts = torch.rand(n, 5408, device=dev) * 20
    labels = torch.randint(0, 10, (n,), device=dev)
    ar = None
    if a.tp > 1:
        from splitlearning_amd.parallel.rccl import ipc_allreduce, native_allreduce, self_comm
        if a.allreduce == "ipc":
            # the peer-mapped all-reduce fused into head_fwd, one rank (no peer to wait for)
            ipc = H.C().IpcAllReduce(1, 0, 64 * 1024)
            ipc.open([ipc.handle()])
            ar = ipc_allreduce(ipc)
        else:
            ar = native_allreduce(self_comm())
    tail = TailEngine(ServerTailSisa(), sisa_server_spec(), dev, tp_rank=0, tp_size=a.tp, allreduce=ar)
    slot = OptSlot(adam(1e-3, 1e-5))
    if a.path == "local":
        from splitlearning_amd.data.device_dataset import DeviceShard
        from splitlearning_amd.engine import FrontEngine
        from splitlearning_amd.models import ClientFrontSisa
        x = torch.randint(0, 256, (4096, 784), dtype=torch.uint8)
        y = torch.randint(0, 10, (4096,))
        shard = DeviceShard(x, y, dev)
        front = FrontEngine(ClientFrontSisa(), dev)
        aslot = OptSlot(adam(1e-3, 1e-5))
        order = shard.shuffled_order(torch.Generator().manual_seed(0))
        for i in range(a.steps):
            s = (i * 16) % 4096
            front.local_step(shard, order[s:s + 16], aslot)
    elif a.path == "graph":
        from splitlearning_amd.engine.graphs import GraphedServerSteps
        gs = GraphedServerSteps(tail, slot, 16, 16, 5408)
        # one run() per epoch of n // 16 steps, like SisaSession.server_epoch
        per = n // 16
        reps = max(1, a.steps // per)
        import time
        for i in range(reps):
            if i == reps // 2:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
            gs.run(acts, labels, per)
        torch.cuda.synchronize()
        if a.time:
            dt = time.perf_counter() - t0
            print(f"path=graph tp={a.tp} us_per_step={dt / ((reps - reps // 2) * per) * 1e6:.2f}")
    elif a.path == "native":
        import time
        per = n // 16
        reps = max(1, a.steps // per)
        for i in range(reps):
            if i == reps // 2:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
            tail.lookahead_prologue(acts[:16])
            tail.run_native_epoch(acts, labels, slot, 16, True)
        torch.cuda.synchronize()
        if a.time:
            dt = time.perf_counter() - t0
            print(f"path=native tp={a.tp} us_per_step={dt / ((reps - reps // 2) * per) * 1e6:.2f}")
    else:
        if a.path == "lookahead":
            tail.lookahead_prologue(acts[:16])
        import time
        for i in range(a.steps):
            if i == a.steps // 2:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
            s = (i * 16) % n
            x, y = acts[s:s + 16], labels[s:s + 16]
            if a.path == "lookahead":
                tail.train_fwd_bwd3(x, y, need_dx=False, pre=True)
                s2 = ((i + 1) * 16) % n
                tail.fused_step(slot, x_next=acts[s2:s2 + 16])
            elif a.path == "fused":
                tail.train_fwd_bwd3(x, y, need_dx=False)
                tail.fused_step(slot)
            else:
                out = tail.forward(x, train=True)
                _, d = H.softmax_ce(out, y, 1 / 16)
                tail.backward_dgrad(d, need_dx=False)
                tail.backward_step(slot)
        torch.cuda.synchronize()
        if a.time:
            dt = time.perf_counter() - t0
            print(f"path={a.path} tp={a.tp} us_per_step={dt / (a.steps - a.steps // 2) * 1e6:.2f}")
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
