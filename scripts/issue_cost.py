"""Host (CPU) cost of issuing Bob's server steps: Python look-ahead loop vs the native
executor (_C.ServerEpoch).  Times the host call that enqueues one epoch of 64 steps, with
the GPU first blocked behind a long spin so the launch queue never throttles the host.

    python scripts/issue_cost.py [--tp 8]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from splitlearning_amd import ops  # noqa: E402
from splitlearning_amd.engine import OptSlot, TailEngine, adam  # noqa: E402
from splitlearning_amd.models import ServerTailSisa, sisa_server_spec  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tp", type=int, default=8)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ops.set_backend("hip")
    n = 16 * 64
    acts = torch.rand(n, 5408, device=dev) * 20
    labels = torch.randint(0, 10, (n,), device=dev)
    ar = None
    if a.tp > 1:
        from splitlearning_amd.parallel.rccl import native_allreduce, self_comm
        ar = native_allreduce(self_comm())
    tail = TailEngine(ServerTailSisa(), sisa_server_spec(), dev, tp_rank=0, tp_size=a.tp, allreduce=ar)
    slot = OptSlot(adam(1e-3, 1e-5))

    def python_epoch():
        tail.lookahead_prologue(acts[:16])
        pre = True
        for s in range(0, n, 16):
            nxt = acts[s + 16:s + 32] if s + 32 <= n else None
            tail.train_fwd_bwd3(acts[s:s + 16], labels[s:s + 16], need_dx=False, pre=pre)
            tail.fused_step(slot, x_next=nxt)
            pre = nxt is not None

    def native_epoch():
        tail.lookahead_prologue(acts[:16])
        tail.run_native_epoch(acts, labels, slot, 16, True)

    for name, fn in (("python", python_epoch), ("native", native_epoch)) * 2:
        fn()
        torch.cuda.synchronize()
        torch.cuda._sleep(200_000_000)      # keep the GPU busy so the host never waits on the queue
        t0 = time.perf_counter()
        fn()
        dt = time.perf_counter() - t0
        torch.cuda.synchronize()
        print(f"tp={a.tp} {name}: host issue {dt / 64 * 1e6:.1f} us per step", flush=True)


if __name__ == "__main__":
    main()
