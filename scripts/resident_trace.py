"""Phase timeline of the register-resident server epoch (csrc/resident.hip, RES_MARK points)
at a TP = 8 shard (1-rank peer-mapped stand-in), one MI355X: wall-clock stamps of workgroup 0
(an fc1 workgroup, a logit-row reducer and an fc2-row owner) and of workgroup G - 1 (fc2 rows
only), mean us per interval over steps 8 .. trace_steps - 1.

    python scripts/resident_trace.py [--tp 8] [--steps 256] [--trace 64]
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

NAMES = ["wait A", "h1 from partials", "fc2 rows", "exchange + h2", "logit partials + arrive B",
         "wait B (reducer)", "softmax-CE + arrive C", "wait C", "dz2 / W3 / b2 / W2 + arrive D", "wait D",
         "dz1 (MFMA) + mask", "b1 / W1 Adam", "x_next + look-ahead + arrive A"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tp", type=int, default=8)
    ap.add_argument("--steps", type=int, default=256)
    ap.add_argument("--trace", type=int, default=64)
    a = ap.parse_args()
    C = H.C()
    dev = torch.device("cuda", 0)
    ops.set_backend("hip")
    B = 16
    torch.manual_seed(0)
    acts = torch.rand(B * a.steps, 5408, device=dev) * 20
    labels = torch.randint(0, 100, (B * a.steps,), device=dev)
    from splitlearning_amd.parallel.rccl import ipc_allreduce
    ipc = C.IpcAllReduce(1, 0, 64 * 1024)
    ipc.open([ipc.handle()])
    tail = TailEngine(ServerTailSisa(), sisa_server_spec(), dev, tp_rank=0, tp_size=a.tp,
                      allreduce=ipc_allreduce(ipc))
    slot = OptSlot(adam(1e-3, 1e-5))
    assert tail.resident_ok(slot, B)
    ex = tail._resident_executor(slot, B)
    khz = ex.clock_khz()
    for rep in range(3):
        tr = torch.zeros(2, a.trace, 16, dtype=torch.long, device=dev)
        loss = torch.empty(B * a.steps, device=dev)
        torch.cuda.synchronize()
        fc, t, _ = ex.run(acts, labels, loss, 0, tail.fwd_count, slot.t, tr)
        tail.fwd_count, slot.t = int(fc), int(t)
        torch.cuda.synchronize()
    tr = tr.cpu().double() * 1000.0 / khz        # us
    for wi, who in ((0, "workgroup 0"), (1, "workgroup G-1")):
        x = tr[wi, 8:]
        step = (x[1:, 0] - x[:-1, 0]).mean().item()
        print(f"== {who}: step {step:.2f} us (stamp 0 to stamp 0)")
        for k in range(13):
            a0, a1 = x[:, k], x[:, k + 1]
            ok = (a0 > 0) & (a1 > 0)
            if ok.any():
                print(f"  {k:2d}->{k + 1:2d} {NAMES[k]:34s} {(a1 - a0)[ok].mean().item():6.2f} us")
        # inside "wait D": the parameter updates (9 -> 14), W2's publication (14 -> 15), the wait (15 -> 10)
        for k0, k1, nm in ((9, 14, "b3 / W3 / b2 / W2 updates"), (14, 15, "W2 publication"),
                           (15, 10, "B4 loads + wait D")):
            a0, a1 = x[:, k0], x[:, k1]
            ok = (a0 > 0) & (a1 > 0)
            if ok.any():
                print(f"  {k0:2d}->{k1:2d} {nm:34s} {(a1 - a0)[ok].mean().item():6.2f} us")
        # fc2-only workgroups: wait D is skipped; stamp 9 -> next step's stamp 0
        nxt = (x[1:, 0] - x[:-1, 9]).mean().item()
        print(f"  9 -> next 0 (rest of step)                {nxt:6.2f} us")


if __name__ == "__main__":
    main()
