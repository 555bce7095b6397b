"""Bitwise check of the look-ahead LDS tile layouts (kernel variant 1 = 0 padded / 1 plain /
2 XOR-swizzled): one native-executor server epoch per layout from the same initial state
must give identical weights and losses (the layout only moves data through LDS)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from splitlearning_amd import ops  # noqa: E402
from splitlearning_amd.engine import OptSlot, TailEngine, adam  # noqa: E402
from splitlearning_amd.models import ServerTailSisa, sisa_server_spec  # noqa: E402
from splitlearning_amd.ops import hip_ops as H  # noqa: E402


def run(variant, tp):
    C = H.C()
    C.set_variant(1, variant)
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    acts = torch.rand(16 * 8, 5408, device=dev) * 20
    labels = torch.randint(0, 10, (16 * 8,), device=dev)
    ar = None
    if tp > 1:
        from splitlearning_amd.parallel.rccl import native_allreduce, self_comm
        ar = native_allreduce(self_comm())
    torch.manual_seed(1)
    tail = TailEngine(ServerTailSisa(), sisa_server_spec(), dev, tp_rank=0, tp_size=tp, allreduce=ar)
    slot = OptSlot(adam(1e-3, 1e-5))
    tail.lookahead_prologue(acts[:16])
    loss = tail.run_native_epoch(acts, labels, slot, 16, True)
    torch.cuda.synchronize()
    C.set_variant(1, 0)
    return [loss.clone()] + [L.W.detach().clone() for L in tail.layers]


ops.set_backend("hip")
for tp in (1, 8):
    ref = run(0, tp)
    for v in (1, 2):
        out = run(v, tp)
        same = all(torch.equal(a, b) for a, b in zip(ref, out))
        print(f"tp={tp} variant1={v} bitwise_equal={same}", flush=True)
        assert same
print("layout check ok")
