"""Determinism / accuracy probe of the vanilla persistent epoch: two identical sessions run the
same persistent epochs (must be bitwise equal), and a per-batch session gives the reference
(max |diff| / max |ref| per tensor)."""
import os
import sys
import tempfile

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
from test_split_native_gpu import _session, _states  # noqa: E402

from pathlib import Path  # noqa: E402

dev = torch.device("cuda", 0)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
tmp = Path(tempfile.mkdtemp())
sq1 = _session("vanilla", tmp, True, dev, B, persist=True)
sq2 = _session("vanilla", tmp, True, dev, B, persist=True)
sp = _session("vanilla", tmp, True, dev, B)
order = sp.alices[1].train.shuffled_order(torch.Generator().manual_seed(4))[:B * 6 + 3].to(dev)
for e in range(3):
    for s in (sq1, sq2, sp):
        s.split_epoch(1, order, order.numel())
    torch.cuda.synchronize()
    a, b, c = _states(sq1, "vanilla"), _states(sq2, "vanilla"), _states(sp, "vanilla")
    print(f"epoch {e}: persistent counts {sq1.native_split_epochs}")
    for k in a:
        same = torch.equal(a[k], b[k])
        d = (a[k] - c[k]).abs().max().item() / max(c[k].abs().max().item(), 1e-12)
        d12 = (a[k] - b[k]).abs().max().item()
        print(f"  {k:28s} bitwise-repeat {same!s:5s} (max diff {d12:.3e})  rel diff vs per-batch {d:.3e}")
