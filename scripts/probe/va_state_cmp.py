"""Compare saved vanilla states bitwise (scripts/probe/va_state_dump.py): first file = reference."""
import sys

import torch

ref = torch.load(sys.argv[1], weights_only=True)
for f in sys.argv[2:]:
    st = torch.load(f, weights_only=True)
    same = [k for k in ref if torch.equal(ref[k], st[k])]
    worst = max(((ref[k] - st[k]).abs().max().item(), k) for k in ref)
    print(f"{f} vs {sys.argv[1]}: {len(same)} of {len(ref)} tensors bitwise equal; max |d| {worst[0]:.3g} ({worst[1]})")
