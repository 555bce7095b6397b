"""Vanilla persistent epoch: run STEPS steps as one launch from a fixed init and save every
parameter / momentum tensor (compare variants of csrc/vanilla.hip bitwise with va_state_cmp.py).

    python scripts/probe/va_state_dump.py OUT.pt [steps]
"""
import os
import sys
import tempfile
from pathlib import Path

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
# the tests' session helpers (a variant tree of scripts/ab_variants.py has no tests/: the main tree's)
sys.path.insert(1, os.path.join(os.environ.get("GRAFT_REPO_ROOT", ROOT), "tests"))
sys.path.insert(1, os.path.join(ROOT, "tests"))
from test_split_native_gpu import _session, _states  # noqa: E402

dev = torch.device("cuda", 0)
out = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
B = 16
s = _session("vanilla", Path(tempfile.mkdtemp()), True, dev, B, persist=True)
tr = s.alices[1].train
reps = -(-(steps * B) // len(tr.y))
order = torch.cat([tr.shuffled_order(torch.Generator().manual_seed(40 + r)) for r in range(reps)])[:steps * B].to(dev)
s.split_epoch(1, order, order.numel())
torch.cuda.synchronize()
assert s.native_split_epochs.get("persistent") == 1, s.__dict__.get("split_persist_reason")
torch.save({k: v.detach().cpu() for k, v in _states(s, "vanilla").items()}, out)
print(f"saved {out}: {steps} steps")
