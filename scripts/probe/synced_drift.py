"""Per-step synced comparison of a persistent server executor with fp32 torch over many steps:
before every step torch is re-synchronised to the executor's weights / moments / step count
(tests/test_hybrid_gpu.py::test_hybrid_step_matches_torch_adam_every_step, but for STEPS steps),
one step runs on both (the executor as a one-step launch, or --launch to run the executor
free in one launch and only compare at the end), and the fc1 first-moment error is reported
per 16-row block whenever it exceeds a tolerance.

    python scripts/probe/synced_drift.py [hybrid|resident|lps] [steps] [n1]
"""
import copy
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_hybrid_gpu import _engine, _ref_forward, _spec, _sync_torch  # noqa: E402

from splitlearning_amd.models.zoo import _MLP  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "hybrid"
STEPS = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
n1 = int(sys.argv[3]) if len(sys.argv) > 3 else 5000
cuda = torch.device("cuda", 0)
B, seed_base, lr = 16, 21, 1e-3
spec = _spec(n1=n1, p=0.5)
g = torch.Generator(device=cuda).manual_seed(5)
acts = torch.rand(B * STEPS, 5408, generator=g, device=cuda) * 20
labels = torch.randint(0, 100, (B * STEPS,), generator=g, device=cuda)
torch.manual_seed(23)
base = _MLP(spec)
te, slot = _engine(base, spec, cuda, seed_base, "#sd")
ref = copy.deepcopy(base).to(cuda)
opt = torch.optim.Adam(ref.parameters(), lr=lr, weight_decay=1e-5)
if kind == "hybrid":
    ex = te._hybrid_executor(slot, B)
elif kind == "resident":
    ex = te._resident_executor(slot, B)
bad_steps = 0
for i in range(STEPS):
    x, y = acts[i * B:(i + 1) * B], labels[i * B:(i + 1) * B]
    _sync_torch(ref, opt, te, slot, i)
    opt.zero_grad()
    lr_ = F.cross_entropy(_ref_forward(ref, x, seed_base, i + 1), y, reduction="none")
    lr_.mean().backward()
    opt.step()
    if kind == "lps":
        lo, _ = te.train_fwd_bwd3(x, y, need_dx=False)
        te.fused_step(slot)
        le = lo
    else:
        le = torch.empty(B, device=cuda)
        fc, t, _ = ex.run(x.contiguous(), y.contiguous(), le, seed_base, te.fwd_count, slot.t)
        te.fwd_count, slot.t = int(fc), int(t)
    p1 = dict(ref.named_parameters())["fc1.weight"]
    m_t = opt.state[p1]["exp_avg"]
    m_e = slot.states["fc1.weight"]["m"]
    scale = m_t.abs().max().item()
    d = (m_e - m_t).abs().reshape(-1, 16, m_t.shape[1]).amax(dim=(1, 2)) if m_t.shape[0] % 16 == 0 else \
        torch.nn.functional.pad((m_e - m_t).abs(), (0, 0, 0, (-m_t.shape[0]) % 16)).reshape(-1, 16, m_t.shape[1]).amax(dim=(1, 2))
    worst = int(torch.argmax(d))
    rel = d[worst].item() / max(scale, 1e-30)
    ld = (le - lr_.detach()).abs().max().item()
    if rel > 1e-2 or ld > 1e-3 or i % 100 == 0:
        print(f"step {i}: fc1 m worst row block {worst} max |d| {d[worst].item():.3g} = {rel:.3g} of max |m| "
              f"({scale:.3g}); loss max |d| {ld:.3g}", flush=True)
        if rel > 1e-2:
            bad_steps += 1
            if bad_steps > 20:
                break
print(f"{kind}: {bad_steps} steps with a row-block m error above 1 % of max |m|")
