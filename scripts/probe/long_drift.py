"""Where do a long persistent server epoch and the launch-per-stage executor part ways?  Runs
STEPS steps of model2_sisa (fc1 N1 wide) on the hybrid / resident executor, on launch-per-stage,
on launch-per-stage with one-ulp-perturbed inputs, and in fp32 torch (Adam wd 1e-5, the same
dropout masks), then prints every tensor's relative L2 distance to torch and the spatial
pattern (16 x 256 fc1 tiles) of the fc1 first-moment gap.

    python scripts/probe/long_drift.py [hybrid|resident] [steps] [n1]
"""
import copy
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_hybrid_gpu import _engine, _ref_forward, _spec  # noqa: E402
from test_long_launch_gpu import _rel, _tail_states, _ulp  # noqa: E402

from splitlearning_amd.engine.resident import _launch_per_stage_epoch  # noqa: E402
from splitlearning_amd.models.zoo import _MLP  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "hybrid"
STEPS = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
n1 = int(sys.argv[3]) if len(sys.argv) > 3 else (5000 if kind == "hybrid" else 628)
cuda = torch.device("cuda", 0)
B, seed_base = 16, 21
spec = _spec(n1=n1, p=0.5)
g = torch.Generator(device=cuda).manual_seed(5)
acts = torch.rand(B * STEPS, 5408, generator=g, device=cuda) * 20
labels = torch.randint(0, 100, (B * STEPS,), generator=g, device=cuda)
torch.manual_seed(23)
base = _MLP(spec)
pe, s1 = _engine(base, spec, cuda, seed_base, "#d1")
lp, s3 = _engine(base, spec, cuda, seed_base, "#d3")
ct, s4 = _engine(base, spec, cuda, seed_base, "#d4")
(pe.run_resident_epoch if kind == "resident" else pe.run_hybrid_epoch)(acts, labels, s1, B)
_launch_per_stage_epoch(lp, s3, acts, labels, B)
_launch_per_stage_epoch(ct, s4, _ulp(acts), labels, B)
ref = copy.deepcopy(base).to(cuda)
opt = torch.optim.Adam(ref.parameters(), lr=1e-3, weight_decay=1e-5)
for i in range(STEPS):
    opt.zero_grad()
    F.cross_entropy(_ref_forward(ref, acts[i * B:(i + 1) * B], seed_base, i + 1), labels[i * B:(i + 1) * B]).backward()
    opt.step()
torch.cuda.synchronize()
tr = {}
for name, p in ref.named_parameters():
    ln = name.split(".")[0]
    nm = f"{ln}.{'W' if name.endswith('weight') else 'b'}"
    tr[nm] = p.detach()
    tr[f"{ln}.{name.split('.')[1]}.m"] = opt.state[p]["exp_avg"]
    tr[f"{ln}.{name.split('.')[1]}.v"] = opt.state[p]["exp_avg_sq"]
a, c, d = _tail_states(pe, s1), _tail_states(lp, s3), _tail_states(ct, s4)
print(f"{kind}, {STEPS} steps, fc1 {n1} rows: relative L2 distance to fp32 torch")
print(f"{'tensor':22s} {kind:>10s} {'lps':>10s} {'lps-ulp':>10s} {kind + '-lps':>12s}")
for k in sorted(tr):
    print(f"{k:22s} {_rel(a[k], tr[k]):10.3g} {_rel(c[k], tr[k]):10.3g} {_rel(d[k], tr[k]):10.3g} {_rel(a[k], c[k]):12.3g}")
m_p, m_l = a["fc1.weight.m"], c["fc1.weight.m"]
N, K = m_p.shape
nb, kb = (N + 15) // 16, (K + 255) // 256
dm = torch.zeros(nb, kb, device=cuda)
for r in range(nb):
    for q in range(kb):
        x, y = m_p[16 * r:16 * r + 16, 256 * q:256 * q + 256], m_l[16 * r:16 * r + 16, 256 * q:256 * q + 256]
        dm[r, q] = (x - y).norm() / y.norm().clamp_min(1e-30)
print(f"fc1 m tile gaps ({nb} x {kb} tiles of 16 x 256): median {dm.median().item():.3g}, max {dm.max().item():.3g}")
top = torch.topk(dm.reshape(-1), 12)
print("worst tiles (row block, column block, gap):", [(int(i) // kb, int(i) % kb, round(v.item(), 3)) for v, i in zip(top.values, top.indices)])
print("per column block median gap:", [round(v, 3) for v in dm.median(0).values.tolist()])
big = (m_p - m_l).abs()
i = int(torch.argmax(big))
print(f"largest element gap at ({i // K}, {i % K}): {kind} {m_p.reshape(-1)[i].item():.4g} lps {m_l.reshape(-1)[i].item():.4g} "
      f"torch {tr['fc1.weight.m'].reshape(-1)[i].item():.4g}")
