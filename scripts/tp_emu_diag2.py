"""TP-emulation vs TP=1 divergence against a rounding-noise baseline: TP=1 with the other
fc2-dgrad summation order (variant 8 = 1).  Prints per-step loss gaps and weight-diff stats."""
import copy
import sys
import os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splitlearning_amd.engine import OptSlot, TailEngine, adam  # noqa
from splitlearning_amd.models import ServerTailSisa, sisa_server_spec  # noqa
from splitlearning_amd.ops import hip_ops as H  # noqa

cuda = torch.device("cuda", 0)
C = H.C()
B, steps = 16, 72
for scale in (30.0, 1.0):
    g = torch.Generator().manual_seed(11)
    n = B * steps
    acts = (torch.rand(n, 5408, generator=g) * scale).to(cuda)
    labels = torch.randint(0, 10, (n,), generator=g).to(cuda)
    torch.manual_seed(0)
    base = ServerTailSisa()

    def run_ref(variant, tag):
        C.set_variant(8, variant)
        t = TailEngine(copy.deepcopy(base), sisa_server_spec(), cuda, seed_base=7, ws_tag=tag)
        s = OptSlot(adam(1e-3, 1e-5))
        t.lookahead_prologue(acts[:B])
        l = t.run_native_epoch(acts, labels, s, B, True)
        C.set_variant(8, 0)
        return t, l
    ref, lref = run_ref(0, f"#a{scale}")
    alt, lalt = run_ref(1, f"#b{scale}")
    res = {"tp1-alt": (alt, lalt, [l.W for l in alt.layers])}
    for T in (2, 8):
        sh = [TailEngine(copy.deepcopy(base), sisa_server_spec(), cuda, tp_rank=r, tp_size=T, allreduce=None,
                         seed_base=7, ws_tag=f"#e{scale}.{T}.{r}") for r in range(T)]
        ss = [OptSlot(adam(1e-3, 1e-5)) for _ in range(T)]
        le = TailEngine.emulate_tp_epoch(sh, ss, acts, labels, B)
        Ws = [torch.cat([s.layers[0].W for s in sh], 0), torch.cat([s.layers[1].W for s in sh], 1), sh[0].layers[2].W]
        res[f"tp{T}"] = (None, le, Ws)
    torch.cuda.synchronize()
    print(f"== acts scale {scale}: ref loss first/last batch mean {lref[:B].mean().item():.3f} / {lref[-B:].mean().item():.3f}")
    for name, (_, l, Ws) in res.items():
        gaps = [(l[i * B:(i + 1) * B] - lref[i * B:(i + 1) * B]).abs().max().item() for i in range(steps)]
        fr = [((W - R.W).abs() > 1e-4).float().mean().item() for W, R in zip(Ws, ref.layers)]
        mx = [(W - R.W).abs().max().item() for W, R in zip(Ws, ref.layers)]
        print(f"{name:8s} loss gap step1 {gaps[0]:.2e} step8 {gaps[7]:.2e} step32 {gaps[31]:.2e} step72 {gaps[-1]:.2e} "
              f"| frac>1e-4 {fr[0]:.2e} {fr[1]:.2e} {fr[2]:.2e} | max {mx[0]:.2e} {mx[1]:.2e} {mx[2]:.2e}", flush=True)
