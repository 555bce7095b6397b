"""Learnable-label trajectories: engine vs torch vs engine-alt (other dgrad order), SISA Adam
128 steps; and the vanilla split epoch vs composed torch SGD: per-step/window stats."""
import copy
import os
import sys
import tempfile
import torch
import torch.nn.functional as F
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splitlearning_amd.engine import OptSlot, TailEngine, adam  # noqa
from splitlearning_amd.models import ServerTailSisa, sisa_server_spec  # noqa
from splitlearning_amd.ops import rng, hip_ops  # noqa

cuda = torch.device("cuda", 0)
C = hip_ops.C()


def ref_fwd(mod, x, seed_base, step):
    h = x
    for i, lin in enumerate(mod.linears()):
        ls = mod.spec.layers[i]
        h = F.linear(h, lin.weight, lin.bias)
        if ls.relu:
            h = F.relu(h)
        if ls.dropout:
            keep = rng.keep_mask(rng.step_seed(seed_base, i, step), h.shape[0], h.shape[1], ls.dropout, device=h.device)
            h = h * keep / (1 - ls.dropout)
    return h


B, steps, lr, sb = 16, 128, 1e-3, 99
for scale in (1.0, 30.0):
    for learn in (False, True):
        g = torch.Generator().manual_seed(21)
        n = B * steps
        acts = (torch.rand(n, 5408, generator=g) * scale).to(cuda)
        if learn:
            P = torch.randn(5408, 10, generator=g).to(cuda)
            labels = ((acts - acts.mean(0)) @ P).argmax(1)
        else:
            labels = torch.randint(0, 10, (n,), generator=g).to(cuda)
        torch.manual_seed(4)
        base = ServerTailSisa()
        ref = copy.deepcopy(base).to(cuda)
        w0 = {k: v.clone() for k, v in ref.state_dict().items()}
        opt = torch.optim.Adam(ref.parameters(), lr=lr, weight_decay=1e-5)

        def engine(variant, tag):
            C.set_variant(8, variant)
            te = TailEngine(copy.deepcopy(base), sisa_server_spec(), cuda, seed_base=sb, ws_tag=tag)
            slot = OptSlot(adam(lr, 1e-5))
            te.lookahead_prologue(acts[:B])
            l = te.run_native_epoch(acts, labels, slot, B, True)
            C.set_variant(8, 0)
            return te, l
        te, le = engine(0, f"#e{scale}{learn}")
        ta, la = engine(2, f"#a{scale}{learn}")
        lr_ = []
        for i in range(steps):
            opt.zero_grad()
            loss = F.cross_entropy(ref_fwd(ref, acts[i * B:(i + 1) * B], sb, i + 1), labels[i * B:(i + 1) * B],
                                   reduction="none")
            loss.mean().backward()
            opt.step()
            lr_.append(loss.detach())
        torch.cuda.synchronize()
        lt = torch.cat(lr_)
        win = lambda l: l.view(-1, 16 * B).mean(1)  # noqa: E731  8 windows of 16 steps
        print(f"== scale {scale} learnable {learn}")
        print("   torch windows ", [round(v, 3) for v in win(lt).tolist()])
        print("   engine windows", [round(v, 3) for v in win(le).tolist()])
        print("   alt windows   ", [round(v, 3) for v in win(la).tolist()])
        gap = lambda a, b: [round((a[i * B:(i + 1) * B] - b[i * B:(i + 1) * B]).abs().max().item(), 5) for i in (0, 1, 2, 3, 7, 15, 31, 63, 127)]  # noqa
        print("   gap e-t steps 1,2,3,4,8,16,32,64,128", gap(le, lt))
        print("   gap a-e                          ", gap(la, le))
        sd = te.module.state_dict()
        sa = ta.module.state_dict()
        for k, v in ref.state_dict().items():
            moved = (v - w0[k]).norm().item()
            print(f"   {k:11s} |e-t|/|t-w0| {(sd[k] - v).norm().item() / moved:.3f}  |a-e|/|t-w0| {(sa[k] - sd[k]).norm().item() / moved:.3f}")
