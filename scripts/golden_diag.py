"""Engine vs torch divergence diagnostics (SISA Adam server steps; vanilla split SGD epoch)."""
import copy
import os
import sys
import torch
import torch.nn.functional as F
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from splitlearning_amd.engine import OptSlot, TailEngine, adam  # noqa
from splitlearning_amd.models import ServerTailSisa, sisa_server_spec  # noqa
from splitlearning_amd.ops import rng, hip_ops  # noqa

cuda = torch.device("cuda", 0)


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


def stats(a, b):
    d = (a - b).abs()
    return f"max {d.max().item():.2e} f>1e-6 {(d > 1e-6).float().mean().item():.2e} f>1e-4 {(d > 1e-4).float().mean().item():.2e}"


B, lr, sb = 16, 1e-3, 99
for scale in (1.0, 30.0):
    g = torch.Generator().manual_seed(21)
    acts = (torch.rand(B * 4, 5408, generator=g) * scale).to(cuda)
    labels = torch.randint(0, 10, (B * 4,), generator=g).to(cuda)
    torch.manual_seed(4)
    base = ServerTailSisa()
    for nsteps in (1, 2, 3):
        ref = copy.deepcopy(base).to(cuda)
        opt = torch.optim.Adam(ref.parameters(), lr=lr, weight_decay=1e-5)
        te = TailEngine(copy.deepcopy(base), sisa_server_spec(), cuda, seed_base=sb, ws_tag=f"#{scale}{nsteps}")
        slot = OptSlot(adam(lr, 1e-5))
        a = acts[:B * nsteps].contiguous()
        y = labels[:B * nsteps].contiguous()
        te.lookahead_prologue(a[:B])
        le = te.run_native_epoch(a, y, slot, B, True)
        grads = None
        for i in range(nsteps):
            opt.zero_grad()
            loss = F.cross_entropy(ref_fwd(ref, a[i * B:(i + 1) * B], sb, i + 1), y[i * B:(i + 1) * B])
            loss.backward()
            if i == 0:
                grads = {k: p.grad.clone() for k, p in ref.named_parameters()}
            opt.step()
        torch.cuda.synchronize()
        sd = te.module.state_dict()
        print(f"scale {scale} steps {nsteps}:")
        for k, v in ref.state_dict().items():
            print(f"   {k:12s} {stats(sd[k], v)}")
        if nsteps == 1:
            for k, gr in grads.items():
                print(f"   |grad| {k:12s} median {gr.abs().median().item():.2e} frac<1e-7 {(gr.abs() < 1e-7).float().mean().item():.2e} "
                      f"frac==0 {(gr == 0).float().mean().item():.2e}")
