"""Diagnose TP-emulation vs TP=1 divergence: per-layer weight diffs after k steps, with the
look-ahead on/off and the wgrad grid form forced."""
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
B = 16
g = torch.Generator().manual_seed(11)
n = B * 3
acts = (torch.rand(n, 5408, generator=g) * 30).to(cuda)
labels = torch.randint(0, 10, (n,), generator=g).to(cuda)
torch.manual_seed(0)
base = ServerTailSisa()
tag = 0
for T in (2,):
    for la in (False, True):
        for grid in (0, 1, 2):
            C.set_variant(2, grid)
            for nsteps in (1, 2, 3):
                tag += 1
                a = acts[:B * nsteps]
                y = labels[:B * nsteps]
                ref = TailEngine(copy.deepcopy(base), sisa_server_spec(), cuda, seed_base=7, ws_tag=f"#r{tag}")
                rs = OptSlot(adam(1e-3, 1e-5))
                if la:
                    ref.lookahead_prologue(a[:B])
                lr_ = ref.run_native_epoch(a.contiguous(), y.contiguous(), rs, B, la, lookahead=la)
                sh = [TailEngine(copy.deepcopy(base), sisa_server_spec(), cuda, tp_rank=r, tp_size=T, allreduce=None,
                                 seed_base=7, ws_tag=f"#e{tag}.{r}") for r in range(T)]
                ss = [OptSlot(adam(1e-3, 1e-5)) for _ in range(T)]
                le = TailEngine.emulate_tp_epoch(sh, ss, a.contiguous(), y.contiguous(), B, lookahead=la)
                torch.cuda.synchronize()
                W1 = torch.cat([s.layers[0].W for s in sh], 0)
                W2 = torch.cat([s.layers[1].W for s in sh], 1)
                W3 = sh[0].layers[2].W
                d = [(W1 - ref.layers[0].W).abs().max().item(), (W2 - ref.layers[1].W).abs().max().item(),
                     (W3 - ref.layers[2].W).abs().max().item(), (le - lr_).abs().max().item()]
                print(f"T={T} la={la} grid={grid} steps={nsteps}: dW1 {d[0]:.3e} dW2 {d[1]:.3e} dW3 {d[2]:.3e} "
                      f"dloss {d[3]:.3e}", flush=True)
C.set_variant(2, 0)
