"""HIP-graph replay of Bob's server steps is bit-identical to the eager step sequence."""
import pytest
import torch

from splitlearning_amd.engine import OptSlot, TailEngine, adam
from splitlearning_amd.engine.graphs import GraphedServerSteps
from splitlearning_amd.models import ServerTailSisa, sisa_server_spec
from splitlearning_amd.ops import hip_ops

pytestmark = pytest.mark.gpu


def _tail(dev):
    torch.manual_seed(0)
    return TailEngine(ServerTailSisa(), sisa_server_spec(), dev, seed_base=42)


def test_graph_replay_matches_eager(cuda):
    g = torch.Generator().manual_seed(0)
    n, B, G = 16 * 40, 16, 8
    acts = (torch.rand(n, 5408, generator=g) * 30).to(cuda)
    labels = torch.randint(0, 10, (n,), generator=g).to(cuda)
    # eager
    te, se = _tail(cuda), OptSlot(adam(1e-3, 1e-5))
    for s in range(0, n, B):
        out = te.forward(acts[s:s + B], train=True)
        _, d = hip_ops.softmax_ce(out, labels[s:s + B], 1.0 / B)
        te.backward_dgrad(d, need_dx=False)
        te.backward_step(se)
    # graphed (first 32 steps) + eager tail (8 steps)
    tg, sg = _tail(cuda), OptSlot(adam(1e-3, 1e-5))
    gs = GraphedServerSteps(tg, sg, B, G, 5408)
    gs.run(acts, labels, 32)
    for s in range(32 * B, n, B):
        out = tg.forward(acts[s:s + B], train=True)
        _, d = hip_ops.softmax_ce(out, labels[s:s + B], 1.0 / B)
        tg.backward_dgrad(d, need_dx=False)
        tg.backward_step(sg)
    torch.cuda.synchronize()
    assert sg.t == se.t == 40 and tg.fwd_count == te.fwd_count
    for L1, L2 in zip(te.layers, tg.layers):
        assert torch.equal(L1.W, L2.W) and torch.equal(L1.b, L2.b)
