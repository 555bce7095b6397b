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


def test_native_rccl_allreduce_is_capturable(cuda):
    from splitlearning_amd.parallel.rccl import self_comm
    tpc = self_comm()
    assert tpc.size == 1 and tpc.rank == 0
    x = torch.arange(16., device=cuda)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            y = x * 2
            tpc.allreduce_sum(y)
            z = y + 1
    torch.cuda.current_stream().wait_stream(s)
    x.fill_(3.0)
    g.replay()
    torch.cuda.synchronize()
    assert torch.all(z == 7)


def test_graphed_tp_tail_with_native_allreduce(cuda):
    """A column/row-sharded tail (TP plumbing) captured with the native all-reduce
    in the graph: replay equals the same sharded tail run eagerly."""
    from splitlearning_amd.parallel.rccl import native_allreduce, self_comm
    ar = native_allreduce(self_comm())
    g = torch.Generator().manual_seed(1)
    n, B, G = 16 * 16, 16, 8
    acts = (torch.rand(n, 5408, generator=g) * 30).to(cuda)
    labels = torch.randint(0, 10, (n,), generator=g).to(cuda)

    def mk():
        torch.manual_seed(0)
        return TailEngine(ServerTailSisa(), sisa_server_spec(), cuda, tp_rank=0, tp_size=2, allreduce=ar,
                          seed_base=5)
    te, se = mk(), OptSlot(adam(1e-3, 1e-5))
    for s in range(0, n, B):
        out = te.forward(acts[s:s + B], train=True)
        _, d = hip_ops.softmax_ce(out, labels[s:s + B], 1.0 / B)
        te.backward_dgrad(d, need_dx=False)
        te.backward_step(se)
    tg, sg = mk(), OptSlot(adam(1e-3, 1e-5))
    GraphedServerSteps(tg, sg, B, G, 5408).run(acts, labels, n // B)
    torch.cuda.synchronize()
    for L1, L2 in zip(te.layers, tg.layers):
        assert torch.equal(L1.W, L2.W) and torch.equal(L1.b, L2.b)
