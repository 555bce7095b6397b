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


def _eager_step(t, slot, x, y):
    if t.fused3_ok():
        t.train_fwd_bwd3(x, y, need_dx=False)
        t.fused_step(slot)
        return
    out = t.forward(x, train=True)
    _, d = hip_ops.softmax_ce(out, y, 1.0 / x.shape[0])
    t.backward_dgrad(d, need_dx=False)
    t.backward_step(slot)


def test_graph_replay_matches_eager(cuda):
    g = torch.Generator().manual_seed(0)
    n, B, G = 16 * 40, 16, 8
    acts = (torch.rand(n, 5408, generator=g) * 30).to(cuda)
    labels = torch.randint(0, 10, (n,), generator=g).to(cuda)
    # eager (same kernel sequence as the graph: the fused path when available)
    te, se = _tail(cuda), OptSlot(adam(1e-3, 1e-5))
    for s in range(0, n, B):
        _eager_step(te, se, acts[s:s + B], labels[s:s + B])
    # graphed (first 32 steps) + eager tail (8 steps)
    tg, sg = _tail(cuda), OptSlot(adam(1e-3, 1e-5))
    gs = GraphedServerSteps(tg, sg, B, G, 5408)
    gs.run(acts, labels, 32)
    for s in range(32 * B, n, B):
        _eager_step(tg, sg, acts[s:s + B], labels[s:s + B])
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
        _eager_step(te, se, acts[s:s + B], labels[s:s + B])
    tg, sg = mk(), OptSlot(adam(1e-3, 1e-5))
    GraphedServerSteps(tg, sg, B, G, 5408).run(acts, labels, n // B)
    torch.cuda.synchronize()
    for L1, L2 in zip(te.layers, tg.layers):
        assert torch.equal(L1.W, L2.W) and torch.equal(L1.b, L2.b)


@pytest.mark.parametrize("need_dx", [False, True])
@pytest.mark.parametrize("kind", ["adam", "sgd"])
def test_fused_server_step_matches_generic(cuda, need_dx, kind):
    from splitlearning_amd.engine import sgd_momentum
    g = torch.Generator().manual_seed(2)
    B, steps = 16, 4
    acts = (torch.rand(B * steps, 5408, generator=g) * 30).to(cuda)
    labels = torch.randint(0, 10, (B * steps,), generator=g).to(cuda)
    mk_slot = (lambda: OptSlot(adam(1e-3, 1e-5))) if kind == "adam" else (lambda: OptSlot(sgd_momentum(1e-2)))
    ta, sa = _tail(cuda), mk_slot()
    tb, sb = _tail(cuda), mk_slot()
    assert tb.fused3_ok()
    for s in range(0, B * steps, B):
        x, y = acts[s:s + B], labels[s:s + B]
        out = ta.forward(x, train=True)
        loss_a, d = hip_ops.softmax_ce(out, y, 1.0 / B)
        dxa = ta.backward_dgrad(d, need_dx=need_dx)
        ta.backward_step(sa)
        loss_b, dxb = tb.train_fwd_bwd3(x, y, need_dx=need_dx)
        tb.fused_step(sb)
        torch.testing.assert_close(loss_b, loss_a, rtol=1e-4, atol=1e-5)
        if need_dx:
            torch.testing.assert_close(dxb, dxa, rtol=1e-3, atol=1e-5)
    torch.cuda.synchronize()
    for L1, L2 in zip(ta.layers, tb.layers):
        if kind == "sgd":   # plain SGD: parameter error = lr * gradient rounding difference
            torch.testing.assert_close(L1.W, L2.W, rtol=1e-4, atol=1e-4)
            continue
        d = (L1.W - L2.W).abs()   # Adam: rounding noise on ~zero gradients moves by up to lr
        assert d.max().item() < 1e-2 and (d > 1e-5).float().mean().item() < 1e-4
