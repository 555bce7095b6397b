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


def _eager_epoch(t, slot, acts, labels, B, s0=0, pre=None):
    """SisaSession.server_epoch's eager loop (fused path + fc1 look-ahead chain)."""
    n = labels.numel()
    la = t.lookahead_ok(B)
    if pre is None:
        pre = False
        if la and s0 + B <= n:
            t.lookahead_prologue(acts[s0:s0 + B])
            pre = True
    for s in range(s0, n, B):
        x, y = acts[s:s + B], labels[s:s + B]
        nxt = acts[s + B:s + 2 * B] if la and s + 2 * B <= n else None
        t.train_fwd_bwd3(x, y, need_dx=False, pre=pre)
        t.fused_step(slot, x_next=nxt)
        pre = nxt is not None


def test_graph_replay_matches_eager(cuda):
    g = torch.Generator().manual_seed(0)
    n, B, G = 16 * 40 + 5, 16, 8
    acts = (torch.rand(n, 5408, generator=g) * 30).to(cuda)
    labels = torch.randint(0, 10, (n,), generator=g).to(cuda)
    # eager (same kernel sequence as the graph: the fused path + look-ahead chain)
    te, se = _tail(cuda), OptSlot(adam(1e-3, 1e-5))
    _eager_epoch(te, se, acts, labels, B)
    # graphed (first 32 steps) + eager tail (8 full steps + a 5-row batch)
    tg, sg = _tail(cuda), OptSlot(adam(1e-3, 1e-5))
    gs = GraphedServerSteps(tg, sg, B, G, 5408)
    pre = gs.run(acts, labels, 32)
    assert pre
    _eager_epoch(tg, sg, acts, labels, B, s0=32 * B, pre=pre)
    torch.cuda.synchronize()
    assert sg.t == se.t == 41 and tg.fwd_count == te.fwd_count
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
    _eager_epoch(te, se, acts, labels, B)
    tg, sg = mk(), OptSlot(adam(1e-3, 1e-5))
    GraphedServerSteps(tg, sg, B, G, 5408).run(acts, labels, n // B)
    torch.cuda.synchronize()
    for L1, L2 in zip(te.layers, tg.layers):
        assert torch.equal(L1.W, L2.W) and torch.equal(L1.b, L2.b)


@pytest.mark.parametrize("tp", [1, 8])
@pytest.mark.parametrize("need_dx", [False, True])
@pytest.mark.parametrize("kind", ["adam", "sgd"])
def test_fused_server_step_matches_generic(cuda, need_dx, kind, tp):
    """Fused 3-layer step == the generic per-layer step; tp=8 runs rank 0's shard of a
    tensor-parallel tail (1-rank all-reduce): the row-parallel fc2 takes its unsplit path."""
    from splitlearning_amd.engine import sgd_momentum
    g = torch.Generator().manual_seed(2)
    B, steps = 16, 4
    acts = (torch.rand(B * steps, 5408, generator=g) * 30).to(cuda)
    labels = torch.randint(0, 10, (B * steps,), generator=g).to(cuda)
    mk_slot = (lambda: OptSlot(adam(1e-3, 1e-5))) if kind == "adam" else (lambda: OptSlot(sgd_momentum(1e-2)))
    if tp == 1:
        mk = lambda: _tail(cuda)  # noqa: E731
    else:
        from splitlearning_amd.parallel.rccl import native_allreduce, self_comm
        ar = native_allreduce(self_comm())

        def mk():
            torch.manual_seed(0)
            return TailEngine(ServerTailSisa(), sisa_server_spec(), cuda, tp_rank=0, tp_size=tp, allreduce=ar,
                              seed_base=42)
    ta, sa = mk(), mk_slot()
    tb, sb = mk(), mk_slot()
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
            torch.testing.assert_close(dxb, dxa, rtol=1e-3, atol=2e-4)
        torch.cuda.synchronize()
        for L1, L2 in zip(ta.layers, tb.layers):
            # one step from the same state: summation-order rounding only, except rare
            # elements (Adam: a ~zero gradient's sign is noise, a move of up to lr; SGD-m: a
            # hidden unit on the ReLU boundary flips in one path)
            dw = (L1.W - L2.W).abs()
            assert dw.max().item() < 2e-2 and (dw > 1e-5).float().mean().item() < 1e-4
        _resync(ta, sa, tb, sb)      # free-running fp32 trajectories of this training are chaotic


def _resync(src, src_slot, dst, dst_slot):
    """dst := src (weights, biases, optimizer moments, step count)."""
    with torch.no_grad():
        for La, Lb in zip(src.layers, dst.layers):
            Lb.W.copy_(La.W)
            Lb.b.copy_(La.b)
        for name, st in src_slot.states.items():
            for k, v in st.items():
                dst_slot.states[name][k].copy_(v)
    dst_slot.t = src_slot.t


def test_lookahead_matches_plain_fused(cuda):
    """The fc1 look-ahead (next batch's product formed inside the wgrad+Adam kernel) only
    changes fc1's summation order: same trajectory as the plain fused steps."""
    g = torch.Generator().manual_seed(3)
    B, steps = 16, 6
    acts = (torch.rand(B * steps, 5408, generator=g) * 30).to(cuda)
    labels = torch.randint(0, 10, (B * steps,), generator=g).to(cuda)
    ta, sa = _tail(cuda), OptSlot(adam(1e-3, 1e-5))
    tb, sb = _tail(cuda), OptSlot(adam(1e-3, 1e-5))
    assert tb.lookahead_ok(B)
    for s in range(0, B * steps, B):
        ta.train_fwd_bwd3(acts[s:s + B], labels[s:s + B], need_dx=False)
        ta.fused_step(sa)
    _eager_epoch(tb, sb, acts, labels, B)
    torch.cuda.synchronize()
    for L1, L2 in zip(ta.layers, tb.layers):
        d = (L1.W - L2.W).abs()
        assert d.max().item() < 1e-2 and (d > 1e-4).float().mean().item() < 1e-4


def test_wgrad_group_lookahead_kernel(cuda):
    """pn slabs summed == x_next @ W1_new^T with W1_new the weights after the update."""
    from splitlearning_amd.engine import sgd_momentum
    g = torch.Generator().manual_seed(4)
    M, N, K, mn = 16, 300, 1000, 11
    A = torch.randn(M, K, generator=g).to(cuda)
    dz = torch.randn(M, N, generator=g).to(cuda)
    W = torch.randn(N, K, generator=g).to(cuda)
    b = torch.randn(N, generator=g).to(cuda)
    xn = torch.randn(mn, K, generator=g).to(cuda)
    slot = OptSlot(sgd_momentum(1e-2))
    sw, sbias = slot.state("w", W), slot.state("b", b)
    pn = hip_ops.lookahead_slabs(cuda, K, mn, N)
    Wref = W.clone()
    hip_ops.wgrad_group_([(dz, A, W, sw, b, sbias)], M, slot.cfg, slot.tick(), x_next=xn, p_next=pn)
    torch.cuda.synchronize()
    W_new = Wref - 1e-2 * (dz.t() @ A)          # first SGD-momentum step: buf = g
    torch.testing.assert_close(W, W_new, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(pn.sum(0), xn @ W.t(), rtol=1e-4, atol=1e-3)


def _vanilla_session(cuda, tmp_path):
    from splitlearning_amd.config import parse_args
    from splitlearning_amd.data.mnist import write_shards
    from splitlearning_amd.parallel.dist import Comm, Placement
    from splitlearning_amd.protocols import VanillaSession
    args = parse_args(["--vanilla", "--world_size", "2", "--seed", "5", "--num_samples", "1500", "--no_tqdm",
                       "--datapath", str(tmp_path / "d"), "--log_dir", str(tmp_path / "logs")])
    if not (tmp_path / "d").exists():
        write_shards(args, verbose=False)
    comm = Comm(0, 1, cuda, Placement.make(2, 1, 1))
    return VanillaSession(args, comm, cuda)


@pytest.mark.parametrize("ahead", [True, False])
def test_vanilla_pipelined_epoch_matches_per_batch_steps(cuda, tmp_path, ahead):
    """split_epoch (Alice's next forward before Bob's update, fc1 look-ahead in Bob's
    wgrad kernel; or, ahead=False, the overlap order used when no Bob shard shares the
    Alice's GPU) follows the same trajectory as one split_step per batch."""
    sa = _vanilla_session(cuda, tmp_path)
    sb = _vanilla_session(cuda, tmp_path)
    sb.split_lookahead = lambda cid: ahead
    assert sb.tail.lookahead_ok(16)
    a = sa.alices[1]
    order = a.train.shuffled_order(torch.Generator().manual_seed(9))[:16 * 6 + 5]   # a partial last batch
    n = order.numel()
    for s in range(0, n, 16):
        sa.split_step(1, order[s:s + 16], min(16, n - s))
    sb.split_epoch(1, order, n)
    torch.cuda.synchronize()
    for L1, L2 in zip(sa.tail.layers, sb.tail.layers):
        d = (L1.W - L2.W).abs()
        assert d.max().item() < 1e-2 and (d > 1e-4).float().mean().item() < 1e-4
    wa = sa.alices[1].front.module.state_dict()
    wb = sb.alices[1].front.module.state_dict()
    for k in wa:
        torch.testing.assert_close(wa[k], wb[k], rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("ahead", [True, False])
def test_ushape_pipelined_epoch_matches_per_batch_steps(cuda, tmp_path, ahead):
    """U-shape split_epoch (grouped Bob step with the fc1 look-ahead, or the overlap order)
    == per-batch split_step."""
    from splitlearning_amd.config import parse_args
    from splitlearning_amd.data.mnist import write_shards
    from splitlearning_amd.parallel.dist import Comm, Placement
    from splitlearning_amd.protocols import UShapeSession
    args = parse_args(["--world_size", "2", "--seed", "6", "--num_samples", "1500", "--no_tqdm",
                       "--datapath", str(tmp_path / "d"), "--log_dir", str(tmp_path / "logs")])
    write_shards(args, verbose=False)
    mk = lambda: UShapeSession(args, Comm(0, 1, cuda, Placement.make(2, 1, 1)), cuda)  # noqa: E731
    sa, sb = mk(), mk()
    sb.split_lookahead = lambda cid: ahead
    assert sb.tail.grouped_ok(16)
    order = sa.alices[1].train.shuffled_order(torch.Generator().manual_seed(3))[:16 * 6 + 7]
    n = order.numel()
    for s in range(0, n, 16):
        sa.split_step(1, order[s:s + 16], min(16, n - s))
    sb.split_epoch(1, order, n)
    torch.cuda.synchronize()
    for L1, L2 in zip(sa.tail.layers, sb.tail.layers):
        d = (L1.W - L2.W).abs()
        assert d.max().item() < 1e-2 and (d > 1e-4).float().mean().item() < 1e-4
    for ma, mb in ((sa.alices[1].front.module, sb.alices[1].front.module),
                   (sa.alices[1].head.module, sb.alices[1].head.module)):
        for (k, va), vb in zip(ma.state_dict().items(), mb.state_dict().values()):
            torch.testing.assert_close(va, vb, rtol=1e-3, atol=1e-4, msg=k)


@pytest.mark.parametrize("tp", [1, 8])
@pytest.mark.parametrize("kind", ["adam", "sgd"])
@pytest.mark.parametrize("B", [16, 64])
def test_native_server_epoch_matches_python(cuda, tp, kind, B):
    """_C.ServerEpoch (csrc/engine.cpp) issues the same launches, seeds and step counts as the
    Python look-ahead loop: bit-identical weights, optimizer state and losses (tp = 8: rank
    0's shard, row-parallel fc2 through the native 1-rank communicator)."""
    from splitlearning_amd.engine import sgd_momentum
    from splitlearning_amd.parallel.rccl import native_allreduce, self_comm
    g = torch.Generator().manual_seed(8)
    n = B * 9 + 5                                       # full batches + a partial last one
    acts = (torch.rand(n, 5408, generator=g) * 30).to(cuda)
    labels = torch.randint(0, 10, (n,), generator=g).to(cuda)
    ar = native_allreduce(self_comm()) if tp > 1 else None
    mk_slot = (lambda: OptSlot(adam(1e-3, 1e-5))) if kind == "adam" else (lambda: OptSlot(sgd_momentum(1e-2)))

    def mk():
        torch.manual_seed(0)
        return TailEngine(ServerTailSisa(), sisa_server_spec(), cuda, tp_rank=0, tp_size=tp, allreduce=ar,
                          seed_base=1234567)
    ta, sa = mk(), mk_slot()
    tb, sb = mk(), mk_slot()
    assert tb.native_epoch_ok(B)
    losses = []
    ta.lookahead_prologue(acts[:B])
    pre = True
    for s in range(0, n, B):
        nxt = acts[s + B:s + 2 * B] if s + 2 * B <= n else None
        loss, _ = ta.train_fwd_bwd3(acts[s:s + B], labels[s:s + B], need_dx=False, pre=pre)
        losses.append(loss)
        ta.fused_step(sa, x_next=nxt)
        pre = nxt is not None
    tb.lookahead_prologue(acts[:B])
    loss_b = tb.run_native_epoch(acts, labels, sb, B, True)
    torch.cuda.synchronize()
    assert torch.equal(torch.cat(losses), loss_b)
    assert (ta.fwd_count, sa.t) == (tb.fwd_count, sb.t)
    for L1, L2 in zip(ta.layers, tb.layers):
        assert torch.equal(L1.W, L2.W) and torch.equal(L1.b, L2.b)
    for name, st in sa.states.items():
        for k, v in st.items():
            assert torch.equal(v, sb.states[name][k]), (name, k)


def test_concat_pipelined_epoch_matches_per_step(cuda, tmp_path):
    """ConcatSession.concat_epoch (epoch-wide layout, grouped step + fc1 look-ahead) ==
    one concat_step per t, with clients of different sizes (exhausted / partial batches)."""
    from splitlearning_amd.config import parse_args
    from splitlearning_amd.parallel.dist import Comm, Placement
    from splitlearning_amd.protocols import ConcatSession

    class S(ConcatSession):
        def _load_client_shard(self, cid):
            from splitlearning_amd.data.mnist import synthetic_mnist
            n = 90 + 37 * cid
            x, y = synthetic_mnist(n + 20, seed=cid)
            return ({"x": torch.from_numpy(x[:n]), "y": torch.from_numpy(y[:n])},
                    {"x": torch.from_numpy(x[n:]), "y": torch.from_numpy(y[n:])})
    args = parse_args(["--sisa", "--concat", "--world_size", "3", "--seed", "4", "--no_tqdm",
                       "--log_dir", str(tmp_path / "logs")])
    mk = lambda: S(args, Comm(0, 1, cuda, Placement.make(3, 1, 1)), cuda)  # noqa: E731
    sa, sb = mk(), mk()
    caches = [sa.get_activation_and_labels(c) for c in (1, 2)]
    caches_b = [sb.get_activation_and_labels(c) for c in (1, 2)]
    for (a1, l1), (a2, l2) in zip(caches, caches_b):
        assert torch.equal(a1, a2) and torch.equal(l1, l2)
    T = max(-(-c[1].numel() // sa.B) for c in caches)
    na = sum(sa.concat_step(caches, t) for t in range(T))
    nb = sb.concat_epoch(caches_b)
    torch.cuda.synchronize()
    assert na == nb == sum(c[1].numel() for c in caches)
    for L1, L2 in zip(sa.tail.layers, sb.tail.layers):
        d = (L1.W - L2.W).abs()
        assert d.max().item() < 1e-2 and (d > 1e-4).float().mean().item() < 1e-4


