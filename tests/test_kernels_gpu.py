"""Numerics of every HIP kernel against the fp32 eager-PyTorch reference of the same op."""
import pytest
import torch

from splitlearning_amd.config import OptimCfg
from splitlearning_amd.ops import hip_ops, torch_ops

pytestmark = pytest.mark.gpu


def _close(a, b, rtol=1e-4, atol=1e-4):
    torch.testing.assert_close(a.float().cpu(), b.float().cpu(), rtol=rtol, atol=atol)


def _shard(n, dev, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randint(0, 256, (n, 784), generator=g, dtype=torch.uint8)
    return x.to(dev)


def _conv_params(dev, seed=1):
    g = torch.Generator().manual_seed(seed)
    w = (torch.rand(32, 1, 3, 3, generator=g) - 0.5) * 0.1
    b = (torch.rand(32, generator=g) - 0.5) * 0.1
    return w.to(dev), b.to(dev)


@pytest.mark.parametrize("B", [1, 7, 16, 300])
def test_conv_fwd(cuda, B):
    x = _shard(1000, cuda)
    idx = torch.randperm(1000, device=cuda)[:B]
    w, b = _conv_params(cuda)
    y, am = hip_ops.conv_front_fwd(x, idx, w, b)
    yr, amr = torch_ops.conv_front_fwd(x, idx, w, b)
    _close(y, yr, rtol=1e-5, atol=2e-4)
    pos = (yr > 1e-3)
    # argmax agrees except on near-ties, where fp summation order may pick the other window cell
    mism = (am[pos] != amr[pos]).float().mean().item()
    assert mism < 1e-4
    labels = torch.randint(0, 10, (1000,), device=cuda)
    y2, am2, lab = hip_ops.conv_front_fwd(x, idx, w, b, labels=labels)     # labels gathered in passing
    assert torch.equal(lab, labels[idx]) and torch.equal(y2, y) and torch.equal(am2, am)


@pytest.mark.parametrize("kind", ["grad", "sgd", "adam"])
def test_conv_bwd(cuda, kind):
    B = 16
    x = _shard(500, cuda)
    idx = torch.randperm(500, device=cuda)[:B]
    w, b = _conv_params(cuda)
    y, am = torch_ops.conv_front_fwd(x, idx, w, b)
    dy = torch.randn(B, 5408, device=cuda)
    dwr, dbr = torch_ops.conv_front_bwd(dy, y, am, x, idx, w, b)
    if kind == "grad":
        dw, db = hip_ops.conv_front_bwd(dy, y, am, x, idx, w, b)
        _close(dw, dwr, rtol=1e-4, atol=1e-2)
        _close(db, dbr, rtol=1e-4, atol=1e-3)
        return
    cfg = OptimCfg("adam", 1e-3, weight_decay=1e-5) if kind == "adam" else OptimCfg("sgd", 1e-3, momentum=0.9)
    def st(p):
        return {"m": torch.full_like(p, 0.01), "v": torch.full_like(p, 0.02)} if kind == "adam" else \
            {"buf": torch.full_like(p, 0.01)}
    w1, b1, w2, b2 = w.clone(), b.clone(), w.clone(), b.clone()
    sw1, sb1, sw2, sb2 = st(w), st(b), st(w), st(b)
    hip_ops.conv_front_bwd_step_(dy, y, am, x, idx, w1, b1, cfg, sw1, sb1, 3)
    torch_ops.apply_update_(w2, dwr, sw2, cfg, 3)
    torch_ops.apply_update_(b2, dbr, sb2, cfg, 3)
    # gradients here are O(1e3) (raw 0..255 pixels x N(0,1) cut gradients); the two-stage
    # reduction's summation order differs from torch's at ~1e-7 relative
    _close(w1, w2, rtol=1e-4, atol=1e-4)
    _close(b1, b2, rtol=1e-4, atol=1e-5)
    for k in sw1:
        _close(sw1[k], sw2[k], rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("M,N,K", [(16, 5000, 5408), (16, 1000, 5000), (16, 100, 1000), (5, 10, 100),
                                    (16, 37, 52), (200, 100, 1000), (1000, 5000, 5408), (8000, 1000, 5000),
                                    (129, 130, 36), (300, 10, 100), (1000, 100, 1000), (14000, 5000, 5408),
                                    (200, 1000, 5000)])
@pytest.mark.parametrize("relu,drop", [(False, 0.0), (True, 0.0), (True, 0.5)])
@pytest.mark.parametrize("gemm", [0, 2])
def test_linear_fwd(cuda, M, N, K, relu, drop, gemm):
    """M <= 128: the skinny split-K kernels; M > 128: the in-tree LDS-tiled MFMA GEMM with its
    fused epilogue (gemm 0, the default: 14000 x 5000 x 5408 takes the tail split of its last
    partial round, 1000 x 100 x 1000 the deep split-K of a small grid, 200 x 1000 x 5000 16 slices
    of a 16-tile grid) or hipBLASLt + the
    in-tree epilogue (gemm 2: variant 11)."""
    if gemm and M <= 128:
        pytest.skip("the tiled GEMM serves M > 128")
    x = torch.randn(M, K, device=cuda)
    w = torch.randn(N, K, device=cuda) / K ** 0.5
    b = torch.randn(N, device=cuda)
    seed = 0x1234_5678_9ABC
    yr = torch_ops.linear_fwd(x, w, b, relu, drop, seed, col_offset=3)
    C = hip_ops.C()
    C.set_variant(11, gemm)
    try:
        y = hip_ops.linear_fwd(x, w, b, relu, drop, seed, col_offset=3)
        _close(y, yr, rtol=1e-4, atol=1e-4)
    finally:
        C.set_variant(11, 0)


@pytest.mark.parametrize("M,N,K,max_split", [(16, 1000, 5000, 16), (16, 1000, 628, 1), (16, 1000, 1000, 1),
                                              (64, 1000, 5000, 16), (16, 100, 1000, 16), (5, 37, 52, 16),
                                              (16, 1000, 1252, 2)])
def test_linear_fwd_partial(cuda, M, N, K, max_split):
    """Un-reduced split-K slabs of x @ w.T (fc2 forward of the server step; max_split 1 = the
    row-parallel TP shard's plain partial product)."""
    x = torch.randn(M, K, device=cuda)
    w = torch.randn(N, K, device=cuda) / K ** 0.5
    P = hip_ops.linear_fwd_partial(x, w, max_split=max_split, key="tpart")
    assert 1 <= P.shape[0] <= max_split
    _close(P.sum(0), x @ w.t(), rtol=1e-4, atol=1e-4)


def test_linear_fwd_wide_k_uses_the_k_loop_form(cuda):
    """K past the one-round-trip form's reach (the concat fc1 at k = 8: K = 43264) runs the
    k-loop skinny kernel (csrc/linear.hip skinny_fwd_kernel)."""
    x = torch.randn(16, 43264, device=cuda)
    w = torch.randn(200, 43264, device=cuda) / 43264 ** 0.5
    b = torch.randn(200, device=cuda)
    y = hip_ops.linear_fwd(x, w, b, True, 0.0, 1)
    _close(y, torch.relu(x @ w.t() + b), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("M,N,K", [(16, 5000, 5408), (16, 1000, 5000), (16, 100, 1000), (16, 10, 100),
                                    (3, 37, 52), (16, 1000, 628), (64, 1000, 5000), (40, 1000, 604),
                                    (16, 12, 8), (200, 1000, 5000), (1000, 100, 1000), (200, 5000, 5408),
                                    (1000, 1000, 5000), (300, 24, 40), (130, 2052, 132)])
@pytest.mark.parametrize("masked", [False, True])
def test_linear_dgrad(cuda, M, N, K, masked):
    """The split-N + reduce pair (the mask fused into the reduce), or one masked launch."""
    dz = torch.randn(M, N, device=cuda)
    w = torch.randn(N, K, device=cuda) / N ** 0.5
    h = torch.relu(torch.randn(M, K, device=cuda)) if masked else None
    dx = hip_ops.linear_dgrad(dz, w, h, 2.0)
    dxr = torch_ops.linear_dgrad(dz, w, h, 2.0)
    _close(dx, dxr, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("M,N,K", [(16, 5000, 5408), (16, 100, 1000), (7, 10, 100), (40, 33, 20)])
@pytest.mark.parametrize("kind", ["grad", "sgd", "adam"])
def test_linear_wgrad_opt(cuda, M, N, K, kind):
    dz = torch.randn(M, N, device=cuda)
    a = torch.randn(M, K, device=cuda)
    if kind == "grad":
        dw, db = hip_ops.linear_wgrad(dz, a)
        dwr, dbr = torch_ops.linear_wgrad(dz, a)
        _close(dw, dwr, rtol=1e-4, atol=1e-4)
        _close(db, dbr, rtol=1e-4, atol=1e-4)
        return
    cfg = OptimCfg("adam", 1e-3, weight_decay=1e-5) if kind == "adam" else OptimCfg("sgd", 1e-2, momentum=0.9)
    w = torch.randn(N, K, device=cuda)
    b = torch.randn(N, device=cuda)
    def st(p):
        return {"m": torch.randn_like(p) * 0.1, "v": torch.rand_like(p) * 0.1} if kind == "adam" else \
            {"buf": torch.randn_like(p) * 0.1}
    sw, sb = st(w), st(b)
    sw2 = {k: v.clone() for k, v in sw.items()}
    sb2 = {k: v.clone() for k, v in sb.items()}
    w2, b2 = w.clone(), b.clone()
    hip_ops.linear_wgrad_step_(dz, a, w, b, cfg, sw, sb, 5)
    torch_ops.linear_wgrad_step_(dz, a, w2, b2, cfg, sw2, sb2, 5)
    _close(w, w2, rtol=1e-4, atol=1e-5)
    _close(b, b2, rtol=1e-4, atol=1e-5)
    for k in sw:
        _close(sw[k], sw2[k], rtol=1e-4, atol=1e-5)
        _close(sb[k], sb2[k], rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("M,C", [(16, 100), (16, 10), (16, 5408), (9, 100), (1000, 100)])
def test_softmax_ce(cuda, M, C):
    x = torch.randn(M, C, device=cuda) * 3
    y = torch.randint(0, min(C, 10), (M,), device=cuda)
    y[0] = -100
    loss, d = hip_ops.softmax_ce(x, y, 1.0 / M)
    lr, dr = torch_ops.softmax_ce(x, y, 1.0 / M)
    _close(loss, lr, rtol=1e-5, atol=1e-5)
    _close(d, dr, rtol=1e-5, atol=1e-6)
    ref = torch.nn.functional.cross_entropy(x, y, reduction="sum") / M
    assert abs(loss.sum().item() / M - ref.item()) < 1e-4


@pytest.mark.parametrize("M,C", [(16, 100), (3001, 100), (77, 10)])
def test_eval_counters(cuda, M, C):
    x = torch.randn(M, C, device=cuda)
    y = torch.randint(0, 10, (M,), device=cuda)
    x[torch.arange(M // 2, device=cuda), y[: M // 2]] += 10.0
    c = hip_ops.eval_counters(x, y, 9)
    cr = torch_ops.eval_counters(x, y, 9)
    assert c.cpu().tolist() == cr.cpu().tolist()


def test_opt_flat(cuda):
    p = torch.randn(1001, device=cuda)
    g = torch.randn(1001, device=cuda)
    cfg = OptimCfg("adam", 1e-3, weight_decay=1e-5)
    st = {"m": torch.zeros_like(p), "v": torch.zeros_like(p)}
    p2, st2 = p.clone(), {k: v.clone() for k, v in st.items()}
    hip_ops.apply_update_(p, g, st, cfg, 1)
    torch_ops.apply_update_(p2, g, st2, cfg, 1)
    _close(p, p2, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("kind", ["sgd", "adam"])
@pytest.mark.parametrize("B", [16, 5])
def test_conv_local_step(cuda, kind, B):
    x = _shard(400, cuda)
    y_all = torch.randint(0, 10, (400,), device=cuda)
    idx = torch.randperm(400, device=cuda)[:B]
    w, b = _conv_params(cuda)
    cfg = OptimCfg("adam", 1e-3, weight_decay=1e-5) if kind == "adam" else OptimCfg("sgd", 1e-3, momentum=0.9)
    def st(p):
        return {"m": torch.zeros_like(p), "v": torch.zeros_like(p)} if kind == "adam" else \
            {"buf": torch.zeros_like(p)}
    w1, b1, w2, b2 = w.clone(), b.clone(), w.clone(), b.clone()
    s = [st(w), st(b), st(w), st(b)]
    for t in (1, 2):
        l1 = hip_ops.conv_local_step_(x, y_all, idx, w1, b1, cfg, s[0], s[1], t)
        l2 = torch_ops.conv_local_step_(x, y_all, idx, w2, b2, cfg, s[2], s[3], t)
        _close(l1, l2, rtol=1e-4, atol=1e-4)
    # Adam's normalised step amplifies rounding on ~zero gradients: compare loosely there
    _close(w1, w2, rtol=1e-3, atol=3e-4 if kind == "adam" else 1e-6)
    _close(b1, b2, rtol=1e-3, atol=3e-4 if kind == "adam" else 1e-6)


@pytest.mark.parametrize("kind", ["sgd", "adam"])
@pytest.mark.parametrize("M,shapes,mn", [(16, [(5000, 5408), (1000, 5000)], 16), (20, [(100, 1000), (33, 20)], 5),
                                         (7, [(10, 100)], 0), (64, [(1000, 5408), (100, 1000)], 64),
                                         (48, [(300, 1000)], 37)])
def test_wgrad_group(cuda, kind, M, shapes, mn):
    """Grouped wgrad+optimizer (+ layer-0 look-ahead forward, up to 64 rows) == per-layer fp32 reference."""
    cfg = OptimCfg("adam", 1e-3, weight_decay=1e-5) if kind == "adam" else OptimCfg("sgd", 1e-2, momentum=0.9)

    def st(p):
        return {"m": torch.randn_like(p) * 0.1, "v": torch.rand_like(p) * 0.1} if kind == "adam" else \
            {"buf": torch.randn_like(p) * 0.1}
    layers, refs = [], []
    for N, K in shapes:
        dz, a = torch.randn(M, N, device=cuda), torch.randn(M, K, device=cuda)
        w, b = torch.randn(N, K, device=cuda), torch.randn(N, device=cuda)
        sw, sb = st(w), st(b)
        refs.append((dz, a, w.clone(), b.clone(), {k: v.clone() for k, v in sw.items()},
                     {k: v.clone() for k, v in sb.items()}))
        layers.append((dz, a, w, sw, b, sb))
    kw = {}
    if mn:
        xn = torch.randn(mn, shapes[0][1], device=cuda)
        kw = {"x_next": xn, "p_next": hip_ops.lookahead_slabs(cuda, shapes[0][1], mn, shapes[0][0])}
    hip_ops.wgrad_group_(layers, M, cfg, 4, **kw)
    for (dz, a, w2, b2, sw2, sb2), L in zip(refs, layers):
        torch_ops.linear_wgrad_step_(dz, a, w2, b2, cfg, sw2, sb2, 4)
        _close(L[2], w2, rtol=1e-4, atol=1e-5)
        _close(L[4], b2, rtol=1e-4, atol=1e-5)
        for k in sw2:
            _close(L[3][k], sw2[k], rtol=1e-4, atol=1e-5)
            _close(L[5][k], sb2[k], rtol=1e-4, atol=1e-5)
    if mn:
        _close(kw["p_next"].sum(0), kw["x_next"] @ layers[0][2].t(), rtol=1e-4, atol=2e-3)


@pytest.mark.parametrize("kind", ["sgd", "adam"])
def test_wgrad_group_alternating_walk_is_bit_identical(cuda, kind):
    """Consecutive launches walk fc1's tiles in opposite directions (the Infinity Cache reuse
    order, csrc/fused.hip set_traversal): the walk only changes where and when bytes move, so
    two launches on the same inputs (one forward, one reversed) give bitwise the same outputs,
    the look-ahead slabs included."""
    cfg = OptimCfg("adam", 1e-3, weight_decay=1e-5) if kind == "adam" else OptimCfg("sgd", 1e-2, momentum=0.9)
    g = torch.Generator().manual_seed(3)
    M, shapes = 16, [(1000, 5408), (200, 1000), (100, 200)]
    base = [(torch.randn(M, N, generator=g), torch.randn(M, K, generator=g), torch.randn(N, K, generator=g),
             torch.randn(N, generator=g)) for N, K in shapes]
    xn = torch.randn(M, shapes[0][1], generator=g).to(cuda)
    outs = []
    for _ in range(3):
        layers = []
        for dz, a, w, b in base:
            w, b = w.to(cuda), b.to(cuda)
            sw = {"m": torch.full_like(w, 0.01), "v": torch.full_like(w, 0.02)} if kind == "adam" else \
                {"buf": torch.full_like(w, 0.01)}
            sb = {k: torch.full_like(b, 0.01) for k in sw}
            layers.append((dz.to(cuda), a.to(cuda), w, sw, b, sb))
        pn = hip_ops.lookahead_slabs(cuda, shapes[0][1], M, shapes[0][0])
        hip_ops.wgrad_group_(layers, M, cfg, 3, x_next=xn, p_next=pn)
        torch.cuda.synchronize()
        outs.append([t.clone() for L in layers for t in (L[2], L[4], *L[3].values(), *L[5].values())] + [pn.clone()])
    for o in outs[1:]:
        for x, y in zip(outs[0], o):
            assert torch.equal(x, y)


@pytest.mark.parametrize("kind", ["sgd", "adam"])
@pytest.mark.parametrize("rt,pol", [(1, 0), (3, 0), (8, 0), (8, 1), (40, 1)])
@pytest.mark.parametrize("M,shapes,mn", [(16, [(1000, 5408), (200, 1000), (100, 200)], 16),
                                         (7, [(36, 300), (10, 36)], 5), (16, [(300, 1000)], 0)])
def test_wgrad_stream_form_is_bitwise_the_tiled_form(cuda, kind, rt, pol, M, shapes, mn):
    """The streaming wgrad form (variant 22 = row tiles per workgroup, -1 the tiled form: A staged
    once per column walk, the next tile's state in flight; csrc/fused.hip wgrad_stream_kernel) computes every
    element's sums in the tiled form's order: W / states / biases / look-ahead slabs bitwise
    equal, under the shipped and the over-the-cache store policies (variant 21)."""
    C = hip_ops.C()
    cfg = OptimCfg("adam", 1e-3, weight_decay=1e-5) if kind == "adam" else OptimCfg("sgd", 1e-2, momentum=0.9)
    g = torch.Generator().manual_seed(5)
    base = [(torch.randn(M, N, generator=g), torch.randn(M, K, generator=g), torch.randn(N, K, generator=g),
             torch.randn(N, generator=g)) for N, K in shapes]
    xn = torch.randn(max(mn, 1), shapes[0][1], generator=g).to(cuda)
    outs = []
    try:
        for v22 in (-1, rt):
            C.set_variant(22, v22)
            C.set_variant(21, pol)
            layers = []
            for dz, a, w, b in base:
                w, b = w.to(cuda), b.to(cuda)
                sw = {"m": torch.full_like(w, 0.01), "v": torch.full_like(w, 0.02)} if kind == "adam" else \
                    {"buf": torch.full_like(w, 0.01)}
                sb = {k: torch.full_like(b, 0.01) for k in sw}
                layers.append((dz.to(cuda), a.to(cuda), w, sw, b, sb))
            kw = {}
            if mn:
                kw = {"x_next": xn[:mn], "p_next": hip_ops.lookahead_slabs(cuda, shapes[0][1], mn, shapes[0][0])}
            hip_ops.wgrad_group_(layers, M, cfg, 3, **kw)
            torch.cuda.synchronize()
            outs.append([t.clone() for L in layers for t in (L[2], L[4], *L[3].values(), *L[5].values())] +
                        ([kw["p_next"].clone()] if mn else []))
    finally:
        C.set_variant(22, 0)
        C.set_variant(21, 0)
    for x, y in zip(outs[0], outs[1]):
        assert torch.equal(x, y)


@pytest.mark.parametrize("kind", ["sgd", "adam"])
@pytest.mark.parametrize("rt,pin", [(-1, 32), (8, 32), (8, 1008), (40, 496)])
def test_wgrad_pinned_rows_are_bitwise_unpinned(cuda, kind, rt, pin):
    """The pinned-row cache policy (variant 23: the first `pin` rows of layer 0 plain, the rest
    non-temporal; csrc/fused.hip set_traversal -- concat's fc1 by default) changes cache hints
    only: W / states / biases / look-ahead slabs bitwise equal to the unpinned shipped policy,
    with the pinned boundary inside a tile run, past the last row, and on the tiled form."""
    C = hip_ops.C()
    cfg = OptimCfg("adam", 1e-3, weight_decay=1e-5) if kind == "adam" else OptimCfg("sgd", 1e-2, momentum=0.9)
    g = torch.Generator().manual_seed(7)
    M, shapes, mn = 16, [(1000, 5408), (200, 1000), (100, 200)], 16
    base = [(torch.randn(M, N, generator=g), torch.randn(M, K, generator=g), torch.randn(N, K, generator=g),
             torch.randn(N, generator=g)) for N, K in shapes]
    xn = torch.randn(mn, shapes[0][1], generator=g).to(cuda)
    outs = []
    try:
        C.set_variant(22, rt)
        for v23 in (-1, pin):
            C.set_variant(23, v23)
            layers = []
            for dz, a, w, b in base:
                w, b = w.to(cuda), b.to(cuda)
                sw = {"m": torch.full_like(w, 0.01), "v": torch.full_like(w, 0.02)} if kind == "adam" else \
                    {"buf": torch.full_like(w, 0.01)}
                sb = {k: torch.full_like(b, 0.01) for k in sw}
                layers.append((dz.to(cuda), a.to(cuda), w, sw, b, sb))
            pn = hip_ops.lookahead_slabs(cuda, shapes[0][1], mn, shapes[0][0])
            hip_ops.wgrad_group_(layers, M, cfg, 3, x_next=xn, p_next=pn)
            torch.cuda.synchronize()
            outs.append([t.clone() for L in layers for t in (L[2], L[4], *L[3].values(), *L[5].values())] + [pn])
    finally:
        C.set_variant(22, 0)
        C.set_variant(23, 0)
    for x, y in zip(outs[0], outs[1]):
        assert torch.equal(x, y)


@pytest.mark.parametrize("kind", ["sgd", "adam"])
def test_conv_local_epoch_matches_steps(cuda, kind):
    """The C++-looped epoch == the per-step calls (bitwise), incl. a partial last batch."""
    x = _shard(300, cuda)
    y_all = torch.randint(0, 10, (300,), device=cuda)
    order = torch.randperm(300, device=cuda)[:109]
    w, b = _conv_params(cuda)
    cfg = OptimCfg("adam", 1e-3, weight_decay=1e-5) if kind == "adam" else OptimCfg("sgd", 1e-3, momentum=0.9)

    def st(p):
        return {"m": torch.zeros_like(p), "v": torch.zeros_like(p)} if kind == "adam" else \
            {"buf": torch.zeros_like(p)}
    w1, b1, w2, b2 = w.clone(), b.clone(), w.clone(), b.clone()
    s = [st(w), st(b), st(w), st(b)]
    l1 = hip_ops.conv_local_epoch_(x, y_all, order, 16, w1, b1, cfg, s[0], s[1], 3)
    l2 = torch.cat([hip_ops.conv_local_step_(x, y_all, order[i:i + 16], w2, b2, cfg, s[2], s[3], 3 + j)
                    for j, i in enumerate(range(0, 109, 16))])
    torch.cuda.synchronize()
    assert torch.equal(l1, l2) and torch.equal(w1, w2) and torch.equal(b1, b2)
    for k in s[0]:
        assert torch.equal(s[0][k], s[2][k]) and torch.equal(s[1][k], s[3][k])


@pytest.mark.parametrize("M,S2,N2,C", [(16, 4, 1000, 100), (7, 1, 1000, 100), (16, 8, 1000, 10), (16, 16, 1000, 100), (16, 20, 1000, 100),
                                       (3, 2, 512, 97), (16, 1, 1000, 300)])
def test_server_head3(cuda, M, S2, N2, C):
    """fc2 slab reduce + epilogue, fc3, softmax-CE, fc3 dgrad, fc2 ReLU/dropout backward
    against the eager composition of the same ops."""
    g = torch.Generator().manual_seed(7)
    P2 = (torch.randn(S2, M, N2, generator=g) * 0.5).to(cuda)
    b2 = (torch.randn(N2, generator=g) * 0.1).to(cuda)
    W3 = (torch.randn(C, N2, generator=g) * 0.05).to(cuda)
    b3 = (torch.randn(C, generator=g) * 0.1).to(cuda)
    y = torch.randint(0, min(C, 10), (M,), generator=g).to(cuda)
    y[0] = -100                                        # ignored row
    seed = 1234567
    h2, dlog, dz2, loss = hip_ops.server_head3(P2, b2, True, 0.5, seed, W3, b3, y, 1.0 / M)
    h2r = torch_ops.linear_epilogue(P2.sum(0).cpu(), b2.cpu(), True, 0.5, seed)
    logits = h2r @ W3.cpu().t() + b3.cpu()
    lossr, dlogr = torch_ops.softmax_ce(logits, y.cpu(), 1.0 / M)
    dz2r = (dlogr @ W3.cpu()) * (h2r > 0) * 2.0
    _close(h2, h2r)
    _close(loss, lossr, rtol=1e-4, atol=1e-5)
    _close(dlog, dlogr, rtol=1e-4, atol=1e-6)
    _close(dz2, dz2r, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("M,G", [(16, 2), (16, 4), (9, 8)])
def test_server_head_grouped_cross_entropy(cuda, M, G):
    """G cross-entropy groups of 100 logits (SISA-concat's k heads): per-(row, group) label,
    scale and loss; ignored (row, group) pairs give zero loss and zero dlogits.  G = 4 / 8 (C =
    400 / 800) take head_fwd's output groups over gridDim.z and head_bwd's wide partial-logit
    reads (csrc/fused.hip)."""
    g = torch.Generator().manual_seed(G)
    N2, C = 1000, 100 * G
    P2 = (torch.randn(4, M, N2, generator=g) * 0.5).to(cuda)
    b2 = (torch.randn(N2, generator=g) * 0.1).to(cuda)
    W3 = (torch.randn(C, N2, generator=g) * 0.05).to(cuda)
    b3 = (torch.randn(C, generator=g) * 0.1).to(cuda)
    y = torch.randint(0, 10, (M, G), generator=g).to(cuda)
    y[M - 1, 0] = -100
    y[0, G - 1] = -100
    sc = (1.0 / torch.randint(1, M + 1, (M, G), generator=g).float()).to(cuda)
    h2, dlog, dz2, loss = hip_ops.server_head3(P2, b2, True, 0.5, 7, W3, b3, y, 1.0, groups=G, gscale=sc)
    h2r = torch_ops.linear_epilogue(P2.sum(0).cpu(), b2.cpu(), True, 0.5, 7)
    logits = (h2r @ W3.cpu().t() + b3.cpu()).view(M * G, 100)
    lossr, dr = torch_ops.softmax_ce(logits, y.cpu().view(-1), 1.0)
    dr = (dr.view(M, G, 100) * sc.cpu().view(M, G, 1)).view(M, C)
    dz2r = (dr @ W3.cpu()) * (h2r > 0) * 2.0
    _close(h2, h2r)
    _close(loss.view(-1), lossr, rtol=1e-4, atol=1e-5)
    _close(dlog, dr, rtol=1e-4, atol=1e-6)
    _close(dz2, dz2r, rtol=1e-4, atol=1e-6)


def test_relu_mask(cuda):
    g = torch.Generator().manual_seed(11)
    d, h = torch.randn(16, 100, generator=g).to(cuda), torch.randn(16, 100, generator=g).to(cuda)
    torch.testing.assert_close(hip_ops.relu_mask(d, h, 2.0), torch_ops.relu_mask(d, h, 2.0))


@pytest.mark.parametrize("kind", ["sgd", "adam"])
@pytest.mark.parametrize("M", [16, 7, 32])
def test_head_step_matches_torch(cuda, kind, M):
    """_C.head_step (the U-shape head's forward + CE + dgrad + optimizer in one launch) ==
    the fp32 torch reference of the same step (the MFMA kernel up to 16 rows, the FMA kernel
    beyond)."""
    _head_step_check(cuda, kind, M)


def _head_step_check(cuda, kind, M):
    cfg = OptimCfg("adam", 1e-3) if kind == "adam" else OptimCfg("sgd", 1e-2, momentum=0.9)
    g = torch.Generator().manual_seed(2)
    x = torch.rand(M, 100, generator=g)
    W, b = torch.randn(10, 100, generator=g) * 0.1, torch.randn(10, generator=g) * 0.1
    y = torch.randint(0, 10, (M,), generator=g)
    st = lambda p: ({"m": torch.full_like(p, 0.01), "v": torch.full_like(p, 0.02)} if kind == "adam"  # noqa: E731
                    else {"buf": torch.full_like(p, 0.01)})
    sw_ref, sb_ref = st(W), st(b)
    Wr, br = W.clone().requires_grad_(), b.clone().requires_grad_()
    xr = x.clone().requires_grad_()
    loss_ref = torch.nn.functional.cross_entropy(xr @ Wr.t() + br, y, reduction="none")
    loss_ref.mean().backward()
    Wn, bn = W.clone(), b.clone()
    torch_ops.apply_update_(Wn, Wr.grad, sw_ref, cfg, 3)
    torch_ops.apply_update_(bn, br.grad, sb_ref, cfg, 3)
    Wg, bg = W.to(cuda), b.to(cuda)
    swg, sbg = {k: v.to(cuda) for k, v in st(W).items()}, {k: v.to(cuda) for k, v in st(b).items()}
    loss, dx = hip_ops.head_step_(x.to(cuda), Wg, bg, y.to(cuda), 1.0 / M, cfg, swg, sbg, 3)
    _close(loss, loss_ref.detach(), rtol=1e-5, atol=1e-5)
    _close(dx, xr.grad, rtol=1e-5, atol=1e-6)
    _close(Wg, Wn, rtol=1e-5, atol=1e-6)
    _close(bg, bn, rtol=1e-5, atol=1e-6)
    for k in swg:
        _close(swg[k], sw_ref[k], rtol=1e-5, atol=1e-7)
        _close(sbg[k], sb_ref[k], rtol=1e-5, atol=1e-7)
    # mask_by_input: dX also carries the producer's ReLU backward, [x > 0]
    xs = torch.randn(M, 100, generator=g)
    outs = []
    for mask in (False, True):
        W2, b2 = W.to(cuda), b.to(cuda)
        s2w, s2b = {k: v.to(cuda) for k, v in st(W).items()}, {k: v.to(cuda) for k, v in st(b).items()}
        outs.append(hip_ops.head_step_(xs.to(cuda), W2, b2, y.to(cuda), 1.0 / M, cfg, s2w, s2b, 3,
                                       mask_by_input=mask)[1])
    assert torch.equal(outs[1], torch.where(xs.to(cuda) > 0, outs[0], torch.zeros_like(outs[0])))


@pytest.mark.parametrize("kind", ["sgd", "adam"])
def test_front_deferred_update_is_bitwise_immediate(cuda, kind):
    """FrontEngine's deferred client step (the update applied by the next forward in-kernel
    and stored by the next backward; 2 launches per batch instead of 3) gives bitwise the
    same activations, parameters and optimizer states as the immediate form."""
    from splitlearning_amd.data.device_dataset import DeviceShard
    from splitlearning_amd.engine import FrontEngine, OptSlot
    from splitlearning_amd.models import ClientFrontSisa
    cfg = OptimCfg("adam", 1e-3, weight_decay=1e-5) if kind == "adam" else OptimCfg("sgd", 1e-2, momentum=0.9)
    g = torch.Generator().manual_seed(5)
    shard = DeviceShard(torch.randint(0, 256, (300, 784), dtype=torch.uint8, generator=g),
                        torch.randint(0, 10, (300,), generator=g), cuda)
    engines = []
    for _ in range(2):
        torch.manual_seed(11)
        engines.append((FrontEngine(ClientFrontSisa(), cuda), OptSlot(cfg)))
    batches = [torch.randperm(300, generator=g)[:bs].to(cuda) for bs in (16, 16, 16, 7, 16)]
    dys = [torch.randn(idx.numel(), 5408, generator=g).to(cuda) * 1e-2 for idx in batches]
    acts = [[], []]
    for e, (fe, slot) in enumerate(engines):
        for idx, dy in zip(batches, dys):
            y, am, lab = fe.forward(shard, idx, with_labels=True)
            acts[e].append((y.clone(), am.clone(), lab.clone()))
            fe.backward_step(dy, y, am, shard, idx, slot, defer=(e == 1))
        fe.flush()
    torch.cuda.synchronize()
    for (ya, aa, la), (yb, ab, lb) in zip(*acts):
        assert torch.equal(ya, yb) and torch.equal(aa, ab) and torch.equal(la, lb)
    (fa, sa), (fb, sb) = engines
    for ta, tb in zip(fa.params, fb.params):
        assert torch.equal(ta, tb)
    assert sa.t == sb.t == len(batches)
    for name in sa.states:
        for k in sa.states[name]:
            assert torch.equal(sa.states[name][k], sb.states[name][k]), (name, k)


@pytest.mark.parametrize("kind", ["adam", "sgd"])
def test_multi_alice_local_epoch_is_bitwise_per_alice(cuda, kind):
    """Co-located Alices stepped together (one launch per step for all of them, Dirichlet-like
    unequal shard sizes, partial last batches) == each Alice's own local epoch, bitwise, over
    two epochs (the per-Alice optimizer step counters carry on)."""
    from splitlearning_amd.data.device_dataset import DeviceShard
    from splitlearning_amd.engine import FrontEngine, OptSlot
    from splitlearning_amd.models import ClientFrontSisa
    sizes = [100, 37, 64, 16, 5, 250]
    cfg = OptimCfg("adam", 1e-3, weight_decay=1e-5) if kind == "adam" else OptimCfg("sgd", 1e-3, momentum=0.9)

    def world():
        fronts, shards, slots = [], [], []
        for a, n in enumerate(sizes):
            g = torch.Generator().manual_seed(100 + a)
            x = torch.randint(0, 256, (n, 1, 28, 28), generator=g, dtype=torch.uint8)
            y = torch.randint(0, 10, (n,), generator=g)
            torch.manual_seed(a)
            fronts.append(FrontEngine(ClientFrontSisa(), cuda))
            shards.append(DeviceShard(x, y, cuda))
            slots.append(OptSlot(cfg))
        return fronts, shards, slots
    fa, sa, pa = world()
    fb, sb, pb = world()
    for ep in range(2):
        orders = [torch.randperm(n, generator=torch.Generator().manual_seed(7 * ep + a)).to(cuda)
                  for a, n in enumerate(sizes)]
        la = [f.local_epoch(s, o, 16, p) for f, s, o, p in zip(fa, sa, orders, pa)]
        lb = FrontEngine.local_epoch_multi(fb, sb, orders, 16, pb)
        torch.cuda.synchronize()
        for x, y in zip(la, lb):
            assert torch.equal(x, y)
    for f1, f2, p1, p2 in zip(fa, fb, pa, pb):
        for (k, v1), v2 in zip(f1.module.state_dict().items(), f2.module.state_dict().values()):
            assert torch.equal(v1, v2), k
        assert p1.t == p2.t
        for name, st in p1.states.items():
            for k, v in st.items():
                assert torch.equal(v, p2.states[name][k]), (name, k)


@pytest.mark.parametrize("M,N,K", [(1000, 5000, 5408), (300, 130, 1000), (16, 1000, 5000)])
def test_linear_fwd_bf16_compute(cuda, M, N, K):
    """--dtype bf16: operands rounded to bf16 (RNE), fp32 accumulation: equals the fp32 product
    of the bf16-rounded operands up to summation order."""
    C = hip_ops.C()
    x = torch.randn(M, K, device=cuda)
    w = torch.randn(N, K, device=cuda) / K ** 0.5
    b = torch.randn(N, device=cuda)
    C.set_compute_dtype("bf16")
    try:
        y = hip_ops.linear_fwd(x, w, b, True, 0.0, 0)
    finally:
        C.set_compute_dtype("fp32")
    yr = torch.relu(x.bfloat16().float() @ w.bfloat16().float().t() + b)
    _close(y, yr, rtol=1e-4, atol=2e-4)
    # and it is NOT the exact-fp32 product (the mode is really on)
    assert (y - torch.relu(x @ w.t() + b)).abs().max().item() > 1e-3


@pytest.mark.parametrize("M,N,K", [(16, 1000, 5000), (16, 1000, 628), (16, 100, 1000), (64, 1000, 5000), (5, 40, 64)])
def test_linear_dgrad_bf16_mfma(cuda, M, N, K):
    """--dtype bf16 data gradient on bf16 MFMA (v_mfma_f32_16x16x32_bf16 over 32-row steps of
    W, the split-N tails on rounded operands): equals the fp32 product of the bf16-rounded
    operands (exact products, fp32 accumulation) up to summation order, with the ReLU mask."""
    C = hip_ops.C()
    dz = torch.randn(M, N, device=cuda)
    w = torch.randn(N, K, device=cuda) / N ** 0.5
    h = torch.relu(torch.randn(M, K, device=cuda))
    C.set_compute_dtype("bf16")
    try:
        got = hip_ops.linear_dgrad(dz, w, h, 2.0)
    finally:
        C.set_compute_dtype("fp32")
    ref = (dz.bfloat16().float() @ w.bfloat16().float()) * (h > 0).float() * 2.0
    _close(got, ref, rtol=1e-4, atol=2e-4)
    assert (got - torch_ops.linear_dgrad(dz, w, h, 2.0)).abs().max().item() > 1e-4   # really bf16


@pytest.mark.parametrize("M", [16, 64])
def test_xcd_grouped_fc2_products(cuda, M):
    """The XCD-grouped workgroup order of the fc2 forward / dgrad (a permutation of which
    dispatch slot runs which tile) gives the fp32 products: split-K slabs summing to x @ w.T,
    and the masked data gradient, at the full width and at a TP = 8 shard (K = 628, S = 16)."""
    x = torch.randn(M, 5000, device=cuda)
    w = torch.randn(1000, 5000, device=cuda) / 70.0
    dz = torch.randn(M, 1000, device=cuda)
    h = torch.relu(torch.randn(M, 5000, device=cuda))
    _close(hip_ops.linear_fwd_partial(x, w, key="xg").sum(0), x @ w.t(), rtol=1e-4, atol=1e-4)
    _close(hip_ops.linear_dgrad(dz, w, h, 2.0), torch_ops.linear_dgrad(dz, w, h, 2.0), rtol=1e-4, atol=1e-4)
    w8, h8 = w[:, :628].contiguous(), h[:, :628].contiguous()
    _close(hip_ops.linear_dgrad(dz, w8, h8, 2.0), torch_ops.linear_dgrad(dz, w8, h8, 2.0), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("M,R,K,mask", [(200, 1000, 5000, True), (1000, 5000, 5408, False), (14000, 1000, 5000, True),
                                        (130, 100, 1000, True)])
def test_nn_dgrad_gemm_matches_torch(M, R, K, mask):
    """The in-tree NN-layout MFMA GEMM for data gradients of many rows (csrc/gemm.hip
    gemm_nn_dgrad; reference: nn.Linear's backward at --batch_size rows, split_nn.py:156):
    dX = (dZ . W) masked by the previous layer's ReLU / dropout (h > 0 ? . scale : 0), against
    fp32 torch, through ops.hip_ops.linear_dgrad's large-M route (no hipBLASLt)."""
    import torch
    from splitlearning_amd.ops import hip_ops as H
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(M + K)
    dz = torch.randn(M, R, generator=g).to(dev)
    w = (torch.randn(R, K, generator=g) / R ** 0.5).to(dev)
    h = torch.relu(torch.randn(M, K, generator=g)).to(dev) if mask else None
    out = H.linear_dgrad(dz, w, h, 2.0 if mask else 1.0)
    ref = (dz.double() @ w.double())
    if mask:
        ref = torch.where(h > 0, ref * 2.0, torch.zeros_like(ref))
    torch.testing.assert_close(out.double(), ref, rtol=1e-4, atol=1e-4 * ref.abs().max().item())
