"""CPU checks of the eager op set (the ground truth for the HIP kernels) against autograd."""
import math

import numpy as np
import torch
import torch.nn.functional as F

from splitlearning_amd.config import OptimCfg
from splitlearning_amd.models import ClientFront, ClientFrontSisa
from splitlearning_amd.ops import rng, torch_ops


def test_conv_front_matches_module_and_autograd():
    torch.manual_seed(0)
    m = ClientFrontSisa()
    x_u8 = torch.randint(0, 256, (40, 784), dtype=torch.uint8)
    idx = torch.tensor([3, 1, 4, 15, 9, 26, 5, 35])
    w, b = m.conv_params()
    y, am = torch_ops.conv_front_fwd(x_u8, idx, w.detach(), b.detach())
    xf = x_u8[idx].float().reshape(-1, 1, 28, 28)
    yr = m(xf)
    torch.testing.assert_close(y, yr.detach())
    dy = torch.randn_like(y)
    (yr * dy).sum().backward()
    dw, db = torch_ops.conv_front_bwd(dy, y, am, x_u8, idx, w.detach(), b.detach())
    torch.testing.assert_close(dw, w.grad, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(db, b.grad, rtol=1e-4, atol=1e-4)


def test_ushape_front_shape():
    m = ClientFront()
    assert m(torch.zeros(2, 1, 28, 28)).shape == (2, 32, 13, 13)


def test_optimizers_match_torch():
    for kind in ("adam", "sgd"):
        p = torch.randn(50, requires_grad=True)
        p2 = p.detach().clone()
        if kind == "adam":
            opt = torch.optim.Adam([p], lr=1e-2, weight_decay=1e-5)
            cfg = OptimCfg("adam", 1e-2, weight_decay=1e-5)
            st = {"m": torch.zeros(50), "v": torch.zeros(50)}
        else:
            opt = torch.optim.SGD([p], lr=1e-2, momentum=0.9)
            cfg = OptimCfg("sgd", 1e-2, momentum=0.9)
            st = {"buf": torch.zeros(50)}
        for t in range(1, 6):
            g = torch.randn(50)
            p.grad = g.clone()
            opt.step()
            torch_ops.apply_update_(p2, g, st, cfg, t)
        torch.testing.assert_close(p.detach(), p2, rtol=1e-6, atol=1e-7)


def test_softmax_ce_matches_cross_entropy():
    x = torch.randn(16, 5408, requires_grad=True)
    y = torch.randint(0, 10, (16,))
    loss, d = torch_ops.softmax_ce(x.detach(), y, 1.0 / 16)
    ref = F.cross_entropy(x, y)
    ref.backward()
    assert math.isclose(loss.sum().item() / 16, ref.item(), rel_tol=1e-5)
    torch.testing.assert_close(d, x.grad, rtol=1e-5, atol=1e-7)


def test_dropout_hash_statistics_and_tp_invariance():
    m = rng.keep_mask(rng.step_seed(7, 1, 3), 16, 5000, 0.5)
    frac = m.float().mean().item()
    assert 0.47 < frac < 0.53
    # a column shard of the mask equals the mask computed for that shard with col_offset
    shard = rng.keep_mask(rng.step_seed(7, 1, 3), 16, 1250, 0.5, col_offset=2500)
    assert torch.equal(m[:, 2500:3750], shard)
    # different steps differ
    m2 = rng.keep_mask(rng.step_seed(7, 1, 4), 16, 5000, 0.5)
    assert (m != m2).float().mean().item() > 0.3


def test_fmix_matches_reference_constants():
    # pin a few values of the hash so the HIP twin (csrc/common.h) can be checked against them
    v = rng._fmix32(torch.tensor([0, 1, 0xDEADBEEF], dtype=torch.int64)).tolist()
    def fmix(x):
        x ^= x >> 16; x = (x * 0x85EBCA6B) & 0xFFFFFFFF; x ^= x >> 13
        x = (x * 0xC2B2AE35) & 0xFFFFFFFF; x ^= x >> 16
        return x
    assert v == [fmix(0), fmix(1), fmix(0xDEADBEEF)]


def test_linear_ops_match_autograd():
    torch.manual_seed(1)
    x = torch.randn(16, 64, requires_grad=True)
    lin = torch.nn.Linear(64, 32)
    z = lin(x)
    h = F.relu(z)
    dh = torch.randn_like(h)
    (h * dh).sum().backward()
    dz = dh * (h > 0)
    dw, db = torch_ops.linear_wgrad(dz, x.detach())
    torch.testing.assert_close(dw, lin.weight.grad, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(db, lin.bias.grad, rtol=1e-5, atol=1e-6)
    dx = torch_ops.linear_dgrad(dz, lin.weight.detach())
    torch.testing.assert_close(dx, x.grad, rtol=1e-5, atol=1e-6)


def test_eval_counters():
    logits = torch.tensor([[0.1, 0.9], [0.8, 0.2], [0.3, 0.7]])
    labels = torch.tensor([1, 1, 1])
    c = torch_ops.eval_counters(logits, labels, omit_label=1).tolist()
    assert c == [2, 3, 2, 3, 0, 0]
    _ = np  # keep numpy import (shared fixtures elsewhere)


def test_bf16_compute_rule_torch_ops():
    """--dtype bf16 on the torch path: operands rounded to bf16, fp32 accumulation."""
    from splitlearning_amd.ops import torch_ops as K
    g = torch.Generator().manual_seed(0)
    x, w, b = torch.randn(8, 40, generator=g), torch.randn(12, 40, generator=g), torch.randn(12, generator=g)
    dz = torch.randn(8, 12, generator=g)
    r = lambda t: t.bfloat16().float()  # noqa: E731
    K.set_compute_dtype("bf16")
    try:
        y = K.linear_fwd(x, w, b, False, 0.0, 0)
        dx = K.linear_dgrad(dz, w)
        dw, db = K.linear_wgrad(dz, x)
    finally:
        K.set_compute_dtype("fp32")
    torch.testing.assert_close(y, r(x) @ r(w).t() + b)
    torch.testing.assert_close(dx, r(dz) @ r(w))
    torch.testing.assert_close(dw, r(dz).t() @ r(x))
    torch.testing.assert_close(db, r(dz).sum(0))
    assert not torch.allclose(y, x @ w.t() + b, rtol=1e-5, atol=1e-5)


def test_padded_plan_layout():
    """`TailEngine.padded_plan`: each client's whole batches in order, its short final batch
    zero-padded to B rows with ignored labels; a single whole-batch client is passed through."""
    import torch
    from splitlearning_amd.engine.tail import TailEngine
    a1, y1 = torch.arange(5 * 3, dtype=torch.float32).view(5, 3), torch.arange(5)
    a2, y2 = -torch.ones(4, 3), torch.full((4,), 7)
    X, Y, rows = TailEngine.padded_plan([(a1, y1), (a2, y2)], 2)
    assert rows == [2, 2, 1, 2, 2] and X.shape == (10, 3)
    assert torch.equal(X[:5], a1) and torch.equal(X[5], torch.zeros(3)) and torch.equal(X[6:], a2)
    assert Y.tolist() == [0, 1, 2, 3, 4, -100, 7, 7, 7, 7]
    X1, Y1, r1 = TailEngine.padded_plan([(a2, y2)], 2)
    assert X1 is a2 and Y1 is y2 and r1 == [2, 2]
