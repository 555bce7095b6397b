"""Eager PyTorch implementations of every framework op.

These are (a) the CPU execution path (gloo multi-process tests, CPU runs of
`split_nn.py`) and (b) the fp32 ground truth the HIP kernels are tested
against.  Signatures are identical to `ops.hip_ops`; `ops.__init__` picks one
per call by device.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from .rng import keep_mask

CUT = 5408


# ---------------------------------------------------------------- conv front
def conv_front_fwd(x_u8: torch.Tensor, idx: torch.Tensor, w: torch.Tensor, b: torch.Tensor, labels=None):
    """Gather rows `idx` of the uint8 shard, conv3x3(1->32)+bias, ReLU, maxpool2x2.

    Returns (y [B,5408] fp32 NCHW-flattened, am uint8 [B,5408] argmax-in-window 0..3),
    plus `labels[idx]` when the shard's labels are given.
    """
    if labels is not None:
        return conv_front_fwd(x_u8, idx, w, b) + (labels.index_select(0, idx),)
    x = x_u8.index_select(0, idx).to(torch.float32).reshape(-1, 1, 28, 28)
    z = F.relu(F.conv2d(x, w, b))
    y, ind = F.max_pool2d(z, 2, 2, return_indices=True)
    # ind is the flat index into 26x26; convert to 2-bit window position
    r = ind // 26
    c = ind % 26
    am = ((r % 2) * 2 + (c % 2)).to(torch.uint8)
    return y.reshape(-1, CUT).contiguous(), am.reshape(-1, CUT).contiguous()


def conv_front_bwd(dy, y, am, x_u8, idx, w, b):
    """Gradients of conv weight/bias given dL/dy for the pooled, flattened output."""
    B = dy.shape[0]
    x = x_u8.index_select(0, idx).to(torch.float32).reshape(B, 1, 28, 28)
    g = (dy * (y > 0)).reshape(B, 32, 13, 13)
    amr = am.reshape(B, 32, 13, 13).long()
    dz = torch.zeros(B, 32, 26, 26, dtype=dy.dtype, device=dy.device)
    ph = torch.arange(13, device=dy.device).view(1, 1, 13, 1)
    pw = torch.arange(13, device=dy.device).view(1, 1, 1, 13)
    rr = 2 * ph + amr // 2
    cc = 2 * pw + amr % 2
    dz.view(B, 32, -1).scatter_(2, (rr * 26 + cc).reshape(B, 32, -1), g.reshape(B, 32, -1))
    dw = torch.nn.grad.conv2d_weight(x, w.shape, dz)
    db = dz.sum(dim=(0, 2, 3))
    return dw, db


# ---------------------------------------------------------------- linear
# `--dtype bf16`: GEMM operands rounded to bf16, fp32 accumulation (the HIP kernels' rule,
# csrc/common.h bfr); parameters and optimizer state stay fp32
_BF16 = False


def set_compute_dtype(dtype: str):
    global _BF16
    if dtype not in ("fp32", "bf16"):
        raise ValueError(dtype)
    _BF16 = dtype == "bf16"


def _r(t: torch.Tensor) -> torch.Tensor:
    return t.to(torch.bfloat16).to(t.dtype) if _BF16 else t


def linear_fwd(x, w, b, relu: bool, drop_p: float, seed: int, col_offset: int = 0,
               out: torch.Tensor | None = None):
    y = _r(x) @ _r(w).t()
    if b is not None:
        y = y + b
    if relu:
        y = F.relu(y)
    if drop_p > 0:
        keep = keep_mask(seed, y.shape[0], y.shape[1], drop_p, col_offset, device=y.device)
        y = y * keep * (1.0 / (1.0 - drop_p))
    if out is not None:
        out.copy_(y)
        return out
    return y


def linear_epilogue(P, b, relu: bool, drop_p: float, seed: int, col_offset: int = 0):
    """bias + ReLU + dropout applied to an already-reduced GEMM result (row-parallel layers)."""
    y = P if b is None else P + b
    if relu:
        y = F.relu(y)
    if drop_p > 0:
        keep = keep_mask(seed, y.shape[0], y.shape[1], drop_p, col_offset, device=y.device)
        y = y * keep * (1.0 / (1.0 - drop_p))
    return y


def linear_dgrad(dz, w, h_prev=None, scale: float = 1.0):
    """dx = dz @ w; if h_prev is given, also back-propagate through the previous
    layer's ReLU(+dropout): dx *= scale * [h_prev > 0]."""
    dx = _r(dz) @ _r(w)
    if h_prev is not None:
        dx = dx * (h_prev > 0) * scale
    return dx


def linear_wgrad(dz, a):
    return _r(dz).t() @ _r(a), _r(dz).sum(0)


# ---------------------------------------------------------------- optimizers
def adam_update_(p, g, m, v, t, lr, beta1, beta2, eps, wd):
    if wd:
        g = g.add(p, alpha=wd)
    m.mul_(beta1).add_(g, alpha=1 - beta1)
    v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    bc1 = 1 - beta1 ** t
    bc2 = 1 - beta2 ** t
    denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
    p.addcdiv_(m, denom, value=-lr / bc1)


def sgd_update_(p, g, buf, lr, momentum, wd):
    if wd:
        g = g.add(p, alpha=wd)
    if momentum:
        buf.mul_(momentum).add_(g)
        p.add_(buf, alpha=-lr)
    else:
        p.add_(g, alpha=-lr)


def apply_update_(p, g, st: dict, cfg, t: int):
    if cfg.kind == "adam":
        adam_update_(p, g, st["m"], st["v"], t, cfg.lr, cfg.beta1, cfg.beta2, cfg.eps,
                     cfg.weight_decay)
    elif cfg.kind == "sgd":
        sgd_update_(p, g, st["buf"], cfg.lr, cfg.momentum, cfg.weight_decay)
    else:
        raise ValueError(cfg.kind)


def linear_wgrad_step_(dz, a, w, b, cfg, st_w: dict, st_b: dict, t: int):
    with torch.no_grad():
        dw, db = linear_wgrad(dz, a)
        apply_update_(w, dw, st_w, cfg, t)
        if b is not None:
            apply_update_(b, db, st_b, cfg, t)


def conv_front_bwd_step_(dy, y, am, x_u8, idx, w, b, cfg, st_w, st_b, t):
    with torch.no_grad():
        dw, db = conv_front_bwd(dy, y, am, x_u8, idx, w, b)
        apply_update_(w, dw, st_w, cfg, t)
        apply_update_(b, db, st_b, cfg, t)


def conv_local_step_(x_u8, y_all, idx, w, b, cfg, st_w, st_b, t, loss_rows=None):
    """SISA client step: CE over the 5408-wide activation (Q5), backward, optimizer."""
    with torch.no_grad():
        act, am = conv_front_fwd(x_u8, idx, w, b)
        loss, d = softmax_ce(act, y_all[idx], 1.0 / idx.numel())
        conv_front_bwd_step_(d, act, am, x_u8, idx, w, b, cfg, st_w, st_b, t)
    return loss


def conv_local_epoch_(x_u8, y_all, order, B: int, w, b, cfg, st_w, st_b, t0: int):
    """ceil(n/B) client steps over `order` (steps t0, t0+1, ...); per-sample losses [n]."""
    out = []
    for i, s in enumerate(range(0, order.numel(), B)):
        out.append(conv_local_step_(x_u8, y_all, order[s:s + B], w, b, cfg, st_w, st_b, t0 + i))
    return torch.cat(out) if out else torch.empty(0, device=x_u8.device)


# ---------------------------------------------------------------- loss / metrics
def softmax_ce(logits, labels, scale: float, ignore_index: int = -100):
    """Row-wise cross-entropy. Returns (per-row loss [M] (0 for ignored rows),
    dlogits = scale * (softmax - onehot) (0 rows for ignored))."""
    lse = torch.logsumexp(logits, dim=1)
    valid = labels != ignore_index
    safe = torch.where(valid, labels, torch.zeros_like(labels))
    picked = logits.gather(1, safe.view(-1, 1)).squeeze(1)
    loss = torch.where(valid, lse - picked, torch.zeros_like(lse))
    p = torch.softmax(logits, dim=1)
    p.scatter_add_(1, safe.view(-1, 1), -torch.ones_like(picked).view(-1, 1))
    d = p * scale * valid.view(-1, 1)
    return loss, d


def relu_mask(d, h, scale: float = 1.0):
    """d * scale * [h > 0] (a layer's own ReLU/dropout backward)."""
    return d * (h > 0) * scale


def eval_counters(logits, labels, omit_label: int):
    """[correct, total, correct_unlearned, total_unlearned, correct_remaining, total_remaining]
    (reference `eval_breakdown`, data_entities_vanilla.py:159-202)."""
    pred = logits.argmax(dim=1)
    ok = pred == labels
    unl = labels == omit_label
    rem = ~unl
    return torch.stack([ok.sum(), torch.tensor(labels.numel(), device=labels.device),
                        (ok & unl).sum(), unl.sum(), (ok & rem).sum(), rem.sum()]).to(torch.int64)
