"""HIP (gfx950) implementations of the framework ops, over `splitlearning_amd._C`.

Same signatures as `ops.torch_ops`.  Importing this module loads the in-tree
extension and raises if it is missing: on a GPU the HIP path is the one that
runs, it never falls back silently.
"""
from __future__ import annotations

import torch

from .. import _native

CUT = 5408
KIND = {"sgd": 1, "adam": 2}


def C():
    return _native.load()


def _opt_args(cfg, t):
    if cfg is None:
        return (0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 1)
    return (KIND[cfg.kind], cfg.lr, cfg.beta1, cfg.beta2, cfg.eps, cfg.weight_decay, cfg.momentum, max(t, 1))


def _s1(st):
    return st.get("v") if "v" in st else None


def _s0(st):
    return st["m"] if "m" in st else st["buf"]


# ---------------------------------------------------------------- conv front
def conv_front_fwd(x_u8, idx, w, b, y=None, am=None):
    B = int(idx.numel())
    if y is None:
        y = torch.empty(B, CUT, device=x_u8.device, dtype=torch.float32)
    if am is None:
        am = torch.empty(B, CUT, device=x_u8.device, dtype=torch.uint8)
    C().conv_fwd(x_u8, idx, 0, B, w.detach(), b.detach(), y, am)
    return y, am


def conv_front_bwd(dy, y, am, x_u8, idx, w, b):
    dw = torch.empty_like(w)
    db = torch.empty_like(b)
    C().conv_bwd_opt(dy, y, am, x_u8, idx, 0, int(idx.numel()), w.detach(), b.detach(), dw, None, db, None,
                     *_opt_args(None, 0))
    return dw, db


def conv_front_bwd_step_(dy, y, am, x_u8, idx, w, b, cfg, st_w, st_b, t):
    C().conv_bwd_opt(dy, y, am, x_u8, idx, 0, int(idx.numel()), w.detach(), b.detach(), _s0(st_w), _s1(st_w),
                     _s0(st_b), _s1(st_b), *_opt_args(cfg, t))


# ---------------------------------------------------------------- linear
# eval-time inference with many rows goes through hipBLASLt (plain library GEMM)
# plus the fused epilogue kernel; the skinny kernels cover the training batch sizes.
LARGE_M = 128


def linear_fwd(x, w, b, relu: bool, drop_p: float, seed: int, col_offset: int = 0, out=None):
    M, N = x.shape[0], w.shape[0]
    if out is None:
        out = torch.empty(M, N, device=x.device, dtype=torch.float32)
    w = w.detach()
    bias = b.detach() if b is not None else None
    if M > LARGE_M:
        P = torch.mm(x, w.t())
        C().linear_epilogue(P, bias, out, relu, float(drop_p), seed & ((1 << 64) - 1), col_offset)
    else:
        C().linear_fwd(x, w, bias, out, relu, float(drop_p), seed & ((1 << 64) - 1), col_offset)
    return out


def linear_epilogue(P, b, relu: bool, drop_p: float, seed: int, col_offset: int = 0):
    out = torch.empty_like(P)
    C().linear_epilogue(P, b.detach() if b is not None else None, out, relu, float(drop_p),
                        seed & ((1 << 64) - 1), col_offset)
    return out


_WS: dict = {}


def _workspace(device, n):
    key = (device, torch.cuda.current_stream(device).cuda_stream)
    ws = _WS.get(key)
    if ws is None or ws.numel() < n:
        ws = torch.empty(max(n, 1 << 20), device=device, dtype=torch.float32)
        _WS[key] = ws
    return ws


def linear_dgrad(dz, w, h_prev=None, scale: float = 1.0, out=None):
    M, K = dz.shape[0], w.shape[1]
    if out is None:
        out = torch.empty(M, K, device=dz.device, dtype=torch.float32)
    ws = _workspace(dz.device, 8 * M * K)
    C().linear_dgrad(dz, w.detach(), h_prev, float(scale), out, ws)
    return out


def linear_wgrad(dz, a):
    n, k = dz.shape[1], a.shape[1]
    w = torch.zeros(n, k, device=dz.device)
    b = torch.zeros(n, device=dz.device)
    dw = torch.empty_like(w)
    db = torch.empty_like(b)
    C().linear_wgrad_opt(dz, a, w, dw, None, b, db, None, *_opt_args(None, 0))
    return dw, db


def linear_wgrad_step_(dz, a, w, b, cfg, st_w, st_b, t):
    C().linear_wgrad_opt(dz, a, w.detach(), _s0(st_w), _s1(st_w), b.detach() if b is not None else None,
                         _s0(st_b) if b is not None else None, _s1(st_b) if b is not None else None,
                         *_opt_args(cfg, t))


def apply_update_(p, g, st, cfg, t):
    C().opt_flat(p.detach(), g, _s0(st), _s1(st), *_opt_args(cfg, t))


# ---------------------------------------------------------------- loss / metrics
def softmax_ce(logits, labels, scale: float, ignore_index: int = -100, d_out=None):
    M = logits.shape[0]
    loss = torch.empty(M, device=logits.device, dtype=torch.float32)
    d = torch.empty_like(logits) if d_out is None else d_out
    C().softmax_ce(logits, labels, int(ignore_index), float(scale), loss, d)
    return loss, d


def eval_counters(logits, labels, omit_label: int, counters=None):
    if counters is None:
        counters = torch.zeros(6, device=logits.device, dtype=torch.int64)
    C().eval_counters(logits, labels, int(omit_label), counters)
    return counters
