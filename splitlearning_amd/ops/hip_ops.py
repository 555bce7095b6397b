"""HIP (gfx950) implementations of the framework ops, over `splitlearning_amd._C`.

Same signatures as `ops.torch_ops` (plus optional graph-replay hooks: `dyn` = a device
tensor holding {step_size, inv_bc2_sqrt} for Adam, `dseed` = a device tensor holding
{seed_lo, seed_hi} for dropout).  Importing this module does not load the extension;
the first call does, and raises if it is missing: on a GPU the HIP path is the one that
runs, it never falls back silently.
"""
from __future__ import annotations

import torch

from .. import _native

CUT = 5408
KIND = {"sgd": 1, "adam": 2}
M64 = (1 << 64) - 1


def C():
    return _native.load()


def _ptr(t):
    return 0 if t is None else t.data_ptr()


def _opt_args(cfg, t, dyn=None):
    if cfg is None:
        return (0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 1, 0)
    return (KIND[cfg.kind], cfg.lr, cfg.beta1, cfg.beta2, cfg.eps, cfg.weight_decay, cfg.momentum, max(t, 1),
            _ptr(dyn))


def _s1(st):
    return st.get("v")


def _s0(st):
    return st["m"] if "m" in st else st["buf"]


_SLAB: dict = {}


def _slab(device, B):
    s = _SLAB.get(device)
    if s is None or s.numel() < B * 320:
        if s is not None:
            _WS_RETIRED.append(s)       # never free a handed-out buffer (see _workspace)
        s = torch.empty(max(B, 64, 2 * (s.numel() // 320) if s is not None else 0) * 320, device=device,
                        dtype=torch.float32)
        _SLAB[device] = s
    return s


# ---------------------------------------------------------------- conv front
def conv_front_fwd(x_u8, idx, w, b, y=None, am=None, labels=None):
    """(y, am); with `labels` (the shard's [N] labels) also the batch's labels, gathered by
    the same kernel: (y, am, labels[idx])."""
    B = int(idx.numel())
    if y is None:
        y = torch.empty(B, CUT, device=x_u8.device, dtype=torch.float32)
    if am is None:
        am = torch.empty(B, CUT, device=x_u8.device, dtype=torch.uint8)
    lab = None if labels is None else torch.empty(B, device=x_u8.device, dtype=torch.int64)
    C().conv_fwd(x_u8, idx, B, w.detach(), b.detach(), y, am, labels, lab)
    return (y, am) if labels is None else (y, am, lab)


def conv_front_fwd_multi(items, chunk: int = 8192):
    """Frozen-front forwards (no argmax) of several Alices, one launch per `chunk` rows for
    up to 16 of them: items [(x_u8, idx or None (rows 0 .. n), n, w, b)] -> [y [n, 5408]]."""
    outs = [torch.empty(int(n), CUT, device=x.device, dtype=torch.float32) for x, _, n, _, _ in items]
    for g in range(0, len(items), 16):
        C().conv_fwd_multi([(x, idx, int(n), w.detach(), b.detach(), y)
                            for (x, idx, n, w, b), y in zip(items[g:g + 16], outs[g:g + 16])], int(chunk))
    return outs


def conv_front_bwd(dy, y, am, x_u8, idx, w, b):
    """dW, db only (kind 0 writes the gradient into the state slot)."""
    B = int(idx.numel())
    dw = torch.empty_like(w)
    db = torch.empty_like(b)
    C().conv_bwd_step(dy, y, am, x_u8, idx, B, w.detach(), b.detach(), _slab(dy.device, B), dw, None, db, None,
                      *_opt_args(None, 0))
    return dw, db


def conv_front_bwd_step_(dy, y, am, x_u8, idx, w, b, cfg, st_w, st_b, t, dyn=None):
    """Per-sample dW partials (one workgroup per sample) + reduce/optimizer (one workgroup)."""
    B = int(idx.numel())
    C().conv_bwd_step(dy, y, am, x_u8, idx, B, w.detach(), b.detach(), _slab(dy.device, B), _s0(st_w), _s1(st_w),
                      _s0(st_b), _s1(st_b), *_opt_args(cfg, t, dyn))


def conv_front_fwd_pending(x_u8, idx, w, b, labels, pend):
    """(y, am, labels[idx]) with the deferred optimizer step `pend` = (slab, B, cfg, st_w,
    st_b, t) applied inside the kernel (not stored)."""
    B = int(idx.numel())
    dev = x_u8.device
    y = torch.empty(B, CUT, device=dev, dtype=torch.float32)
    am = torch.empty(B, CUT, device=dev, dtype=torch.uint8)
    lab = torch.empty(B, device=dev, dtype=torch.int64)
    slab, pB, cfg, st_w, st_b, t = pend
    C().conv_fwd_pending(x_u8, idx, B, w.detach(), b.detach(), y, am, labels, lab, slab, int(pB), _s0(st_w),
                         _s1(st_w), _s0(st_b), _s1(st_b), *_opt_args(cfg, t))
    return y, am, lab


def conv_front_bwd_defer_(dy, y, am, x_u8, idx, w, b, slab, pend, st_w, st_b):
    """This step's dW/db partials into `slab`, no update launch; the pending step `pend`
    (or None) is stored by the same launch."""
    B = int(idx.numel())
    if pend is None:
        C().conv_bwd_defer(dy, y, am, x_u8, idx, B, w.detach(), b.detach(), slab, None, 0, _s0(st_w), _s1(st_w),
                           _s0(st_b), _s1(st_b), *_opt_args(None, 0))
        return
    pslab, pB, cfg, pw, pb, t = pend
    C().conv_bwd_defer(dy, y, am, x_u8, idx, B, w.detach(), b.detach(), slab, pslab, int(pB), _s0(pw), _s1(pw),
                       _s0(pb), _s1(pb), *_opt_args(cfg, t))


def conv_apply_(pend, w, b):
    """Store a deferred client optimizer step."""
    slab, pB, cfg, st_w, st_b, t = pend
    C().conv_apply(slab, int(pB), w.detach(), b.detach(), _s0(st_w), _s1(st_w), _s0(st_b), _s1(st_b),
                   *_opt_args(cfg, t))


def conv_local_step_(x_u8, y_all, idx, w, b, cfg, st_w, st_b, t, loss_rows=None, dyn=None):
    """SISA client step in two kernels: gather+conv+pool+softmax-CE(5408)+dW partials,
    then reduce+optimizer.  Returns per-sample losses."""
    B = int(idx.numel())
    if loss_rows is None:
        loss_rows = torch.empty(B, device=x_u8.device, dtype=torch.float32)
    C().conv_local_step(x_u8, idx, y_all, B, w.detach(), b.detach(), _slab(x_u8.device, B), loss_rows,
                        _s0(st_w), _s1(st_w), _s0(st_b), _s1(st_b), *_opt_args(cfg, t, dyn))
    return loss_rows


def conv_local_epoch_(x_u8, y_all, order, B: int, w, b, cfg, st_w, st_b, t0: int):
    """ceil(n/B) SISA client steps over `order` in one host call (steps t0, t0+1, ...).
    Returns the per-sample losses [n]."""
    n = int(order.numel())
    loss_rows = torch.empty(n, device=x_u8.device, dtype=torch.float32)
    if n == 0:
        return loss_rows
    args = _opt_args(cfg, t0)
    ws = _workspace(x_u8.device, 2 * B * 320 + 2 * 960, "convepoch")
    C().conv_local_epoch(x_u8, order, y_all, int(B), w.detach(), b.detach(), _slab(x_u8.device, B), loss_rows,
                         _s0(st_w), _s1(st_w), _s0(st_b), _s1(st_b), *args[:7], int(t0), ws)
    return loss_rows


def conv_local_epoch_multi_(items, B: int, cfg):
    """Local epochs of several co-located Alices stepped together: one launch per step for all
    of them (csrc/conv.hip conv_local_epoch_multi).  items: [(x_u8, y_all, order, w, b, st_w,
    st_b, t0)], one per Alice, each with its own parameters and optimizer state.  Returns the
    per-sample losses of each Alice."""
    if not items:
        return []
    dev = items[0][0].device
    k = len(items)
    per = 2 * B * 320 + 2 * 960
    ws = _workspace(dev, k * per, "convmulti")
    nmax = max(-(-int(it[2].numel()) // B) for it in items)
    tb = C().alice_step_desc_bytes() * nmax * k
    table = _TABLE.get(dev)
    if table is None or table.numel() < tb:
        if table is not None:
            _WS_RETIRED.append(table)
        table = torch.empty(max(tb, 1 << 16), device=dev, dtype=torch.uint8)
        _TABLE[dev] = table
    alices, losses = [], []
    for a, (x, y_all, order, w, b, st_w, st_b, t0) in enumerate(items):
        loss = torch.empty(int(order.numel()), device=dev, dtype=torch.float32)
        losses.append(loss)
        alices.append((x, order, y_all, w.detach(), b.detach(), _s0(st_w), _s1(st_w), _s0(st_b), _s1(st_b),
                       ws[a * per:(a + 1) * per], loss, int(t0)))
    C().conv_local_epoch_multi(alices, int(B), KIND[cfg.kind], cfg.lr, cfg.beta1, cfg.beta2, cfg.eps,
                               cfg.weight_decay, cfg.momentum, table)
    return losses


_TABLE: dict = {}


# ---------------------------------------------------------------- linear
# training batches (M <= 128) run the skinny split-K kernels.  Many rows (evaluation over a
# test set, large batches): the forward product runs the in-tree LDS-tiled MFMA GEMM
# (csrc/gemm.hip, fused bias / ReLU / dropout epilogue) in fp32 and bf16 alike — 73-93 % of
# hipBLASLt's fp32 rate on the evaluation shapes (profiles/r3i_gemm_bench.txt; the evaluation
# phase is ~15 ms of a 5.8 s schedule, so the library's lead does not move the headline) —
# with variant 11 = 2 selecting hipBLASLt + the in-tree epilogue instead.  The data gradient
# of a batch past 128 rows (`--batch_size` > 128 only) has no in-tree NN-layout GEMM: it goes
# to hipBLASLt (variant 11 = 1: the skinny kernel, which re-reads W once per 16 rows).
LARGE_M = 128


def set_compute_dtype(dtype: str):
    """`--dtype`: GEMM operands in fp32 (exact) or bf16 (fp32 accumulation); master weights
    and optimizer state stay fp32."""
    C().set_compute_dtype(dtype)


def _library_gemm(M: int, dgrad: bool = False) -> bool:
    """Whether a product of M > 128 rows goes to hipBLASLt: only under variant 11 = 2 (the A/B
    slot of scripts/gemm_bench.py); never inside a HIP graph capture (the library may not
    allocate or initialise there).  Default: the in-tree tiled MFMA GEMMs (csrc/gemm.hip: the NT
    form for forwards, the NN form for data gradients)."""
    if M <= LARGE_M or torch.cuda.is_current_stream_capturing():
        return False
    return C().get_variant(11) == 2


def linear_fwd(x, w, b, relu: bool, drop_p: float, seed: int, col_offset: int = 0, out=None, dseed=None):
    M, N = x.shape[0], w.shape[0]
    if out is None:
        out = torch.empty(M, N, device=x.device, dtype=torch.float32)
    w = w.detach()
    bias = b.detach() if b is not None else None
    if _library_gemm(M):
        P = torch.mm(x, w.t())
        C().linear_epilogue(P, bias, out, relu, float(drop_p), seed & M64, col_offset, _ptr(dseed))
        return out
    if M <= LARGE_M:
        ws = _fwd_workspace(x.device, 16 * M * N)
    elif ((M + 255) // 256) * ((N + 127) // 128) < 512:
        ws = _workspace(x.device, 8 * M * N, "gemm")     # split-K slabs of the tiled GEMM (csrc/gemm.hip)
    else:
        # a large grid's last partial round split over K: at most one round of 256 x 128 slabs
        ws = _workspace(x.device, 1024 * 256 * 128, "gemm")
    C().linear_fwd(x, w, bias, out, relu, float(drop_p), seed & M64, col_offset, _ptr(dseed), ws)
    return out


def linear_epilogue(P, b, relu: bool, drop_p: float, seed: int, col_offset: int = 0, out=None, dseed=None):
    """P: [M, N] pre-activations or [S, M, N] split-K partial slabs (reduced here)."""
    if out is None:
        out = torch.empty(P.shape[-2:], device=P.device, dtype=torch.float32)
    C().linear_epilogue(P, b.detach() if b is not None else None, out, relu, float(drop_p), seed & M64, col_offset,
                        _ptr(dseed))
    return out


_WS: dict = {}
_WS_RETIRED: list = []


def _workspace(device, n, key="dgrad"):
    """Split-K / split-N partial-sum slabs.  Separate buffers per producer: slabs handed to
    a later fused consumer ("fc2p" -> server_head3, "dz1p" -> wgrad_group) must not be
    overwritten by the scratch use ("fwd", "dgrad") of the kernels launched in between.

    A buffer that was ever handed out is never freed: captured HIP graphs and native
    executors (engine/graphs.py, engine.cpp) hold its raw device address.  Growing a
    workspace retires the old buffer (kept alive here) and doubles the size, so a
    process retires at most a few buffers per key."""
    ws = _WS.get((device, key))
    if ws is None or ws.numel() < n:
        size = max(n, 1 << 20, 2 * ws.numel() if ws is not None else 0)
        if ws is not None:
            _WS_RETIRED.append(ws)
        ws = torch.empty(size, device=device, dtype=torch.float32)
        _WS[(device, key)] = ws
    return ws


def _fwd_workspace(device, n):
    return _workspace(device, n, "fwd")


def linear_dgrad(dz, w, h_prev=None, scale: float = 1.0, out=None, ws=None):
    M, K = dz.shape[0], w.shape[1]
    if out is None:
        out = torch.empty(M, K, device=dz.device, dtype=torch.float32)
    if M > LARGE_M and dz.shape[1] % 4 == 0 and K % 4 == 0 and C().get_compute_dtype() == "fp32":
        if _library_gemm(M, dgrad=True):
            # A/B only (variant 11 = 2): hipBLASLt product + the in-tree mask launch
            P = torch.mm(dz, w.detach())
            if h_prev is not None:               # scale belongs to the mask (dropout 1/(1-p))
                C().relu_mask(P, h_prev.contiguous(), float(scale), out)
            else:
                out.copy_(P)
            return out
        # many rows (large --batch_size, evaluation): the in-tree NN-layout MFMA GEMM
        # (csrc/gemm.hip gemm_nn_dgrad) with the previous layer's ReLU / dropout mask fused
        if ws is None and ((M + 127) // 128) * ((K + 127) // 128) < 384:
            ws = _workspace(dz.device, 8 * M * K, "gemm")
        C().gemm_nn_dgrad(dz, w.detach(), h_prev.contiguous() if h_prev is not None else None, float(scale), out, ws)
        return out
    if ws is None:
        ws = _workspace(dz.device, 16 * M * K)
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


def linear_wgrad_step_(dz, a, w, b, cfg, st_w, st_b, t, dyn=None):
    C().linear_wgrad_opt(dz, a, w.detach(), _s0(st_w), _s1(st_w), b.detach() if b is not None else None,
                         _s0(st_b) if b is not None else None, _s1(st_b) if b is not None else None,
                         *_opt_args(cfg, t, dyn))


def apply_update_(p, g, st, cfg, t):
    C().opt_flat(p.detach(), g, _s0(st), _s1(st), *_opt_args(cfg, t))


# ---------------------------------------------------------------- fused server step
def linear_fwd_partial(x, w, max_split: int = 16, key: str = "fc2p"):
    """x @ w.T as un-reduced split-K slabs [S, M, N] (S = 1: the plain product)."""
    M, N = x.shape[0], w.shape[0]
    ws = _workspace(x.device, 16 * M * N, key)
    S = C().linear_fwd_partial(x, w.detach(), ws, max_split)
    return ws[:S * M * N].view(S, M, N)


def server_head3(P2, b2, relu2: bool, drop2: float, seed2: int, W3, b3, labels, scale: float,
                 ignore_index: int = -100, dseed=None, groups: int = 1, gscale=None):
    """fc2 epilogue + fc3 + softmax-CE + fc3 dgrad + fc2 ReLU/dropout backward in one launch.
    `groups` > 1: the logits are that many cross-entropy groups (SISA-concat's heads) with
    labels [M, groups] and per-(row, group) scales `gscale` (else `scale`).
    Returns (h2, dlogits, dz2, loss_rows [M] or [M, groups])."""
    M, N2 = P2.shape[-2], P2.shape[-1]
    dev = P2.device
    h2 = torch.empty(M, N2, device=dev)
    dz2 = torch.empty(M, N2, device=dev)
    dlog = torch.empty(M, W3.shape[0], device=dev)
    loss = torch.empty(M, groups, device=dev) if groups > 1 else torch.empty(M, device=dev)
    ws = _workspace(dev, C().head3_slices(N2) * M * W3.shape[0], "head")
    C().server_head3(P2, b2.detach() if b2 is not None else None, relu2, float(drop2), seed2 & M64, _ptr(dseed),
                     W3.detach(), b3.detach() if b3 is not None else None, labels.reshape(-1), int(ignore_index),
                     float(scale), h2, dlog, dz2, loss, ws, int(groups),
                     gscale.reshape(-1).contiguous() if gscale is not None else None)
    return h2, dlog, dz2, loss


def lookahead_slabs(device, K0: int, mn: int, N0: int, tag: str = ""):
    """Workspace for wgrad_group_'s look-ahead forward: [ceil(K0/256), mn, N0]."""
    S = (K0 + 255) // 256
    return _workspace(device, S * mn * N0, "fc1n" + tag)[:S * mn * N0].view(S, mn, N0)


def wgrad_group_(layers, M: int, cfg, t: int, dyn=None, x_next=None, p_next=None):
    """Fused wgrad+optimizer of up to 3 layers in one launch.  Each layer:
    (dz, A, W, st_w, b, st_b).  With `x_next` (<= 64 rows), also writes layer 0's split-K
    partial pre-activations of the next batch under the *updated* weights into `p_next`
    (see lookahead_slabs)."""
    tup = []
    for dz, A, W, st_w, b, st_b in layers:
        tup.append((dz, A, W.detach(), _s0(st_w), _s1(st_w), b.detach() if b is not None else None,
                    _s0(st_b) if b is not None else None, _s1(st_b) if b is not None else None))
    C().wgrad_group(tup, int(M), x_next, p_next, *_opt_args(cfg, t, dyn))


# ---------------------------------------------------------------- loss / metrics
def softmax_ce(logits, labels, scale: float, ignore_index: int = -100, d_out=None, loss_out=None):
    M = logits.shape[0]
    loss = torch.empty(M, device=logits.device, dtype=torch.float32) if loss_out is None else loss_out
    d = torch.empty_like(logits) if d_out is None else d_out
    C().softmax_ce(logits, labels, int(ignore_index), float(scale), loss, d)
    return loss, d


def head_step_(x, W, b, labels, scale: float, cfg, st_w, st_b, t, ignore_index: int = -100,
               mask_by_input: bool = False):
    """One small Linear + CE layer's forward, softmax-CE, data gradient and optimizer step in
    one launch (the U-shape head on Alice).  Returns (loss_rows, dX); dX uses the weights
    before the update, and with `mask_by_input` is also masked by [x > 0] (the producer's
    ReLU backward)."""
    M = x.shape[0]
    loss = torch.empty(M, device=x.device, dtype=torch.float32)
    dx = torch.empty_like(x)
    C().head_step(x.contiguous(), W.detach(), b.detach() if b is not None else None, labels, int(ignore_index),
                  float(scale), bool(mask_by_input), loss, dx, _s0(st_w), _s1(st_w), _s0(st_b) if b is not None else None,
                  _s1(st_b) if b is not None else None, *_opt_args(cfg, t))
    return loss, dx


def relu_mask(d, h, scale: float = 1.0):
    """d * scale * [h > 0] (a layer's own ReLU/dropout backward)."""
    out = torch.empty_like(d)
    C().relu_mask(d.contiguous(), h.contiguous(), float(scale), out)
    return out


def eval_counters(logits, labels, omit_label: int, counters=None):
    if counters is None:
        counters = torch.zeros(6, device=logits.device, dtype=torch.int64)
    C().eval_counters(logits, labels, int(omit_label), counters)
    return counters
