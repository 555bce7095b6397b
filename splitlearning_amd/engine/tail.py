"""MLP-tail executor: Bob's server tail (optionally tensor-parallel) and the
U-shape head on Alice.

Reference semantics: `model2` / `model2_sisa` / `model2_sisa_concat` / `model3`
(models.py:33-94) trained with per-batch optimizer steps; the backward of Bob's
tail is what `dist_autograd.backward` ran on Bob (data_entities_vanilla.py:231)
and Bob's own `loss.backward(); optimizer.step()` in SISA
(data_entities_vanilla_sisa.py:305-313).

MI355X design:
* every Linear runs on the fused skinny kernels (fwd with bias/ReLU/dropout
  epilogue; dgrad with the previous layer's ReLU/dropout backward fused; wgrad
  fused into the optimizer so dW never touches HBM);
* backward is split in two phases — all dgrads first (`backward_dgrad`, which
  yields dL/d(cut activation) for the client as early as possible), then all
  wgrad+optimizer kernels (`backward_step`) — so the cut-layer gradient's
  transfer overlaps the parameter update (SURVEY §3.2 "legal overlap");
* tensor parallelism over a process group (Megatron-style, semantics-preserving):
  fc1 column-parallel (output features sharded, dropout mask hashed on the global
  column so it is TP-invariant), fc2 row-parallel (one all-reduce of the [B,·]
  partial sums per forward), fc3 replicated.  At TP degree T each GPU streams
  1/T of the fc1/fc2 weights and optimizer state — the HBM-bound part of the
  step — and at T >= 2 a shard of Bob's fp32 Adam state (384 MB in total) fits in
  the 256 MB Infinity Cache.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch

from .. import ops
from ..models.zoo import LinearSpec, TailSpec
from ..ops.rng import step_seed
from .slots import OptSlot


def _persist_workgroups(tail) -> int:
    """Workgroups of a persistent epoch launch: 0 = one per CU, launched cooperatively; a
    positive count (the ranks-share-one-GPU rehearsal, or SL_PERSIST_WORKGROUPS for profiling
    tools that cannot follow a cooperative launch) = that many, plain launch."""
    n = int(getattr(tail, "resident_workgroups", 0))
    return n if n > 0 else int(os.environ.get("SL_PERSIST_WORKGROUPS", "0"))


@dataclass
class _Layer:
    spec: LinearSpec
    style: str               # "rep" | "col" | "row"
    W: torch.Tensor          # [N_local, K_local]
    b: torch.Tensor          # [N_local]
    col_off: int             # global index of local output column 0
    in_off: int              # global index of local input column 0 (row-parallel)


class TailEngine:
    def __init__(self, module: torch.nn.Module, spec: TailSpec, device: torch.device,
                 tp_rank: int = 0, tp_size: int = 1, allreduce=None, seed_base: int = 0, ws_tag: str = ""):
        """`ws_tag`: private scratch / hand-off buffers for this engine (several shards of one
        tail living in one process: the single-process TP emulation, `emulate_tp_epoch`)."""
        self.spec = spec
        self.ws_tag = ws_tag
        self.device = device
        self.ops = ops.impl(device)
        self.tp_rank, self.tp_size = tp_rank, tp_size
        self.allreduce = allreduce
        self.seed_base = seed_base
        self.training = True
        self.fwd_count = 0
        self.module = module
        self.layers: list[_Layer] = []
        lin = module.linears()
        nl = len(lin)
        for i, (ls, mod) in enumerate(zip(spec.layers, lin)):
            style = "rep"
            if tp_size > 1 and nl >= 2:
                style = "col" if i == 0 else ("row" if i == 1 else "rep")
            W, b = mod.weight.data, mod.bias.data
            col_off = in_off = 0
            if style == "col":
                n = W.shape[0]
                s, e = _shard_range(n, tp_rank, tp_size)
                W, b, col_off = W[s:e], b[s:e], s
            elif style == "row":
                k = W.shape[1]
                s, e = _shard_range(k, tp_rank, tp_size)
                W, in_off = W[:, s:e], s
            W = W.to(device).contiguous()
            b = b.to(device).contiguous()
            if tp_size == 1:
                # the module's parameters *are* the device tensors (state_dict works directly)
                mod.weight.data = W
                mod.bias.data = b
            self.layers.append(_Layer(ls, style, W, b, col_off, in_off))
        self.acts: list[torch.Tensor] = []
        self.dz: list[torch.Tensor] = []
        self._train_fwd = False
        self._pre = None          # pending look-ahead fc1 partial slabs (see fused_step)
        # cross-entropy groups of the last layer's outputs (SISA-concat: one 100-way head per
        # client, protocols/concat.py); 1 = one softmax over all outputs
        self.ce_groups = 1

    # ------------------------------------------------------------------ forward
    def forward(self, x: torch.Tensor, train: bool | None = None, dseeds=None, pre: bool = False) -> torch.Tensor:
        """`dseeds[i]` (graph replay only): device int32[2] holding layer i's dropout seed.
        `pre`: layer 0's product for `x` was formed by the previous `group_step(x_next=x)`;
        only its epilogue runs here."""
        train = self.training if train is None else train
        self.fwd_count += 1
        step = self.fwd_count
        acts = [x]
        h = x
        P0 = None
        if pre:
            P0, self._pre = self._pre, None
            assert P0 is not None and P0.shape[1] == x.shape[0], "no pending look-ahead for this batch"
        for i, L in enumerate(self.layers):
            ls = L.spec
            drop = ls.dropout if train else 0.0
            seed = step_seed(self.seed_base, i, step)
            kw = {} if dseeds is None else {"dseed": dseeds[i]}
            if i == 0 and pre:
                h = self.ops.linear_epilogue(P0, L.b, ls.relu, drop, seed, L.col_off, **kw)
            elif L.style == "row":
                part = self.ops.linear_fwd(h, L.W, None, False, 0.0, 0, 0)
                self.allreduce(part)
                h = self.ops.linear_epilogue(part, L.b, ls.relu, drop, seed, 0, **kw)
            else:
                h = self.ops.linear_fwd(h, L.W, L.b, ls.relu, drop, seed, L.col_off, **kw)
            acts.append(h)
        self.acts = acts
        self._train_fwd = train
        return h

    __call__ = forward

    def forward_block(self, x: torch.Tensor, k_off: int, out_off: int, out_len: int) -> torch.Tensor:
        """Inference (no dropout) of the tail on an input that is non-zero only in layer 0's
        input columns [k_off, k_off + x.shape[1]), returning only the last layer's outputs
        [out_off, out_off + out_len): layer 0 multiplies just that column block of its weight
        and the last layer just those rows.  SISA-concat evaluation (protocols/concat.py):
        Alice j's activation in slot j, zeros elsewhere, read head j — without forming the
        zero-padded [rows, 5408 k] input or the other k - 1 heads."""
        self.fwd_count += 1
        h = x
        n = len(self.layers)
        for i, L in enumerate(self.layers):
            ls = L.spec
            W, b = L.W, L.b
            if i == 0:
                W = W[:, k_off:k_off + x.shape[1]]
            if i == n - 1:
                W, b = W[out_off:out_off + out_len], b[out_off:out_off + out_len]
            if L.style == "row":
                part = self.ops.linear_fwd(h, W, None, False, 0.0, 0, 0)
                self.allreduce(part)
                h = self.ops.linear_epilogue(part, b, ls.relu, 0.0, 0, 0)
            else:
                h = self.ops.linear_fwd(h, W, b, ls.relu, 0.0, 0, L.col_off)
        self.acts = []
        return h

    # ------------------------------------------------------------------ backward
    def backward_dgrad(self, dout: torch.Tensor, need_dx: bool, premasked: bool = False):
        """Phase 1: all data gradients.  Returns dL/dx (a *partial sum* across TP
        ranks when fc1 is column-parallel) if `need_dx`, else None.  `premasked`: the
        consumer already applied this tail's final ReLU backward (no active dropout)."""
        L = self.layers
        n = len(L)
        last = L[-1].spec
        dz = dout
        drop_on = bool(last.dropout and self._train_fwd)
        if premasked and not drop_on:
            pass
        elif last.relu or drop_on:
            scale = 1.0 / (1.0 - last.dropout) if (last.dropout and self._train_fwd) else 1.0
            dz = self.ops.relu_mask(dout, self.acts[-1], scale)
        dzs = [None] * n
        dzs[n - 1] = dz
        dx = None
        for i in range(n - 1, -1, -1):
            if i > 0:
                prev = L[i - 1].spec
                drop_on = prev.dropout > 0 and self._train_fwd
                scale = 1.0 / (1.0 - prev.dropout) if drop_on else 1.0
                hprev = self.acts[i] if (prev.relu or drop_on) else None
                dzs[i - 1] = self.ops.linear_dgrad(dzs[i], L[i].W, hprev, scale)
            elif need_dx:
                dx = self.ops.linear_dgrad(dzs[0], L[0].W, None, 1.0)
        self.dz = dzs
        return dx

    def backward_step(self, slot: OptSlot, t: int | None = None, prefix: str = "", dyn=None):
        """Phase 2: fused wgrad + optimizer update of every layer (one optimizer step).
        `dyn` (graph replay only): device float[2] with Adam's {step_size, 1/sqrt(bc2)}."""
        self._pre = None
        t = slot.tick() if t is None else t
        kw = {} if dyn is None else {"dyn": dyn}
        for i, L in enumerate(self.layers):
            self.ops.linear_wgrad_step_(self.dz[i], self.acts[i], L.W, L.b, slot.cfg,
                                        slot.state(f"{prefix}{L.spec.name}.weight", L.W),
                                        slot.state(f"{prefix}{L.spec.name}.bias", L.b), t, **kw)
        self.dz = []

    def grouped_ok(self, m: int = 0) -> bool:
        """Whether `group_step` can run (HIP backend, <= 3 layers); with `m`, also whether it
        can form the next batch's layer-0 product for m rows (look-ahead)."""
        ok = hasattr(self.ops, "wgrad_group_") and 0 < len(self.layers) <= 3
        if m:
            ok = ok and hasattr(self.ops, "lookahead_slabs") and 0 < m <= 64
        return ok

    def group_step(self, slot: OptSlot, t: int | None = None, prefix: str = "", x_next=None):
        """`backward_step` in ONE launch (every layer's wgrad + optimizer, wgrad_group_), after
        `backward_dgrad`.  `x_next`: also form the next batch's layer-0 product with the updated
        weights, consumed by `forward(x_next, pre=True)` (no separate read of W0)."""
        t = slot.tick() if t is None else t
        layers = [(self.dz[i], self.acts[i], L.W, slot.state(f"{prefix}{L.spec.name}.weight", L.W),
                   L.b, slot.state(f"{prefix}{L.spec.name}.bias", L.b)) for i, L in enumerate(self.layers)]
        pn = None
        if x_next is not None:
            assert self.grouped_ok(x_next.shape[0])
            pn = self.lookahead_slabs(x_next.shape[0])
        self.ops.wgrad_group_(layers, self.acts[0].shape[0], slot.cfg, t, None, x_next=x_next, p_next=pn)
        self._pre = pn
        self.dz = []

    # ------------------------------------------------------------------ fused one-layer head step
    def head_step_ok(self, m: int) -> bool:
        """A single Linear layer (no ReLU / dropout) small enough for `_C.head_step`: the
        U-shape head (reference model3, 100 -> 10)."""
        if not hasattr(self.ops, "head_step_") or len(self.layers) != 1:
            return False
        L = self.layers[0]
        n, k = L.W.shape
        return (not L.spec.relu and L.spec.dropout == 0 and self.tp_size == 1
                and m * k <= 4096 and n * k <= 4096 and m * n <= 1024)

    def head_step(self, x, labels, slot: OptSlot, t: int, prefix: str = "", mask_input: bool = False):
        """forward + softmax-CE (mean) + dL/dx + optimizer step of the one-layer head in one
        launch; same math as forward / softmax_ce / backward_dgrad / backward_step.
        `mask_input`: dL/dx also gets the producer's ReLU backward ([x > 0]).
        Returns (per-row loss, dL/dx)."""
        L = self.layers[0]
        self.fwd_count += 1
        loss, dx = self.ops.head_step_(x, L.W, L.b, labels, 1.0 / x.shape[0], slot.cfg,
                                       slot.state(f"{prefix}{L.spec.name}.weight", L.W),
                                       slot.state(f"{prefix}{L.spec.name}.bias", L.b), t,
                                       mask_by_input=mask_input)
        self.acts, self.dz = [], []
        return loss, dx

    # ------------------------------------------------------------------ fused 3-layer step
    def fused3_ok(self) -> bool:
        """The SISA/vanilla server tail (fc1 ReLU+Dropout, fc2 ReLU+Dropout, fc3 -> CE) on the
        fused HIP kernels: 7-8 launches per step instead of 13 (csrc/fused.hip)."""
        if not hasattr(self.ops, "server_head3") or len(self.layers) != 3:
            return False
        s = [L.spec for L in self.layers]
        return (s[0].relu and s[1].relu and not s[2].relu and s[2].dropout == 0
                and self.layers[2].style == "rep" and s[1].out_features % 4 == 0)

    def lookahead_ok(self, m: int) -> bool:
        """Whether `fused_step(x_next=...)` can pre-compute the next batch's fc1 product."""
        return self.fused3_ok() and hasattr(self.ops, "lookahead_slabs") and 0 < m <= 64

    def lookahead_slabs(self, m: int):
        L1 = self.layers[0]
        if self.ws_tag:
            return self.ops.lookahead_slabs(self.device, L1.W.shape[1], m, L1.W.shape[0], self.ws_tag)
        return self.ops.lookahead_slabs(self.device, L1.W.shape[1], m, L1.W.shape[0])

    def lookahead_prologue(self, x0, out=None):
        """Start a look-ahead chain: fc1's product for the first batch, in slab form (into
        `out` when given: a captured graph's own slab buffer)."""
        L1 = self.layers[0]
        p = self.lookahead_slabs(x0.shape[0]) if out is None else out
        p.zero_()
        p[0].copy_(self.ops.linear_fwd(x0, L1.W, None, False, 0.0, 0, 0))
        self._pre = p

    def train_fwd_bwd3(self, x, labels, need_dx: bool, dseeds=None, pre: bool = False, gscale=None):
        """Training forward + softmax-CE + all data gradients of the 3-layer tail.
        Returns (per-row loss, dL/dx or None); `fused_step` then applies the optimizer.
        `pre`: fc1's product for `x` was already computed by the previous step's
        `fused_step(x_next=x)` (or `lookahead_prologue(x)`); only its epilogue runs here.
        With `ce_groups` = G > 1 (SISA-concat), labels and `gscale` are [M, G]."""
        ops = self.ops
        L1, L2, L3 = self.layers
        M = x.shape[0]
        self.fwd_count += 1
        seeds = [step_seed(self.seed_base, i, self.fwd_count) for i in range(3)]

        def ds(i):
            return {} if dseeds is None else {"dseed": dseeds[i]}
        p1, p2 = L1.spec.dropout, L2.spec.dropout
        P2 = None
        if pre:
            P1 = self._pre
            assert P1 is not None and P1.shape[1] == M, "no pending look-ahead for this batch"
            self._pre = None
            h1 = ops.linear_epilogue(P1, L1.b, True, p1, seeds[0], L1.col_off, **ds(0))
        else:
            self._pre = None
            h1 = ops.linear_fwd(x, L1.W, L1.b, True, p1, seeds[0], L1.col_off, **ds(0))
        if L2.style == "row":
            if L2.W.shape[1] <= 1280:
                # small K shard (TP >= 4): one unsplit product, all-reduced as is — no
                # split-K reduce launch before the collective
                P2 = ops.linear_fwd_partial(h1, L2.W, max_split=1)
            else:
                P2 = ops.linear_fwd(h1, L2.W, None, False, 0.0, 0, 0)
            self.allreduce(P2)
        else:
            P2 = ops.linear_fwd_partial(h1, L2.W)
        G = self.ce_groups
        kw = ds(1) if G == 1 else dict(ds(1), groups=G, gscale=gscale)
        h2, dlog, dz2, loss = ops.server_head3(P2, L2.b, True, p2, seeds[1], L3.W, L3.b, labels, 1.0 / M, **kw)
        s1 = 1.0 / (1.0 - p1) if p1 else 1.0
        dx = None
        # dz1 is materialised (split-N dgrad + reduce/mask kernel): reducing the split-N
        # slabs inside the wgrad staging (every slab load issued at once) measured 250 vs
        # 185 us per step at TP = 1 and 62 vs 56 at TP = 8: all ~8000 workgroups re-read
        # the slabs of their 16 columns, ~9x the L2 traffic of reading dz1, on every
        # workgroup's critical path.
        dz1 = ops.linear_dgrad(dz2, L2.W, h1, s1)
        if need_dx:
            dx = ops.linear_dgrad(dz1, L1.W, None, 1.0)
        self.acts = [x, h1, h2]
        self._wg = [(dz1, x), (dz2, h1), (dlog, h2)]
        self._train_fwd = True
        return loss, dx

    def fused_step(self, slot: OptSlot, t: int | None = None, dyn=None, prefix: str = "", x_next=None):
        """Optimizer step of all three layers in one launch.  `x_next`: the next batch's
        input; while each fc1 weight tile is in registers after its update, the kernel also
        forms that tile's share of x_next @ W1_new^T, so the next step reads W1 once instead
        of twice (fc1's 108 MB forward read disappears; train_fwd_bwd3(pre=True) consumes)."""
        t = slot.tick() if t is None else t
        layers = []
        for (dz, A), L in zip(self._wg, self.layers):
            layers.append((dz, A, L.W, slot.state(f"{prefix}{L.spec.name}.weight", L.W), L.b,
                           slot.state(f"{prefix}{L.spec.name}.bias", L.b)))
        pn = None
        if x_next is not None:
            assert self.lookahead_ok(x_next.shape[0])
            pn = self.lookahead_slabs(x_next.shape[0])
        self.ops.wgrad_group_(layers, self.acts[0].shape[0], slot.cfg, t, dyn, x_next=x_next, p_next=pn)
        self._pre = pn
        self._wg = []

    # ------------------------------------------------------------------ native epoch executor
    def native_epoch_ok(self, B: int) -> bool:
        """Whether `run_native_epoch` can drive this tail: the fused 3-layer HIP path with
        the look-ahead, and (tensor-parallel) the native RCCL communicator."""
        if self.device.type != "cuda" or not self.lookahead_ok(B) or not hasattr(self.ops, "C"):
            return False
        if self.layers[1].style == "row":
            return (getattr(self.allreduce, "comm", None) is not None
                    or getattr(self.allreduce, "ipc", None) is not None)
        return self.tp_size == 1

    def run_native_epoch(self, acts: torch.Tensor, labels: torch.Tensor, slot: OptSlot, B: int, pre: bool,
                         lookahead: bool = True, gscale: torch.Tensor | None = None) -> torch.Tensor:
        """One epoch of fused server steps over `acts`/`labels` (batches of B, last one
        partial) issued from C++ (`_C.ServerEpoch`, csrc/engine.cpp): the same launches,
        seeds and step counts as looping `train_fwd_bwd3` + `fused_step`, without a
        Python round trip per step.  `pre`: the first batch's fc1 product is pending
        (`lookahead_prologue`).  With `ce_groups` = G > 1 (SISA-concat), labels and `gscale`
        (each row-and-group's loss scale) are [n, G].  Returns the per-row losses ([n, G])."""
        ex = self._native_executor(slot, B)
        d = self._native[3]
        if pre:
            assert self._pre is not None and self._pre.data_ptr() == d["pn"].data_ptr(), \
                "pending look-ahead is not in the executor's slab buffer"
        G = self.ce_groups
        loss = torch.empty((acts.shape[0], G) if G > 1 else acts.shape[0], device=self.device)
        fc, t, pre = ex.run(acts, labels.reshape(-1), loss, self.seed_base, self.fwd_count, slot.t, pre, lookahead,
                            gscale.reshape(-1).contiguous() if gscale is not None else None)
        self.fwd_count, slot.t = int(fc), int(t)
        # the executor's own slab buffer holds the pending product (not a re-fetched one)
        self._pre = d["pn"] if pre else None
        return loss

    def _native_executor(self, slot: OptSlot, B: int):
        cached = getattr(self, "_native", None)
        # the executor holds raw workspace addresses: rebuild it when a workspace it uses
        # has been replaced (grown) since it was built
        if (cached is not None and cached[0] is slot and cached[1] == B and cached[3]["groups"] == self.ce_groups
                and cached[3]["pn"].data_ptr() == self.lookahead_slabs(B).data_ptr()):
            return cached[2]
        ops, dev = self.ops, self.device
        L1, L2, L3 = self.layers
        N1, N2, C = L1.W.shape[0], L2.W.shape[0], L3.W.shape[0]
        layers = []
        for L in self.layers:
            sw, sb = slot.state(f"{L.spec.name}.weight", L.W), slot.state(f"{L.spec.name}.bias", L.b)
            layers.append({"W": L.W, "b": L.b, "s0": sw.get("m", sw.get("buf")), "s1": sw.get("v"),
                           "sb0": sb.get("m", sb.get("buf")), "sb1": sb.get("v")})
        cfg = slot.cfg
        kmax = max(L.W.shape[1] for L in self.layers)
        nmax = max(L.W.shape[0] for L in self.layers)
        tg = self.ws_tag
        d = {"layers": layers, "kind": {"sgd": 1, "adam": 2}[cfg.kind], "lr": cfg.lr, "beta1": cfg.beta1,
             "beta2": cfg.beta2, "eps": cfg.eps, "wd": cfg.weight_decay, "momentum": cfg.momentum,
             "p1": L1.spec.dropout, "p2": L2.spec.dropout, "col_off1": L1.col_off, "row2": L2.style == "row",
             "comm": getattr(self.allreduce, "comm", None) if L2.style == "row" else None,
             "ipc": getattr(self.allreduce, "ipc", None) if L2.style == "row" else None, "B": B,
             "groups": self.ce_groups,
             "emulate_tp": L2.style == "row" and self.allreduce is None,
             "pn": self.lookahead_slabs(B),
             "p2ws": ops._workspace(dev, 16 * B * N2, "fc2p" + tg),
             "fwdws": ops._workspace(dev, 16 * B * nmax, "fwd" + tg),
             "dgws": ops._workspace(dev, 16 * B * kmax, "dgrad" + tg),
             "headws": ops._workspace(dev, ops.C().head3_slices(N2) * B * C, "head" + tg),
             "h1": torch.empty(B, N1, device=dev), "h2": torch.empty(B, N2, device=dev),
             "dz1": torch.empty(B, N1, device=dev), "dz2": torch.empty(B, N2, device=dev),
             "dlog": torch.empty(B, C, device=dev)}
        ex = ops.C().ServerEpoch(d)
        self._native = (slot, B, ex, d)      # d keeps the workspaces alive
        return ex

    # ------------------------------------------------------------------ register-resident epoch
    def resident_ok(self, slot: OptSlot, B: int) -> bool:
        """Whether `run_resident_epoch` can drive this shard (`_C.ResidentEpoch`,
        csrc/resident.hip): the fused 3-layer tail with one cross-entropy group, <= 16 rows
        per step, an fc1 shard of <= 768 rows (a TP >= 7 shard of model2_sisa) whose state
        fits the chip's registers and LDS, and, tensor-parallel, the peer-mapped region."""
        if (self.device.type != "cuda" or not self.fused3_ok() or not hasattr(self.ops, "C")
                or self.ce_groups != 1 or not 1 <= B <= 16 or self.layers[0].W.shape[0] > 768):
            return False
        if self.layers[1].style == "row" and getattr(self.allreduce, "ipc", None) is None:
            return False
        return self._resident_executor(slot, B).ok()

    def run_resident_epoch(self, acts: torch.Tensor, labels: torch.Tensor, slot: OptSlot, B: int,
                           step_rows=None) -> torch.Tensor:
        """One epoch over `acts` / `labels` with every full batch in ONE persistent launch that
        keeps this shard's weights and optimizer state on-chip (csrc/resident.hip); a trailing
        partial batch runs on the launch-per-stage executor.  `step_rows`: the plan of
        `padded_plan` (every step's real rows; acts / labels padded to B rows per step): every
        step, short ones included, in the launch.  Same step / seed / Adam-count bookkeeping as
        `run_native_epoch`; the sums run in another order, so results agree with it to fp32
        rounding, not bitwise.  Returns the per-row losses."""
        ex = self._resident_executor(slot, B)
        n = acts.shape[0]
        loss = torch.empty(n, device=self.device)
        fc, t, done = ex.run(acts, labels, loss, self.seed_base, self.fwd_count, slot.t, None, step_rows)
        self.fwd_count, slot.t = int(fc), int(t)
        self._pre = None
        if done < n:
            rest_a, rest_y = acts[done:], labels[done:]
            if self.native_epoch_ok(B):
                loss[done:] = self.run_native_epoch(rest_a, rest_y, slot, B, False)
            else:
                loss[done:], _ = self.train_fwd_bwd3(rest_a, rest_y, need_dx=False)
                self.fused_step(slot)
        return loss

    def _resident_executor(self, slot: OptSlot, B: int):
        cached = getattr(self, "_resident", None)
        if cached is not None and cached[0] is slot and cached[1] == B:
            return cached[2]
        L1, L2, _ = self.layers
        layers = []
        for L in self.layers:
            sw, sb = slot.state(f"{L.spec.name}.weight", L.W), slot.state(f"{L.spec.name}.bias", L.b)
            layers.append({"W": L.W, "b": L.b, "s0": sw.get("m", sw.get("buf")), "s1": sw.get("v"),
                           "sb0": sb.get("m", sb.get("buf")), "sb1": sb.get("v")})
        cfg = slot.cfg
        d = {"layers": layers, "kind": {"sgd": 1, "adam": 2}[cfg.kind], "lr": cfg.lr, "beta1": cfg.beta1,
             "beta2": cfg.beta2, "eps": cfg.eps, "wd": cfg.weight_decay, "momentum": cfg.momentum,
             "p1": L1.spec.dropout, "p2": L2.spec.dropout, "col_off1": L1.col_off, "B": B,
             "ipc": getattr(self.allreduce, "ipc", None) if L2.style == "row" else None,
             "timeout_s": float(getattr(self, "resident_timeout_s", 10.0)),
             "workgroups": _persist_workgroups(self)}
        ex = self.ops.C().ResidentEpoch(d)
        self._resident = (slot, B, ex, d)
        return ex

    # ------------------------------------------------------------------ hybrid epoch
    def hybrid_ok(self, slot: OptSlot, B: int) -> bool:
        """Whether `run_hybrid_epoch` can drive this shard (`_C.HybridEpoch`, csrc/hybrid.hip):
        the fused 3-layer tail with one cross-entropy group, <= 16 rows per step, a WIDE shard
        (fc1 shard <= 5120 rows in 8 x 32 fc2 tiles of <= 128 x 160, fc2 <= 1024 rows, <= 128
        classes) and, tensor-parallel, the peer-mapped region for the in-launch exchange."""
        if (self.device.type != "cuda" or not self.fused3_ok() or not hasattr(self.ops, "C")
                or self.ce_groups != 1 or not 1 <= B <= 16):
            return False
        if self.layers[1].style == "row" and getattr(self.allreduce, "ipc", None) is None:
            return False
        return self._hybrid_executor(slot, B).ok()

    def run_hybrid_epoch(self, acts: torch.Tensor, labels: torch.Tensor, slot: OptSlot, B: int,
                         step_rows=None) -> torch.Tensor:
        """One epoch over `acts` / `labels` with every full batch in ONE persistent launch that
        keeps fc2 / fc3 and the biases on-chip and streams fc1 (csrc/hybrid.hip); a trailing
        partial batch runs on the launch-per-stage executor.  `step_rows`: as
        `run_resident_epoch`.  Same step / seed / Adam-count bookkeeping as `run_native_epoch`;
        the sums run in another order, so results agree with it to fp32 rounding, not bitwise.
        Returns the per-row losses."""
        ex = self._hybrid_executor(slot, B)
        n = acts.shape[0]
        loss = torch.empty(n, device=self.device)
        fc, t, done = ex.run(acts, labels, loss, self.seed_base, self.fwd_count, slot.t, None, None, 0, step_rows)
        self.fwd_count, slot.t = int(fc), int(t)
        self._pre = None
        if done < n:
            rest_a, rest_y = acts[done:], labels[done:]
            if self.native_epoch_ok(B):
                loss[done:] = self.run_native_epoch(rest_a, rest_y, slot, B, False)
            else:
                loss[done:], _ = self.train_fwd_bwd3(rest_a, rest_y, need_dx=False)
                self.fused_step(slot)
        return loss

    def _hybrid_executor(self, slot: OptSlot, B: int):
        cached = getattr(self, "_hybrid", None)
        if cached is not None and cached[0] is slot and cached[1] == B:
            return cached[2]
        L1, L2, _ = self.layers
        layers = []
        for L in self.layers:
            sw, sb = slot.state(f"{L.spec.name}.weight", L.W), slot.state(f"{L.spec.name}.bias", L.b)
            layers.append({"W": L.W, "b": L.b, "s0": sw.get("m", sw.get("buf")), "s1": sw.get("v"),
                           "sb0": sb.get("m", sb.get("buf")), "sb1": sb.get("v")})
        cfg = slot.cfg
        d = {"layers": layers, "kind": {"sgd": 1, "adam": 2}[cfg.kind], "lr": cfg.lr, "beta1": cfg.beta1,
             "beta2": cfg.beta2, "eps": cfg.eps, "wd": cfg.weight_decay, "momentum": cfg.momentum,
             "p1": L1.spec.dropout, "p2": L2.spec.dropout, "col_off1": L1.col_off, "B": B,
             "ipc": getattr(self.allreduce, "ipc", None) if L2.style == "row" else None,
             "timeout_s": float(getattr(self, "resident_timeout_s", 10.0)),
             "workgroups": _persist_workgroups(self), "nt_stores": getattr(self, "hybrid_nt_stores", None),
             "chunk_steps": getattr(self, "hybrid_chunk_steps", None)}
        ex = self.ops.C().HybridEpoch(d)
        self._hybrid = (slot, B, ex, d)
        return ex

    # ------------------------------------------------------------------ persistent-epoch rollback
    def snapshot_state(self, slot: OptSlot, buf: dict | None = None) -> dict:
        """Device-to-device copy of this shard's weights, biases and optimizer state in `slot`
        plus the step / dropout counters, into `buf` (reused across epochs: one allocation of
        the shard's size, ~390 MB at TP = 1, copied at HBM rate, ~0.1 ms).  A persistent epoch
        that fails mid-launch has updated part of W / m / v; `restore_state` undoes it."""
        buf = {} if buf is None else buf
        ts = []
        for L in self.layers:
            ts += [L.W, L.b]
            for nm, p in ((f"{L.spec.name}.weight", L.W), (f"{L.spec.name}.bias", L.b)):
                ts += [slot.state(nm, p)[k] for k in sorted(slot.state(nm, p))]
        with torch.no_grad():
            for i, t in enumerate(ts):
                c = buf.get(i)
                if c is None or c.shape != t.shape or c.device != t.device:
                    c = buf[i] = torch.empty_like(t)
                c.copy_(t)
        buf["tensors"] = ts
        buf["counters"] = (self.fwd_count, slot.t)
        return buf

    def restore_state(self, slot: OptSlot, buf: dict):
        with torch.no_grad():
            for i, t in enumerate(buf["tensors"]):
                t.copy_(buf[i])
        self.fwd_count, slot.t = buf["counters"]
        self._pre = None
        self.acts, self.dz, self._wg = [], [], []

    @staticmethod
    def padded_plan(caches, B: int, ignore: int = -100):
        """One server epoch over several clients' cached (acts, labels), in order, as one
        persistent-launch input: every client's batches of B rows, its short final batch
        zero-padded to B rows with ignored labels.  Returns (acts [S B, K], labels [S B],
        step_rows [S]); the persistent kernels take each step's CE mean over its real rows, and
        a padded row adds exact zeros to every gradient, so the steps are the reference's
        (data_entities_vanilla_sisa.py:298-313: `for cid: for batch in cid's loader: step`).
        A single client with whole batches is returned as is (no copy)."""
        rows = []
        for a, y in caches:
            n = int(y.numel())
            rows += [B] * (n // B) + ([n % B] if n % B else [])
        if len(caches) == 1 and caches[0][1].numel() % B == 0:
            a, y = caches[0]
            return a, y, rows
        S = len(rows)
        a0 = caches[0][0]
        X = torch.zeros(S * B, a0.shape[1], device=a0.device, dtype=a0.dtype)
        Y = torch.full((S * B,), ignore, device=a0.device, dtype=torch.int64)
        s = 0
        for a, y in caches:
            n = int(y.numel())
            full = n - n % B
            X[s * B:s * B + full] = a[:full]
            Y[s * B:s * B + full] = y[:full]
            s += full // B
            if n % B:
                X[s * B:s * B + n % B] = a[full:]
                Y[s * B:s * B + n % B] = y[full:]
                s += 1
        return X, Y, rows

    # ------------------------------------------------------------------ TP emulation
    @staticmethod
    def emulate_tp_epoch(shards: list, slots: list, acts: torch.Tensor, labels: torch.Tensor, B: int,
                         lookahead: bool = True) -> torch.Tensor:
        """One server epoch of a tensor-parallel tail emulated in ONE process: `shards` are the
        T TailEngines of one tail (tp_rank 0..T-1, `allreduce=None`, distinct `ws_tag`s), each
        with its own optimizer slot.  The production native executor (`_C.ServerEpoch`) runs
        every shard; `_C.tp_emulate_epoch` steps them in lock step and stands in for RCCL's
        all-reduce of the row-parallel fc2 products.  Returns shard 0's per-row losses."""
        t0 = shards[0]
        exs = [sh._native_executor(sl, B) for sh, sl in zip(shards, slots)]
        pre = False
        if lookahead and acts.shape[0] >= B:
            for sh in shards:
                sh.lookahead_prologue(acts[:B], out=sh._native[3]["pn"])
            pre = True
        losses = [torch.empty(acts.shape[0], device=t0.device) for _ in shards]
        fc, t, pre = t0.ops.C().tp_emulate_epoch(exs, acts, labels, losses, t0.seed_base, t0.fwd_count,
                                                  slots[0].t, pre, lookahead)
        for sh, sl in zip(shards, slots):
            sh.fwd_count, sl.t = int(fc), int(t)
            sh._pre = None
        return losses[0]

    # ------------------------------------------------------------------ state
    def local_state(self) -> dict:
        out = {}
        for L in self.layers:
            out[f"{L.spec.name}.weight"] = L.W
            out[f"{L.spec.name}.bias"] = L.b
        return out

    def full_state_dict(self, gather=None) -> dict:
        """Reference-layout state_dict (full tensors).  `gather(t) -> list[t]` collects the
        TP shards (all ranks must call it)."""
        sd = {}
        for L in self.layers:
            W, b = L.W, L.b
            if L.style == "col":
                W = torch.cat(gather(W), 0)
                b = torch.cat(gather(b), 0)
            elif L.style == "row":
                W = torch.cat(gather(W.t().contiguous()), 0).t()
            sd[f"{L.spec.name}.weight"] = W.detach().cpu().clone()
            sd[f"{L.spec.name}.bias"] = b.detach().cpu().clone()
        return sd

    def load_full_state_dict(self, sd: dict):
        self._pre = None
        with torch.no_grad():
            for L in self.layers:
                W = sd[f"{L.spec.name}.weight"]
                b = sd[f"{L.spec.name}.bias"]
                if L.style == "col":
                    s, e = _shard_range(W.shape[0], self.tp_rank, self.tp_size)
                    W, b = W[s:e], b[s:e]
                elif L.style == "row":
                    s, e = _shard_range(W.shape[1], self.tp_rank, self.tp_size)
                    W = W[:, s:e]
                L.W.copy_(W)
                L.b.copy_(b)

    def flat_weights(self) -> torch.Tensor:
        return torch.cat([t.reshape(-1) for L in self.layers for t in (L.W, L.b)])

    def load_flat_weights(self, flat: torch.Tensor):
        self._pre = None
        o = 0
        for L in self.layers:
            for t in (L.W, L.b):
                t.copy_(flat[o:o + t.numel()].view_as(t))
                o += t.numel()

    @property
    def flat_numel(self) -> int:
        return sum(t.numel() for L in self.layers for t in (L.W, L.b))

    def reset_parameters(self):
        self._pre = None
        for L, mod in zip(self.layers, self.module.linears()):
            if self.tp_size == 1:
                mod.reset_parameters()
            else:
                raise NotImplementedError("reset of a tensor-parallel tail")


def _shard_range(n: int, r: int, t: int) -> tuple[int, int]:
    """Contiguous, 4-aligned shard boundaries (float4 loads need K % 4 == 0)."""
    per = -(-n // t)
    per = -(-per // 4) * 4
    s = min(n, r * per)
    e = min(n, s + per)
    return s, e
