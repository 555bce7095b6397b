"""Client-front executor (Alice's conv stack) over the fused conv kernels.

Forward = one kernel (`conv_fwd`: gather uint8 rows by index, conv3x3, bias,
ReLU, maxpool, flatten); backward+step = two (`conv_bwd_step`: per-sample pool/ReLU
backward + dW/db partials, then one reduce + SGD-m / Adam update in place).  The SISA
client step is forward + 5408-way CE + partials in one kernel plus the reduce/update
(`conv_local_step`), and a whole local epoch is one host call (`local_epoch`).
Reference: models.py:16-30 (model1_sisa), data_entities_vanilla_sisa.py:55-70.  Parameters are the
`nn.Module`'s own tensors, so `state_dict()` keeps the reference key names
(`conv_layers.0.*` for model1_sisa, `conv1.*` for model1).
"""
from __future__ import annotations

import torch

from .. import ops
from ..data.device_dataset import DeviceShard
from ..models import ClientFront, ClientFrontSisa
from .slots import OptSlot


class FrontEngine:
    def __init__(self, module: ClientFront | ClientFrontSisa, device: torch.device):
        self.module = module.to(device)
        self.device = device
        self.ops = ops.impl(device)
        self.frozen = False
        # deferred optimizer step (split-mode epochs): (slab, B, cfg, st_w, st_b, t) of the last
        # backward, applied by the next forward in-kernel and stored by the next backward, so
        # a training batch is 2 client launches instead of 3; `flush` stores it
        self._pending = None
        self._slabs = None
        self._defer_i = 0

    def _raw_params(self):
        w, b = self.module.conv_params()
        return w.data, b.data

    @property
    def params(self):
        self.flush()
        return self._raw_params()

    def _slab_buf(self, B: int) -> torch.Tensor:
        """Ping-pong partial-slab buffers: a pending step's slabs stay intact while the next
        backward writes its own."""
        if self._slabs is None or self._slabs[0].numel() < B * 320:
            self.flush()                      # a pending step may point into the old buffers
            self._slabs = [torch.empty(max(B, 64) * 320, device=self.device) for _ in range(2)]
        buf = self._slabs[self._defer_i][:B * 320]
        self._defer_i ^= 1
        return buf

    def flush(self):
        """Store a deferred optimizer step (before anything else reads the weights)."""
        p, self._pending = self._pending, None
        if p is not None:
            w, b = self._raw_params()
            self.ops.conv_apply_(p, w, b)

    def forward(self, shard: DeviceShard, idx: torch.Tensor, with_labels: bool = False):
        """(activation, argmax); with_labels: (activation, argmax, shard.y[idx]) from one launch."""
        if self._pending is not None and with_labels:
            w, b = self._raw_params()
            return self.ops.conv_front_fwd_pending(shard.x, idx, w, b, shard.y, self._pending)
        w, b = self.params
        if with_labels:
            return self.ops.conv_front_fwd(shard.x, idx, w, b, labels=shard.y)
        return self.ops.conv_front_fwd(shard.x, idx, w, b)

    def forward_chunked(self, shard: DeviceShard, idx: torch.Tensor, chunk: int = 8192) -> torch.Tensor:
        """Activations for many samples (eval / SISA activation dump)."""
        outs = [self.forward(shard, idx[s:s + chunk])[0] for s in range(0, idx.numel(), chunk)]
        if not outs:
            return torch.empty(0, 5408, device=self.device)
        return outs[0] if len(outs) == 1 else torch.cat(outs, 0)

    @staticmethod
    def forward_multi(fronts: list, shards: list, orders: list, chunk: int = 8192) -> list:
        """`forward_chunked` of several co-located Alices at once (evaluation, SISA activation
        dumps): one launch per chunk of rows for all of them, bitwise each Alice's own
        forward.  `orders[i]` None: the shard's rows in order.  Falls back to one Alice after
        another on the torch backend or float shards."""
        ops_ = fronts[0].ops if fronts else None
        if not fronts or not hasattr(ops_, "conv_front_fwd_multi") or \
                any(sh.x.dtype != torch.uint8 for sh in shards):
            return [f.forward_chunked(sh, o if o is not None else sh.sequential_order(), chunk)
                    for f, sh, o in zip(fronts, shards, orders)]
        items = []
        for f, sh, o in zip(fronts, shards, orders):
            w, b = f.params
            items.append((sh.x, o, sh.n if o is None else int(o.numel()), w, b))
        return ops_.conv_front_fwd_multi(items, chunk)

    def backward_step(self, dy, y, am, shard: DeviceShard, idx, slot: OptSlot, t: int | None = None,
                      prefix: str = "", defer: bool = False):
        """Backward + optimizer step.  `defer` (split-mode epochs, HIP path): launch only the
        dW/db partials and leave the update pending for the next forward/backward (call
        `flush` when the run of steps ends); bitwise the same parameters."""
        if self.frozen:
            # reference: loss.backward() on frozen params raises (Q18)
            raise RuntimeError("element 0 of tensors does not require grad and does not have a grad_fn "
                               "(client front is frozen: call unfreeze_weights first)")
        if defer and hasattr(self.ops, "conv_front_bwd_defer_"):
            w, b = self._raw_params()
            t = slot.tick() if t is None else t
            st_w, st_b = slot.state(prefix + "conv.weight", w), slot.state(prefix + "conv.bias", b)
            slab = self._slab_buf(int(idx.numel()))
            self.ops.conv_front_bwd_defer_(dy, y, am, shard.x, idx, w, b, slab, self._pending, st_w, st_b)
            self._pending = (slab, int(idx.numel()), slot.cfg, st_w, st_b, t)
            return
        w, b = self.params
        t = slot.tick() if t is None else t
        self.ops.conv_front_bwd_step_(dy, y, am, shard.x, idx, w, b, slot.cfg,
                                      slot.state(prefix + "conv.weight", w),
                                      slot.state(prefix + "conv.bias", b), t)

    def local_step(self, shard: DeviceShard, idx, slot: OptSlot):
        """SISA client-only step: CE on the activation itself (Q5) + optimizer, fused."""
        if self.frozen:
            raise RuntimeError("element 0 of tensors does not require grad and does not have a grad_fn "
                               "(client front is frozen: call unfreeze_weights first)")
        w, b = self.params
        t = slot.tick()
        return self.ops.conv_local_step_(shard.x, shard.y, idx, w, b, slot.cfg,
                                         slot.state("conv.weight", w), slot.state("conv.bias", b), t)

    def local_epoch(self, shard: DeviceShard, order, B: int, slot: OptSlot):
        """ceil(len(order)/B) consecutive `local_step`s (last batch partial) in one host call."""
        if self.frozen:
            raise RuntimeError("element 0 of tensors does not require grad and does not have a grad_fn "
                               "(client front is frozen: call unfreeze_weights first)")
        w, b = self.params
        n = int(order.numel())
        nsteps = -(-n // B)
        if nsteps == 0:
            return None
        t0 = slot.t + 1
        st_w, st_b = slot.state("conv.weight", w), slot.state("conv.bias", b)
        loss = self.ops.conv_local_epoch_(shard.x, shard.y, order, B, w, b, slot.cfg, st_w, st_b, t0)
        slot.t += nsteps
        return loss

    @staticmethod
    def local_epoch_multi(fronts: list, shards: list, orders: list, B: int, slots: list):
        """`local_epoch` of several co-located Alices at once: every step of all of them is ONE
        launch (grid batch x Alices), bitwise the per-Alice epochs.  Falls back to one epoch
        after another where the fused multi-Alice kernel does not apply (torch backend)."""
        ops_ = fronts[0].ops
        if not hasattr(ops_, "conv_local_epoch_multi_") or any(f.frozen for f in fronts) or \
                any(sh.x.dtype != torch.uint8 for sh in shards) or len({s.cfg.kind for s in slots}) != 1:
            return [f.local_epoch(sh, o, B, sl) for f, sh, o, sl in zip(fronts, shards, orders, slots)]
        items = []
        for f, sh, o, sl in zip(fronts, shards, orders, slots):
            w, b = f.params
            items.append((sh.x, sh.y, o, w, b, sl.state("conv.weight", w), sl.state("conv.bias", b), sl.t + 1))
        losses = ops_.conv_local_epoch_multi_(items, B, slots[0].cfg)
        for sl, o in zip(slots, orders):
            sl.t += -(-int(o.numel()) // B)
        return losses

    def reset_parameters(self, true_reset: bool):
        """Reference `reset_model` (data_entities_vanilla.py:204-207): reset the direct
        children that have `reset_parameters`.  For model1_sisa that is nothing (Q4) unless
        `true_reset` asks for the evident intent."""
        self.flush()
        with torch.no_grad():
            if true_reset:
                for m in self.module.modules():
                    if hasattr(m, "reset_parameters") and m is not self.module:
                        m.reset_parameters()
            else:
                for m in self.module.children():
                    if hasattr(m, "reset_parameters"):
                        m.reset_parameters()

    # weight relay (the "Snapshot" hand-off between consecutive Alices)
    def flat_weights(self) -> torch.Tensor:
        w, b = self.params
        return torch.cat([w.reshape(-1), b.reshape(-1)])

    def load_flat_weights(self, flat: torch.Tensor):
        w, b = self.params
        w.copy_(flat[:w.numel()].view_as(w))
        b.copy_(flat[w.numel():w.numel() + b.numel()])

    @property
    def flat_numel(self) -> int:
        w, b = self.params
        return w.numel() + b.numel()
