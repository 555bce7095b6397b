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

    @property
    def params(self):
        w, b = self.module.conv_params()
        return w.data, b.data

    def forward(self, shard: DeviceShard, idx: torch.Tensor, with_labels: bool = False):
        """(activation, argmax); with_labels: (activation, argmax, shard.y[idx]) from one launch."""
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

    def backward_step(self, dy, y, am, shard: DeviceShard, idx, slot: OptSlot, t: int | None = None,
                      prefix: str = ""):
        if self.frozen:
            # reference: loss.backward() on frozen params raises (Q18)
            raise RuntimeError("element 0 of tensors does not require grad and does not have a grad_fn "
                               "(client front is frozen: call unfreeze_weights first)")
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

    def reset_parameters(self, true_reset: bool):
        """Reference `reset_model` (data_entities_vanilla.py:204-207): reset the direct
        children that have `reset_parameters`.  For model1_sisa that is nothing (Q4) unless
        `true_reset` asks for the evident intent."""
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
