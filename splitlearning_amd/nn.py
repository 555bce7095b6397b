"""Autograd-aware modules over the framework's kernels, for user-written models.

The engines (engine/) drive the reference architectures without autograd: they know
the whole step and fuse it. A user who builds a different split model out of ordinary
`nn.Module`s and trains it with `loss.backward()` and a `torch.optim` optimizer can use
these layers instead, and still gets the fused kernels on an MI355X:

* `FusedLinear`: Linear + optional ReLU + optional dropout in one forward kernel
  (the skinny split-K MFMA GEMM for batches <= 128, hipBLASLt + fused epilogue above).
  Backward is the dgrad kernel plus the wgrad kernel. Dropout masks come from a
  counter hash, so they are regenerated in backward instead of stored.
* `FusedConvFront`: `model1_sisa`'s Conv2d(1,32,3) + ReLU + MaxPool(2) + flatten, with
  the uint8 gather fused into the forward (models.py:16-30).
* `softmax_cross_entropy`: mean CrossEntropyLoss as one fused forward+backward kernel.

On CPU tensors the same layers run the eager torch implementations (ops/torch_ops.py),
so a model is written once. State-dict keys match `nn.Linear` / `model1_sisa`.
"""
from __future__ import annotations

import math

import torch
from torch import nn

from . import ops
from .ops.rng import step_seed


def _keep_scale(drop: float) -> float:
    return 1.0 / (1.0 - drop) if drop else 1.0


def _linear_impl(x):
    """The skinny kernels stream float4 rows: K % 4 == 0. Other widths use the eager path."""
    if x.shape[-1] % 4:
        return ops.torch_ops
    return ops.impl(x.device)


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, relu: bool, drop: float, seed: int):
        K = _linear_impl(x)
        x = x.contiguous()
        y = K.linear_fwd(x, weight.detach(), bias.detach() if bias is not None else None, relu, drop, seed, 0)
        ctx.save_for_backward(x, weight, y)
        ctx.relu, ctx.drop, ctx.has_bias = relu, drop, bias is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, y = ctx.saved_tensors
        K = _linear_impl(x)
        dz = dy.contiguous()
        if ctx.relu or ctx.drop:
            # y > 0 <=> (kept by dropout) and (ReLU active, when there is a ReLU)
            mask = (y > 0) if ctx.relu else (y != 0)
            dz = dz * mask * _keep_scale(ctx.drop)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = K.linear_dgrad(dz, weight.detach())
        if ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2]):
            dw, db = K.linear_wgrad(dz.contiguous(), x)
        return dx, dw, (db if ctx.has_bias else None), None, None, None


class FusedLinear(nn.Module):
    """`nn.Linear(in, out)` [+ ReLU] [+ Dropout(p)] as one kernel per pass."""

    def __init__(self, in_features: int, out_features: int, bias: bool = True, relu: bool = False,
                 dropout: float = 0.0, seed: int = 0):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.relu, self.dropout, self.seed = relu, float(dropout), seed
        self.weight = nn.Parameter(torch.empty(out_features, in_features))
        self.bias = nn.Parameter(torch.empty(out_features)) if bias else None
        self.calls = 0
        self.reset_parameters()

    def reset_parameters(self):
        # nn.Linear's default init (kaiming-uniform a=sqrt(5), uniform bias)
        nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            bound = 1.0 / math.sqrt(self.in_features) if self.in_features > 0 else 0.0
            nn.init.uniform_(self.bias, -bound, bound)

    def forward(self, x):
        drop = self.dropout if self.training else 0.0
        self.calls += 1
        seed = step_seed(self.seed, 0, self.calls) if drop else 0
        shape = x.shape
        y = _LinearFn.apply(x.reshape(-1, shape[-1]), self.weight, self.bias, self.relu, drop, seed)
        return y.reshape(*shape[:-1], self.out_features)

    def extra_repr(self):
        return (f"in_features={self.in_features}, out_features={self.out_features}, "
                f"relu={self.relu}, dropout={self.dropout}")


class _ConvFrontFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        K = ops.impl(x.device)
        B = x.shape[0]
        xf = x.reshape(B, 784).contiguous()
        idx = torch.arange(B, device=x.device)
        y, am = K.conv_front_fwd(xf, idx, weight.detach(), bias.detach())
        ctx.save_for_backward(xf, idx, weight, bias, y, am)
        return y

    @staticmethod
    def backward(ctx, dy):
        xf, idx, weight, bias, y, am = ctx.saved_tensors
        K = ops.impl(dy.device)
        dw, db = K.conv_front_bwd(dy.contiguous(), y, am, xf, idx, weight.detach(), bias.detach())
        return None, dw.view_as(weight), db.view_as(bias)


class FusedConvFront(nn.Module):
    """`model1_sisa` (Conv2d(1,32,3) -> ReLU -> MaxPool(2,2) -> Flatten) as one kernel.
    Input: [B,1,28,28] or [B,784], float32 or uint8 (raw 0-255 pixels, like the
    reference's unnormalised MNIST). Output: [B,5408]. The input gets no gradient."""

    def __init__(self):
        super().__init__()
        conv = nn.Conv2d(1, 32, 3)
        self.conv_layers = nn.Sequential(conv)      # state_dict: conv_layers.0.{weight,bias}

    def forward(self, x):
        c = self.conv_layers[0]
        return _ConvFrontFn.apply(x, c.weight, c.bias)


class _SoftmaxCEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, ignore_index: int):
        K = ops.impl(logits.device)
        n_valid = int((labels != ignore_index).sum().item())
        scale = 1.0 / max(n_valid, 1)
        loss_rows, d = K.softmax_ce(logits.contiguous(), labels.contiguous(), scale, ignore_index)
        ctx.save_for_backward(d)
        return loss_rows.sum() * scale

    @staticmethod
    def backward(ctx, g):
        (d,) = ctx.saved_tensors
        return d * g, None, None


def softmax_cross_entropy(logits, labels, ignore_index: int = -100):
    """`nn.CrossEntropyLoss()(logits, labels)` (mean over non-ignored rows)."""
    return _SoftmaxCEFn.apply(logits, labels, ignore_index)


__all__ = ["FusedLinear", "FusedConvFront", "softmax_cross_entropy"]
