"""Model zoo: client fronts, server tails and the U-shape head.

Architectures, parameter shapes and **state_dict key names** match the
reference (`/root/reference/models.py:5-94`) so checkpoints are
interchangeable.  The classes are ordinary `nn.Module`s; they own the
parameters.  The hot path does not call their `forward` on GPU: the engine
(`splitlearning_amd.engine`) runs fused HIP kernels over the same parameter
tensors.  `forward` here is the eager PyTorch definition that the numerics
tests use as ground truth.

Layer descriptions are exported as `TailSpec` so the engine and the
tensor-parallel sharder know each Linear's role.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..config import CUT_FEATURES, DROPOUT_P


class ClientFront(nn.Module):
    """Conv2d(1,32,3) -> ReLU -> MaxPool(2,2), output [B,32,13,13].  Reference `model1`
    (models.py:5-14); keys `conv1.weight`, `conv1.bias`."""

    flat_output = False

    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 32, 3)
        self.pool = nn.MaxPool2d(2, 2)

    def conv_params(self):
        return self.conv1.weight, self.conv1.bias

    def forward(self, x):
        return self.pool(F.relu(self.conv1(x)))


class ClientFrontSisa(nn.Module):
    """Sequential(Conv2d, ReLU, MaxPool) -> Flatten, output [B,5408].  Reference
    `model1_sisa` (models.py:16-30); keys `conv_layers.0.weight`, `conv_layers.0.bias`.
    Its direct children (`Sequential`, `Flatten`) have no `reset_parameters`, which
    is why the reference's unlearn reset is a no-op (Q4)."""

    flat_output = True

    def __init__(self):
        super().__init__()
        self.conv_layers = nn.Sequential(nn.Conv2d(1, 32, 3), nn.ReLU(), nn.MaxPool2d(2, 2))
        self.flatten = nn.Flatten()

    def conv_params(self):
        c = self.conv_layers[0]
        return c.weight, c.bias

    def forward(self, x):
        return self.flatten(self.conv_layers(x))


@dataclass
class LinearSpec:
    name: str
    in_features: int
    out_features: int
    relu: bool
    dropout: float        # 0.0 = none


@dataclass
class TailSpec:
    layers: list = field(default_factory=list)

    @property
    def in_features(self):
        return self.layers[0].in_features

    @property
    def out_features(self):
        return self.layers[-1].out_features


class _MLP(nn.Module):
    """Flatten -> [Linear (-> ReLU) (-> Dropout)]*.  Subclasses set `spec`."""

    spec: TailSpec

    def __init__(self, spec: TailSpec):
        super().__init__()
        self.spec = spec
        for ls in spec.layers:
            setattr(self, ls.name, nn.Linear(ls.in_features, ls.out_features))
            if ls.dropout > 0:
                setattr(self, "dropout" + ls.name[-1], nn.Dropout(ls.dropout))

    def linears(self):
        return [getattr(self, ls.name) for ls in self.spec.layers]

    def forward(self, x):
        x = torch.flatten(x, 1)
        for ls in self.spec.layers:
            x = getattr(self, ls.name)(x)
            if ls.relu:
                x = F.relu(x)
            if ls.dropout > 0:
                x = getattr(self, "dropout" + ls.name[-1])(x)
        return x


def ushape_server_spec() -> TailSpec:
    """Reference `model2` (models.py:33-44): fc1 5408->1000 ReLU, fc2 1000->100 ReLU."""
    return TailSpec([LinearSpec("fc1", CUT_FEATURES, 1000, True, 0.0),
                     LinearSpec("fc2", 1000, 100, True, 0.0)])


def sisa_server_spec(num_clients: int = 1, concat: bool = False) -> TailSpec:
    """Reference `model2_sisa` (models.py:46-63) or `model2_sisa_concat(k)` (models.py:66-82)."""
    k = num_clients if concat else 1
    return TailSpec([LinearSpec("fc1", CUT_FEATURES * k, 5000, True, DROPOUT_P),
                     LinearSpec("fc2", 5000, 1000, True, DROPOUT_P),
                     LinearSpec("fc3", 1000, 100 * k, False, 0.0)])


def head_spec() -> TailSpec:
    """Reference `model3` (models.py:87-94): fc3 100->10 (U-shape head, on Alice)."""
    return TailSpec([LinearSpec("fc3", 100, 10, False, 0.0)])


class ServerTailUShape(_MLP):
    def __init__(self):
        super().__init__(ushape_server_spec())


class ServerTailSisa(_MLP):
    def __init__(self):
        super().__init__(sisa_server_spec())


class ServerTailSisaConcat(_MLP):
    def __init__(self, num_clients: int):
        super().__init__(sisa_server_spec(num_clients, concat=True))
        self.num_clients = num_clients


class Head(_MLP):
    def __init__(self):
        super().__init__(head_spec())


# Reference class names (models.py) — same constructors, same state_dict keys.
model1 = ClientFront
model1_sisa = ClientFrontSisa
model2 = ServerTailUShape
model2_sisa = ServerTailSisa
model2_sisa_concat = ServerTailSisaConcat
model3 = Head
