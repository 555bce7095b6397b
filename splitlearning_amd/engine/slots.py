"""Optimizer-state slots.

The reference builds one `DistributedOptimizer` per Alice over Bob's *and* her
own parameters (`data_entities_vanilla.py:37-42`, `data_entities.py:43-47`), so
Bob holds an independent SGD-momentum / Adam state per Alice, and `unlearn`
builds a brand-new one (`data_entities_vanilla.py:132-137`) — SURVEY Q8.  A
`OptSlot` is exactly one such optimizer instance restricted to one worker's
parameters: hyper-parameters, a step counter and lazily created state tensors
(`buf` for SGD, `m`/`v` for Adam) keyed by parameter name.  Bob keeps a dict of
slots keyed by Alice id; the fused kernels read/write the slot's tensors in place.
"""
from __future__ import annotations

import torch

from ..config import OptimCfg


class OptSlot:
    def __init__(self, cfg: OptimCfg):
        self.cfg = cfg
        self.t = 0
        self.states: dict[str, dict[str, torch.Tensor]] = {}

    def state(self, name: str, p: torch.Tensor) -> dict:
        st = self.states.get(name)
        if st is None:
            if self.cfg.kind == "adam":
                st = {"m": torch.zeros_like(p, memory_format=torch.contiguous_format),
                      "v": torch.zeros_like(p, memory_format=torch.contiguous_format)}
            else:
                st = {"buf": torch.zeros_like(p, memory_format=torch.contiguous_format)}
            self.states[name] = st
        return st

    def tick(self) -> int:
        """Advance the step counter (one `optimizer.step()`); returns the new t."""
        self.t += 1
        return self.t

    def nbytes(self) -> int:
        return sum(t.numel() * t.element_size() for st in self.states.values() for t in st.values())


def sgd_momentum(lr: float) -> OptimCfg:
    """torch.optim.SGD(lr, momentum=0.9) (data_entities_vanilla.py:37-42)."""
    from ..config import SGD_MOMENTUM
    return OptimCfg("sgd", lr, momentum=SGD_MOMENTUM)


def adam(lr: float, weight_decay: float = 0.0) -> OptimCfg:
    """torch.optim.Adam(lr[, weight_decay]) (data_entities.py:43-47; data_entities_vanilla_sisa.py:48,266)."""
    return OptimCfg("adam", lr, weight_decay=weight_decay)
