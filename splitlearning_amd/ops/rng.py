"""Counter-based dropout RNG shared bit-for-bit by the HIP kernels and the torch path.

The reference uses `nn.Dropout(0.5)` (models.py:50,52), i.e. a stateful
Bernoulli stream; its masks cannot be reproduced anyway, so the framework uses
a stateless hash of (seed, batch row, *global* feature column).  Hashing the
global column makes the mask independent of how Bob's tail is sharded across
tensor-parallel ranks, and lets the backward pass regenerate nothing: the
ReLU+dropout backward only needs the stored post-dropout activation
(`dz = dh * scale * [h > 0]`).  The HIP twin is `sl_hash_keep` in
`csrc/common.h`; `tests/test_ops_cpu.py` pins the two together.
"""
from __future__ import annotations

import torch

M32 = 0xFFFFFFFF
C_ROW = 0x9E3779B1
C_COL = 0x85EBCA77


def _fmix32(x: torch.Tensor) -> torch.Tensor:
    x = x ^ (x >> 16)
    x = (x * 0x85EBCA6B) & M32
    x = x ^ (x >> 13)
    x = (x * 0xC2B2AE35) & M32
    x = x ^ (x >> 16)
    return x


def split_seed(seed: int) -> tuple[int, int]:
    seed &= (1 << 64) - 1
    return seed & M32, (seed >> 32) & M32


def keep_mask(seed: int, rows: int, cols: int, p: float, col_offset: int = 0,
              device=None) -> torch.Tensor:
    """Boolean keep-mask [rows, cols] for dropout probability p."""
    lo, hi = split_seed(seed)
    r = torch.arange(rows, dtype=torch.int64, device=device).view(-1, 1)
    c = torch.arange(col_offset, col_offset + cols, dtype=torch.int64, device=device).view(1, -1)
    a = _fmix32(((r * C_ROW) & M32) ^ lo)
    h = _fmix32(a ^ (((c * C_COL) & M32) ^ hi))
    thresh = int(p * 4294967296.0)
    return h >= thresh


def step_seed(base: int, layer: int, step: int) -> int:
    """Derive the per-(layer, step) 64-bit seed on the host (no device state)."""
    x = (base * 0x9E3779B97F4A7C15 + layer * 0xBF58476D1CE4E5B9 + step * 0x94D049BB133111EB)
    x &= (1 << 64) - 1
    x ^= x >> 31
    x = (x * 0xD6E8FEB86659FD93) & ((1 << 64) - 1)
    x ^= x >> 32
    return x
