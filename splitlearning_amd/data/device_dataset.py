"""Device-resident client shard with on-device shuffling and batch slicing.

Replaces the reference's per-sample `TensorDataset` + `DataLoader` +
`default_collate` path (`data/relational_table_preprocessor.py:86-92`,
consumed at e.g. `data_entities_vanilla_sisa.py:59`), which SURVEY §6 shows
is the reference's real CPU bottleneck.  The whole shard lives in device
memory as uint8 pixels (784 B/sample: all of MNIST is 55 MB of the 288 GB
HBM); an epoch is a permutation tensor, a batch is a view of 16 indices, and
the conv kernel gathers + converts the rows itself (no collate, no copy).
"""
from __future__ import annotations

from collections import Counter

import torch


class DeviceShard:
    def __init__(self, x_u8: torch.Tensor, y: torch.Tensor, device: torch.device):
        if x_u8.dtype != torch.uint8:
            raise TypeError("shard pixels must be uint8 0..255")
        self.n = int(y.shape[0])
        self.x = x_u8.reshape(self.n, 784).contiguous().to(device, non_blocking=False)
        self.y = y.to(torch.int64).contiguous().to(device)
        self.y_cpu = y.to(torch.int64).cpu()
        self.device = device

    def __len__(self):
        return self.n

    def label_counter(self, order: torch.Tensor | None = None) -> dict:
        ys = self.y_cpu if order is None else self.y_cpu[order.cpu()]
        return dict(Counter(ys.tolist()))

    def shuffled_order(self, gen: torch.Generator) -> torch.Tensor:
        """One epoch's sample order (DataLoader(shuffle=True) semantics).  Drawn from the
        Alice's host generator, so a seeded run gives the same orders on every backend and
        the order is part of the generator state a snapshot saves; on a GPU it is copied from
        pinned memory without blocking the host (a pageable copy would wait for the stream
        to drain before the epoch's launches could be queued)."""
        perm = torch.randperm(self.n, generator=gen)
        if self.device.type != "cuda":
            return perm
        return perm.pin_memory().to(self.device, non_blocking=True)

    def sequential_order(self) -> torch.Tensor:
        return torch.arange(self.n, device=self.device)

    def filtered_order(self, order: torch.Tensor, omit_label: int) -> torch.Tensor:
        """Keep `order`'s relative order, drop samples whose label == omit_label
        (the reference builds its unlearn list exactly this way while iterating
        the shuffled train loader: `data_entities_vanilla_sisa.py:150`)."""
        keep = self.y_cpu[order.cpu()] != omit_label
        return order[keep.to(order.device)]

    @staticmethod
    def batch_slices(n: int, batch_size: int):
        for s in range(0, n, batch_size):
            yield s, min(s + batch_size, n)

    def x_float(self, idx: torch.Tensor) -> torch.Tensor:
        """Gathered float32 NCHW batch (torch path / reference checks only)."""
        return self.x.index_select(0, idx).to(torch.float32).reshape(-1, 1, 28, 28)
