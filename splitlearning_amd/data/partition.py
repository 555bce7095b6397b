"""Dirichlet (LDA) non-IID label partitioner.

Behavioural parity with `/root/reference/data/noniid_partition.py:6-91`
(Hsu et al. 2019): for every class the class's shuffled sample indices are
split over the clients by a Dirichlet(alpha) draw; clients that already hold
>= N/client_num samples get a zero share; the whole draw is repeated until
every client owns at least `min_size` samples; each client's index list is
finally shuffled.  Unlike the reference the RNG is an explicit
`numpy.random.Generator`, so a run can be seeded (Q11).
"""
from __future__ import annotations

from collections import Counter

import numpy as np


def _split_one_class(rng, n_total, alpha, client_num, buckets, idx_k):
    idx_k = idx_k.copy()
    rng.shuffle(idx_k)
    share = rng.dirichlet(np.full(client_num, alpha))
    cap = n_total / client_num
    share = share * np.array([len(b) < cap for b in buckets], dtype=np.float64)
    share = share / share.sum()
    cuts = (np.cumsum(share) * len(idx_k)).astype(int)[:-1]
    for b, part in zip(buckets, np.split(idx_k, cuts)):
        b.extend(part.tolist())


def dirichlet_partition(labels, client_num: int, num_classes: int, alpha: float,
                        rng: np.random.Generator | None = None,
                        min_size: int = 10, max_tries: int = 10000) -> dict[int, np.ndarray]:
    """Return {client_index (0-based): int64 index array}.

    The union of the arrays is a disjoint cover of range(len(labels)).
    """
    labels = np.asarray(labels)
    rng = rng if rng is not None else np.random.default_rng()
    n = labels.shape[0]
    if client_num < 1:
        raise ValueError("client_num must be >= 1")
    if n < client_num * min_size:
        raise ValueError(f"{n} samples cannot give {client_num} clients >= {min_size} each")
    by_class = [np.flatnonzero(labels == k) for k in range(num_classes)]
    for _ in range(max_tries):
        buckets: list[list[int]] = [[] for _ in range(client_num)]
        for idx_k in by_class:
            _split_one_class(rng, n, alpha, client_num, buckets, idx_k)
        if min(len(b) for b in buckets) >= min_size:
            break
    else:  # pragma: no cover - astronomically unlikely with sane inputs
        raise RuntimeError("Dirichlet partition did not reach min_size")
    out = {}
    for i, b in enumerate(buckets):
        arr = np.asarray(b, dtype=np.int64)
        rng.shuffle(arr)
        out[i] = arr
    return out


def class_counts(labels, parts: dict[int, np.ndarray]) -> dict[int, dict[int, int]]:
    """Per-client label histograms (reference `record_data_stats`, noniid_partition.py:94-103)."""
    labels = np.asarray(labels)
    return {c: dict(sorted(Counter(labels[idx].tolist()).items())) for c, idx in parts.items()}
