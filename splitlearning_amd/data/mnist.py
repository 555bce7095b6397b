"""MNIST-shaped data generation and tensor-only client shards.

Reference behaviour (`/root/reference/data/mnist_flat/mnist_flat_generator.py:26-41`,
`data/relational_table_preprocessor.py:57-104`): fetch MNIST, keep raw 0-255
pixels (no normalisation, Q13), Dirichlet-partition over the clients, shuffle
each client's indices, split 80/20 train/test and `torch.save` one train and one
test shard per client as `<datapath>/data_worker{k}_{train,test}.pt`, printing
each client's sorted train-label histogram.

Differences (documented in docs/DEVIATIONS.md):
* there is no network, so the default source is a synthetic, *learnable*
  MNIST-shaped set (class prototypes + per-sample jitter/noise, uint8 pixels);
  a local `.npz` with real MNIST can be supplied with `--mnist_npz`;
* shards are tensor-only dicts `{"x": uint8[n,1,28,28], "y": int64[n]}` that
  load with `torch.load(weights_only=True)` instead of pickled DataLoaders (Q10);
* generation can be seeded.
"""
from __future__ import annotations

import os
from collections import Counter

import numpy as np
import torch

from ..config import MIN_SAMPLES_PER_CLIENT, NUM_CLASSES, TEST_PARTITION
from .partition import dirichlet_partition


def _prototypes(rng: np.random.Generator) -> np.ndarray:
    """10 smooth 28x28 stroke-like templates in [0,1]."""
    yy, xx = np.mgrid[0:28, 0:28].astype(np.float32)
    protos = np.zeros((NUM_CLASSES, 28, 28), np.float32)
    for c in range(NUM_CLASSES):
        img = np.zeros((28, 28), np.float32)
        for _ in range(3 + c % 3):       # a few gaussian strokes per class
            cy, cx = rng.uniform(6, 22, size=2)
            sy, sx = rng.uniform(1.2, 4.5, size=2)
            img += np.exp(-(((yy - cy) / sy) ** 2 + ((xx - cx) / sx) ** 2))
        protos[c] = img / img.max()
    return protos


def synthetic_mnist(n: int, seed: int | None = None) -> tuple[np.ndarray, np.ndarray]:
    """Synthetic MNIST-shaped data: x uint8 [n,1,28,28] (0..255), y int64 [n]."""
    rng = np.random.default_rng(seed)
    protos = _prototypes(np.random.default_rng(1234 if seed is None else seed + 1))
    y = rng.integers(0, NUM_CLASSES, size=n).astype(np.int64)
    x = np.empty((n, 1, 28, 28), np.uint8)
    chunk = 8192
    for s in range(0, n, chunk):
        yc = y[s:s + chunk]
        m = yc.shape[0]
        base = protos[yc]
        # random sub-pixel-ish shift and intensity + additive noise
        shift = rng.integers(-2, 3, size=(m, 2))
        for j in range(m):
            base[j] = np.roll(base[j], tuple(shift[j]), axis=(0, 1))
        inten = rng.uniform(180, 255, size=(m, 1, 1)).astype(np.float32)
        noise = rng.normal(0, 25, size=(m, 28, 28)).astype(np.float32)
        img = np.clip(base * inten + noise, 0, 255)
        x[s:s + m, 0] = img.astype(np.uint8)
    return x, y


def load_source(args) -> tuple[np.ndarray, np.ndarray]:
    path = getattr(args, "mnist_npz", "")
    if path:
        with np.load(path, allow_pickle=False) as z:
            x = np.asarray(z["x"], dtype=np.uint8).reshape(-1, 1, 28, 28)
            y = np.asarray(z["y"]).astype(np.int64)
        return x, y
    return synthetic_mnist(int(getattr(args, "num_samples", 70000)), getattr(args, "seed", None))


def shard_paths(datapath: str, client_id: int) -> tuple[str, str]:
    return (os.path.join(datapath, f"data_worker{client_id}_train.pt"),
            os.path.join(datapath, f"data_worker{client_id}_test.pt"))


def partition_and_split(y: np.ndarray, client_num: int, alpha: float, rng: np.random.Generator,
                        test_partition: float = TEST_PARTITION, classes: int = NUM_CLASSES):
    """The one partition + split used everywhere (CLI shards, the reference-named
    `image_preprocess_dl` API, the benchmark): Dirichlet partition over the clients, then
    per client a shuffle and the 80/20 train/test split
    (`relational_table_preprocessor.py:62-92`).  Returns {client (0-based): (train_idx, test_idx)}."""
    parts = dirichlet_partition(y, client_num, classes, alpha, rng=rng, min_size=MIN_SAMPLES_PER_CLIENT)
    out = {}
    for key, idx in parts.items():
        idx = np.asarray(idx, dtype=np.int64).copy()
        rng.shuffle(idx)                      # relational_table_preprocessor.py:83
        n_train = int(len(idx) * (1 - test_partition))
        out[key] = (idx[:n_train], idx[n_train:])
    return out


def make_client_shards(x: np.ndarray, y: np.ndarray, client_num: int, alpha: float,
                       seed: int | None = None, test_partition: float = TEST_PARTITION):
    """Partition + per-client 80/20 split.  Returns {client_id (1-based): (xtr, ytr, xte, yte)}."""
    rng = np.random.default_rng(seed)
    out = {}
    for key, (tr, te) in partition_and_split(y, client_num, alpha, rng, test_partition).items():
        out[key + 1] = (x[tr], y[tr], x[te], y[te])
    return out


def write_shards(args, verbose: bool = True, layout: str = "image") -> dict[int, tuple[int, int]]:
    """Generate and save every client shard (reference `load_mnist_image`; `layout="flat"`
    = `load_mnist_flat`, rows of 784 pixels)."""
    if layout not in ("image", "flat"):
        raise ValueError(f"unknown shard layout {layout!r}")
    os.makedirs(args.datapath, exist_ok=True)
    x, y = load_source(args)
    shards = make_client_shards(x, y, args.client_num_in_total, args.partition_alpha,
                                seed=getattr(args, "seed", None))
    sizes = {}
    for cid, (xtr, ytr, xte, yte) in shards.items():
        if layout == "flat":
            xtr, xte = xtr.reshape(len(xtr), 784), xte.reshape(len(xte), 784)
        ptr, pte = shard_paths(args.datapath, cid)
        torch.save({"x": torch.from_numpy(np.ascontiguousarray(xtr)),
                    "y": torch.from_numpy(np.ascontiguousarray(ytr))}, ptr)
        torch.save({"x": torch.from_numpy(np.ascontiguousarray(xte)),
                    "y": torch.from_numpy(np.ascontiguousarray(yte))}, pte)
        if verbose:
            print(dict(sorted(Counter(ytr.tolist()).items())))
        sizes[cid] = (len(ytr), len(yte))
    return sizes


def shards_exist(datapath: str, client_num: int) -> bool:
    return all(os.path.exists(p) for c in range(1, client_num + 1) for p in shard_paths(datapath, c))


def load_shard(datapath: str, client_id: int) -> tuple[dict, dict]:
    """Load one client's train/test shard with the code-free loader."""
    ptr, pte = shard_paths(datapath, client_id)
    tr = torch.load(ptr, weights_only=True)
    te = torch.load(pte, weights_only=True)
    for d in (tr, te):
        if set(d) != {"x", "y"}:
            raise ValueError(f"unexpected shard layout: keys {sorted(d)}")
    return tr, te
