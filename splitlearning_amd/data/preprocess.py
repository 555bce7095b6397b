"""Reference-named data API: partition helpers, client preprocessors and shard writers.

The reference's data layer (`/root/reference/data/`) is three modules of free
functions that user code calls directly:

* `non_iid_partition_with_dirichlet_distribution`, `partition_class_samples_with_dirichlet_distribution`,
  `record_data_stats` (`data/noniid_partition.py:6-103`);
* `image_preprocess_dl` / `relational_table_preprocess_dl` (`data/relational_table_preprocessor.py:8-104`),
  which return the FedML-style 8-element list
  `[train_num, test_num, train_global, test_global, train_local_num, train_local, test_local, class_num]`;
* `load_mnist_image` / `load_mnist_flat` (`data/mnist_flat/mnist_flat_generator.py:9-41`), which write
  one train and one test shard per client.

This module keeps those names, arguments and return shapes so scripts written against
the reference keep working, on top of the framework's pieces:

* the partition is `partition.dirichlet_partition` (explicit, seedable RNG);
* every "DataLoader" is a `DeviceLoader`: the client's whole shard sits in device memory,
  an epoch is an on-device permutation and a batch is an index gather — no per-sample
  `TensorDataset.__getitem__` + `default_collate`;
* shards are tensor-only dicts written by `mnist.write_shards` (Q10).  `load_mnist_flat`
  (broken in the reference: it calls an un-imported function, Q22) writes the same shards
  with flat `[n, 784]` rows; `DeviceShard` reads either layout.
"""
from __future__ import annotations

import math
from collections import Counter

import numpy as np
import torch

from ..config import MIN_SAMPLES_PER_CLIENT, NUM_CLASSES, TEST_PARTITION
from .partition import _split_one_class, class_counts, dirichlet_partition


# ---------------------------------------------------------------- partition (noniid_partition.py)
def non_iid_partition_with_dirichlet_distribution(label_list, client_num: int, classes: int, alpha: float,
                                                  task: str = "classification", rng=None,
                                                  min_size: int = MIN_SAMPLES_PER_CLIENT) -> dict[int, list[int]]:
    """{client (0-based): sample indices} — reference `noniid_partition.py:6-73`.

    `task='segmentation'` (multi-label rows) is not supported: the reference's only caller
    passes `task='task'`, which takes the classification branch."""
    if task == "segmentation":
        raise NotImplementedError("segmentation partitioning (multi-label rows) is not used by any mode")
    labels = np.asarray(label_list.cpu() if isinstance(label_list, torch.Tensor) else label_list)
    parts = dirichlet_partition(labels, client_num, classes, alpha, rng=rng, min_size=min_size)
    return {c: idx.tolist() for c, idx in parts.items()}


def partition_class_samples_with_dirichlet_distribution(N: int, alpha: float, client_num: int, idx_batch,
                                                        idx_k, rng=None):
    """Split one class's indices `idx_k` over the clients' lists `idx_batch` in place and
    return `(idx_batch, min_size)` — reference `noniid_partition.py:76-91`."""
    rng = rng if rng is not None else np.random.default_rng()
    _split_one_class(rng, N, alpha, client_num, idx_batch, np.asarray(idx_k))
    return idx_batch, min(len(b) for b in idx_batch)


def record_data_stats(y_train, net_dataidx_map: dict, task: str = "classification") -> dict:
    """{client: {class: count}} — reference `noniid_partition.py:94-103`."""
    labels = np.asarray(y_train.cpu() if isinstance(y_train, torch.Tensor) else y_train)
    return class_counts(labels, {c: np.asarray(idx, dtype=np.int64) for c, idx in net_dataidx_map.items()})


# ---------------------------------------------------------------- device loaders
class DeviceLoader:
    """`DataLoader(TensorDataset(x, y), batch_size, shuffle)` with both tensors resident on
    `device`.  Iterating yields `(x[idx], y[idx])` batches; with `shuffle` each epoch draws a
    fresh permutation from `generator` (the reference reshuffles every epoch)."""

    def __init__(self, x: torch.Tensor, y: torch.Tensor, batch_size: int, shuffle: bool = False,
                 device: torch.device | str | None = None, generator: torch.Generator | None = None):
        if x.shape[0] != y.shape[0]:
            raise ValueError(f"x has {x.shape[0]} rows but y has {y.shape[0]}")
        if batch_size < 1:
            raise ValueError("batch_size must be >= 1")
        device = torch.device(device) if device is not None else x.device
        self.x = x.to(device).contiguous()
        self.y = y.to(device=device, dtype=torch.int64).contiguous()
        self.batch_size = int(batch_size)
        self.shuffle = shuffle
        self.generator = generator
        self.device = device

    @property
    def dataset(self) -> tuple[torch.Tensor, torch.Tensor]:
        """(x, y); `loader.dataset[1]` is the label tensor, like `TensorDataset[:][1]`."""
        return self.x, self.y

    def __len__(self) -> int:
        return math.ceil(self.y.shape[0] / self.batch_size)

    def order(self) -> torch.Tensor:
        n = self.y.shape[0]
        if not self.shuffle:
            return torch.arange(n, device=self.device)
        return torch.randperm(n, generator=self.generator).to(self.device)

    def __iter__(self):
        order = self.order()
        for s in range(0, order.numel(), self.batch_size):
            idx = order[s:s + self.batch_size]
            yield self.x.index_select(0, idx), self.y.index_select(0, idx)

    def label_counter(self) -> dict:
        return dict(Counter(self.y.cpu().tolist()))


def _preprocess_dl(args, data, label_list, test_partition: float, rng, device, generator):
    labels = torch.as_tensor(np.asarray(label_list), dtype=torch.int64)
    x = data if isinstance(data, torch.Tensor) else torch.as_tensor(np.asarray(data))
    if not x.is_floating_point() and x.dtype != torch.uint8:
        x = x.to(torch.float32)
    rng = rng if rng is not None else np.random.default_rng(getattr(args, "seed", None))
    classes = int(getattr(args, "class_num", 0) or NUM_CLASSES)
    # the same partition + split as the CLI's shard writer (mnist.partition_and_split)
    from .mnist import partition_and_split
    splits = partition_and_split(labels.numpy(), args.client_num_in_total, args.partition_alpha, rng,
                                 test_partition, classes)
    train_num, test_num = 0, 0
    train_local_num, train_local, test_local = {}, {}, {}
    tr_x, tr_y, te_x, te_y = [], [], [], []
    for key, (tr_i, te_i) in splits.items():
        n_train = len(tr_i)
        idx = np.concatenate([tr_i, te_i])
        tr, te = torch.from_numpy(tr_i), torch.from_numpy(te_i)
        train_local_num[key] = n_train
        train_local[key] = DeviceLoader(x[tr], labels[tr], args.batch_size, shuffle=True, device=device,
                                        generator=generator)
        test_local[key] = DeviceLoader(x[te], labels[te], args.batch_size, shuffle=False, device=device)
        tr_x.append(x[tr]); tr_y.append(labels[tr]); te_x.append(x[te]); te_y.append(labels[te])
        train_num += n_train
        test_num += len(idx) - n_train
    train_global = DeviceLoader(torch.cat(tr_x), torch.cat(tr_y), args.batch_size, device=device)
    test_global = DeviceLoader(torch.cat(te_x), torch.cat(te_y), args.batch_size, device=device)
    return [train_num, test_num, train_global, test_global, train_local_num, train_local, test_local, classes]


def image_preprocess_dl(args, data, label_list, test_partition: float = TEST_PARTITION, rng=None,
                        device=None, generator=None):
    """Images `[N, 1, 28, 28]` -> per-client loaders (`relational_table_preprocessor.py:57-104`)."""
    return _preprocess_dl(args, data, label_list, test_partition, rng, device, generator)


def relational_table_preprocess_dl(args, data, label_list, test_partition: float = TEST_PARTITION, rng=None,
                                   device=None, generator=None):
    """Tabular rows `[N, F]` -> per-client loaders (`relational_table_preprocessor.py:8-55`)."""
    x = torch.as_tensor(np.asarray(data)) if not isinstance(data, torch.Tensor) else data
    if x.dim() != 2:
        raise ValueError(f"relational tables are [N, F]; got shape {tuple(x.shape)}")
    return _preprocess_dl(args, x, label_list, test_partition, rng, device, generator)


# ---------------------------------------------------------------- shard writers (mnist_flat_generator.py)
def load_mnist_image(args, verbose: bool = True) -> dict[int, tuple[int, int]]:
    """Write every client's `{x: uint8[n,1,28,28], y}` train/test shard (`mnist_flat_generator.py:26-41`)."""
    from .mnist import write_shards
    args.class_num = NUM_CLASSES
    return write_shards(args, verbose=verbose, layout="image")


def load_mnist_flat(args, verbose: bool = True) -> dict[int, tuple[int, int]]:
    """The flat variant (`mnist_flat_generator.py:9-24`): shards hold `[n, 784]` rows."""
    from .mnist import write_shards
    args.class_num = NUM_CLASSES
    return write_shards(args, verbose=verbose, layout="flat")
