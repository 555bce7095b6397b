from .partition import dirichlet_partition, class_counts
from .mnist import (synthetic_mnist, make_client_shards, write_shards, load_shard,
                    shard_paths, shards_exist)
from .device_dataset import DeviceShard

__all__ = ["dirichlet_partition", "class_counts", "synthetic_mnist", "make_client_shards",
           "write_shards", "load_shard", "shard_paths", "shards_exist", "DeviceShard"]
