from .partition import dirichlet_partition, class_counts
from .mnist import (synthetic_mnist, make_client_shards, write_shards, load_shard,
                    shard_paths, shards_exist)
from .device_dataset import DeviceShard
from .preprocess import (DeviceLoader, image_preprocess_dl, relational_table_preprocess_dl,
                         load_mnist_image, load_mnist_flat, non_iid_partition_with_dirichlet_distribution,
                         partition_class_samples_with_dirichlet_distribution, record_data_stats)

__all__ = ["dirichlet_partition", "class_counts", "synthetic_mnist", "make_client_shards",
           "write_shards", "load_shard", "shard_paths", "shards_exist", "DeviceShard",
           "DeviceLoader", "image_preprocess_dl", "relational_table_preprocess_dl", "load_mnist_image",
           "load_mnist_flat", "non_iid_partition_with_dirichlet_distribution",
           "partition_class_samples_with_dirichlet_distribution", "record_data_stats"]
