from .dataset import ArrayDataset, BatchedDataset, prepare_for_training, to_float_images
from .partition import client_train_val, contiguous_clients, shard_clients, train_test_clients
from .sources import (cifar10_dataset, idc_dataset, label_of, list_idc_files, load_files, split,
                      synthetic_dataset)

__all__ = ["ArrayDataset", "BatchedDataset", "prepare_for_training", "to_float_images",
           "client_train_val", "contiguous_clients", "shard_clients", "train_test_clients",
           "cifar10_dataset", "idc_dataset", "label_of", "list_idc_files", "load_files", "split",
           "synthetic_dataset"]
