"""Client partitioners for federated simulation.

* ``contiguous_clients`` — ``fed_model.py:178-180``: client ``i`` = ``skip(i*CLIENT_SIZE)
  .take(CLIENT_SIZE)``.  Combined with the non-IID ordering of ``idc_dataset(iid=False)`` this
  reproduces the pathological label skew of quirk Q10.
* ``train_test_clients`` — ``fed_model.py:55-57,186-189``: clients 0..7 train, 8..9 test (the
  intended semantics of the effectively-ignored ``train_test_client_split``, quirk Q8).
* ``shard_clients`` — ``secure_fed_model.py:206-210``: client ``i`` = ``shard(K, i)``.
* ``client_train_val`` — per-client 80/20 split (``secure_fed_model.py:104-105``).
"""
from __future__ import annotations

from typing import List, Tuple

from .dataset import ArrayDataset


def contiguous_clients(ds: ArrayDataset, num_clients: int, client_size: int) -> List[ArrayDataset]:
    return [ds.skip(i * client_size).take(client_size) for i in range(num_clients)]


def train_test_clients(clients: List[ArrayDataset], num_test: int) -> Tuple[List[ArrayDataset], List[ArrayDataset]]:
    k = len(clients) - num_test
    return clients[:k], clients[k:]


def shard_clients(ds: ArrayDataset, num_clients: int) -> List[ArrayDataset]:
    return [ds.shard(num_clients, i) for i in range(num_clients)]


def client_train_val(ds: ArrayDataset, train_size: int, val_size: int):
    return ds.take(train_size), ds.skip(train_size).take(val_size)
