"""Data layer: tf.data-like ops, IDC PNG directory loader, CIFAR binaries, partitioners (T7)."""
import os

import numpy as np
import pytest
import torch

from idc_models_amd.data import (ArrayDataset, cifar10_dataset, client_train_val, contiguous_clients,
                                 idc_dataset, label_of, list_idc_files, prepare_for_training,
                                 shard_clients, split, synthetic_dataset, train_test_clients)
from idc_models_amd.data.dataset import _buffer_shuffle


def _png_tree(root, layout="balanced", n_per=6, size=50):
    from PIL import Image
    rng = np.random.default_rng(0)
    files = []
    for lab in ("0", "1"):
        for i in range(n_per):
            if layout == "balanced":
                d = os.path.join(root, "data", "balanced_IDC_30k", lab)
            else:
                d = os.path.join(root, "data", "IDC_regular_ps50_idx5", f"{1000 + i % 3}", lab)
            os.makedirs(d, exist_ok=True)
            arr = rng.integers(0, 255, (size + (i % 2) * 3, size, 3), dtype=np.uint8)
            p = os.path.join(d, f"img_{lab}_{i}.png")
            Image.fromarray(arr).save(p)
            files.append(p)
    return files


def test_take_skip_shard_are_disjoint_views():
    ds = ArrayDataset(np.zeros((10, 2, 2, 3), np.uint8), np.arange(10))
    assert list(ds.take(3).labels()) == [0, 1, 2]
    assert list(ds.skip(8).labels()) == [8, 9]
    assert list(ds.shard(3, 1).labels()) == [1, 4, 7]
    tr, va, te = split(ds, (0.8, 0.1, 0.1))
    assert len(tr) + len(va) + len(te) == 10
    assert set(tr.labels()).isdisjoint(set(te.labels()))


def test_shuffle_buffer_is_a_permutation_and_reshuffles_each_epoch():
    idx = np.arange(100)
    rng = np.random.default_rng(0)
    out = _buffer_shuffle(idx, 10, rng)
    assert sorted(out) == list(range(100)) and not np.array_equal(out, idx)
    ds = synthetic_dataset(50, (4, 4, 3), seed=0)
    b = prepare_for_training(ds, 10)
    e1 = np.concatenate([y.numpy() for _, y in b])
    e2 = np.concatenate([y.numpy() for _, y in b])
    assert len(b) == 5 and len(e1) == 50
    assert sorted(e1) == sorted(e2)


def test_batches_drop_remainder_and_repeat():
    ds = synthetic_dataset(25, (4, 4, 3), seed=0)
    assert len(ds.batch(10, drop_remainder=True)) == 2
    assert len(ds.batch(10, repeat=2)) == 5
    xs = [x for x, _ in ds.batch(10, drop_remainder=True)]
    assert all(x.shape == (10, 4, 4, 3) and x.dtype == torch.uint8 for x in xs)


def test_idc_balanced_loader(tmp_path):
    _png_tree(str(tmp_path), "balanced")
    files = list_idc_files(str(tmp_path), "balanced")
    assert len(files) == 12 and {label_of(f) for f in files} == {0, 1}
    ds = idc_dataset(str(tmp_path), "balanced", 50, seed=1)
    assert ds.x.shape == (12, 50, 50, 3) and ds.x.dtype == np.uint8
    assert sorted(ds.labels().tolist()) == [0] * 6 + [1] * 6
    small = idc_dataset(str(tmp_path), "balanced", 10, seed=1)  # secure_fed_model 10x10
    assert small.x.shape == (12, 10, 10, 3)


def test_idc_patient_layout_and_noniid_order(tmp_path):
    _png_tree(str(tmp_path), "patient")
    ds = idc_dataset(str(tmp_path), "patient", 50)
    assert len(ds) == 12
    _png_tree(str(tmp_path / "b"), "balanced")
    nonid = idc_dataset(str(tmp_path / "b"), "balanced", 50, iid=False)
    # get_data(non-iid): all class-1 files first, then class-0 (fed_model.py:161-164)
    assert nonid.labels().tolist() == [1] * 6 + [0] * 6


def test_cifar_binary_loader(tmp_path):
    rng = np.random.default_rng(0)
    for name, n in [("data_batch_%d.bin" % i, 4) for i in range(1, 6)] + [("test_batch.bin", 3)]:
        rec = np.zeros((n, 3073), np.uint8)
        rec[:, 0] = rng.integers(0, 10, n)
        rec[:, 1:] = rng.integers(0, 255, (n, 3072))
        rec.tofile(str(tmp_path / name))
    tr = cifar10_dataset(str(tmp_path), True)
    te = cifar10_dataset(str(tmp_path), False)
    assert tr.x.shape == (20, 32, 32, 3) and te.x.shape == (3, 32, 32, 3)


def test_partitions():
    ds = synthetic_dataset(100, (4, 4, 3), seed=0)
    clients = contiguous_clients(ds, 10, 10)
    assert [len(c) for c in clients] == [10] * 10
    trc, tec = train_test_clients(clients, 2)
    assert len(trc) == 8 and len(tec) == 2
    shards = shard_clients(ds, 3)
    assert sum(len(s) for s in shards) == 100
    a, b = client_train_val(shards[0], 20, 5)
    assert len(a) == 20 and len(b) == 5


def test_noniid_contiguous_clients_are_label_skewed():
    ds = synthetic_dataset(200, (4, 4, 3), seed=1)
    ordered = ds.filter_label(1).concatenate(ds.filter_label(0))
    clients = contiguous_clients(ordered, 10, 20)
    assert set(clients[0].labels().tolist()) == {1}
    assert set(clients[9].labels().tolist()) == {0}


def test_synthetic_is_learnable_signal():
    ds = synthetic_dataset(400, seed=0)
    x = ds.x.astype(np.float32)
    y = ds.y
    # class means differ in channel 0
    assert x[y == 1][..., 0].mean() > x[y == 0][..., 0].mean() + 10
