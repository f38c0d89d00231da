"""Native input pipeline (csrc/data/loader.cpp): PNG decode + resize, shuffle buffer, batcher (T7)."""
import os

import numpy as np
import pytest
import torch

from idc_models_amd.data import ArrayDataset, native, prepare_for_training

pytestmark = pytest.mark.skipif(not native.available(), reason="_idc_data not built")


def _tf_resize_ref(img: np.ndarray, S: int) -> np.ndarray:
    """numpy TF2 bilinear resize (half-pixel centres, edge clamp) on uint8 intensities."""
    h, w, _ = img.shape
    out = np.zeros((S, S, 3), np.float64)
    f = img.astype(np.float64)
    for y in range(S):
        fy = (y + 0.5) * h / S - 0.5
        y0 = int(np.floor(fy)); wy = fy - y0
        ya, yb = min(max(y0, 0), h - 1), min(max(y0 + 1, 0), h - 1)
        for x in range(S):
            fx = (x + 0.5) * w / S - 0.5
            x0 = int(np.floor(fx)); wx = fx - x0
            xa, xb = min(max(x0, 0), w - 1), min(max(x0 + 1, 0), w - 1)
            top = f[ya, xa] + (f[ya, xb] - f[ya, xa]) * wx
            bot = f[yb, xa] + (f[yb, xb] - f[yb, xa]) * wx
            out[y, x] = top + (bot - top) * wy
    return np.clip(np.rint(out), 0, 255).astype(np.uint8)


def test_decode_png_modes_and_resize(tmp_path):
    from PIL import Image
    rng = np.random.default_rng(0)
    rgb = rng.integers(0, 256, (50, 50, 3), dtype=np.uint8)
    small = rng.integers(0, 256, (37, 44, 3), dtype=np.uint8)  # IDC border patches are < 50x50
    gray = rng.integers(0, 256, (50, 50), dtype=np.uint8)
    rgba = rng.integers(0, 256, (50, 50, 4), dtype=np.uint8)
    paths = []
    for name, arr, mode in [("rgb", rgb, "RGB"), ("small", small, "RGB"), ("gray", gray, "L"),
                            ("rgba", rgba, "RGBA")]:
        p = str(tmp_path / f"{name}.png")
        Image.fromarray(arr, mode).save(p)
        paths.append(p)
    pal = Image.fromarray(rgb, "RGB").convert("P")
    pal.save(str(tmp_path / "pal.png"))
    paths.append(str(tmp_path / "pal.png"))
    x, bad = native.decode_pngs(paths, 50, workers=3)
    assert bad == []
    np.testing.assert_array_equal(x[0], rgb)
    ref = _tf_resize_ref(small, 50)
    assert np.abs(x[1].astype(int) - ref.astype(int)).max() <= 1
    np.testing.assert_array_equal(x[2], np.repeat(gray[..., None], 3, -1))
    np.testing.assert_array_equal(x[3], rgba[..., :3])
    np.testing.assert_array_equal(x[4], np.asarray(pal.convert("RGB")))


def test_decode_reports_bad_files(tmp_path):
    p = tmp_path / "broken.png"
    p.write_bytes(b"not a png at all")
    x, bad = native.decode_pngs([str(p), str(tmp_path / "missing.png")], 10)
    assert [i for i, _ in bad] == [0, 1]
    assert not x.any()


@pytest.mark.parametrize("buf", [1, 7, 1000, 5000])
def test_shuffle_order_is_permutation_and_seeded(buf):
    idx = np.arange(3000, dtype=np.int64) * 3
    a = native.shuffle_order(idx, buf, 11)
    b = native.shuffle_order(idx, buf, 11)
    c = native.shuffle_order(idx, buf, 12)
    np.testing.assert_array_equal(np.sort(a), idx)
    np.testing.assert_array_equal(a, b)
    assert np.array_equal(a, c) == (buf == 1)
    if buf == 1:
        np.testing.assert_array_equal(a, idx)  # a one-element buffer is the identity
    if buf == 7:
        # window semantics: element i can only be emitted once element i - buf + 1 was read
        pos = np.empty(len(idx), np.int64)
        pos[np.searchsorted(idx, a)] = np.arange(len(a))
        assert (pos >= np.arange(len(idx)) - buf + 1).all()


@pytest.mark.parametrize("drop", [False, True])
def test_batch_loader_matches_python_gather(drop):
    rng = np.random.default_rng(1)
    x = rng.integers(0, 256, (203, 6, 6, 3), dtype=np.uint8)
    y = rng.integers(0, 2, 203).astype(np.int64)
    it = native.PrefetchIterator(x, y, 32, slots=3, threads=3)
    for ep in range(3):
        order = rng.permutation(203)
        got = list(it.epoch(order, drop))
        nb = 203 // 32 if drop else -(-203 // 32)
        assert len(got) == nb
        for b, (xb, yb) in enumerate(got):
            sel = order[b * 32:(b + 1) * 32]
            np.testing.assert_array_equal(xb.numpy(), x[sel])
            np.testing.assert_array_equal(yb.numpy(), y[sel])
    it.close()


def test_batch_loader_early_exit_then_new_epoch():
    x = np.arange(100 * 4, dtype=np.float32).reshape(100, 4)
    y = np.arange(100, dtype=np.int64)
    it = native.PrefetchIterator(x, y, 10, slots=2, threads=2)
    for i, _ in enumerate(it.epoch(np.arange(100))):
        if i == 3:
            break
    got = [yb.numpy() for _, yb in it.epoch(np.arange(100)[::-1].copy())]
    np.testing.assert_array_equal(np.concatenate(got), np.arange(100)[::-1])
    it.close()


def test_batched_dataset_uses_native_path_and_covers_epoch():
    rng = np.random.default_rng(2)
    x = rng.integers(0, 256, (150, 4, 4, 3), dtype=np.uint8)
    y = np.arange(150, dtype=np.int64)
    ds = prepare_for_training(ArrayDataset(x, y), batch_size=16)
    seen = []
    for xb, yb in ds:
        assert xb.dtype == torch.uint8 and xb.shape[1:] == (4, 4, 3)
        np.testing.assert_array_equal(xb.numpy(), x[yb.numpy()])
        seen.append(yb.numpy())
    assert ds._prefetcher is not None
    assert sorted(np.concatenate(seen).tolist()) == list(range(150))
    e2 = np.concatenate([yb.numpy() for _, yb in ds])
    assert not np.array_equal(np.concatenate(seen), e2)  # reshuffled every epoch


@pytest.mark.gpu
def test_device_prefetch_delivers_cuda_batches():
    rng = np.random.default_rng(3)
    x = rng.integers(0, 256, (300, 50, 50, 3), dtype=np.uint8)
    y = np.arange(300, dtype=np.int64)  # labels = row ids, so every row can be checked
    ds = prepare_for_training(ArrayDataset(x, y), batch_size=64).prefetch_to("cuda:0")
    for _ in range(2):
        seen = []
        for xb, yb in ds:
            assert xb.is_cuda and yb.is_cuda
            xb = xb.float() * 1.0  # consume on the current stream (ordered after the copy)
            ids = yb.cpu().numpy()
            np.testing.assert_array_equal(xb.cpu().numpy().astype(np.uint8), x[ids])
            seen.append(ids)
        assert sorted(np.concatenate(seen).tolist()) == list(range(300))
    ds._prefetcher.close()
