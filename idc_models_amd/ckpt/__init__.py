"""Checkpointing: Keras-layout HDF5 weights + framework-native full-state resume.

Weights (``save_weights`` / ``load_weights``; reference ``fed_model.py:103-105,138``):
Keras HDF5 layout written through libhdf5 by the native ``_idc_h5`` module:
root attrs ``layer_names`` / ``backend`` / ``keras_version``; one group per top-level layer with a
``weight_names`` attr; datasets at ``/<layer>/<sublayer>/<var>:0``.  The nested
``Sequential([base, GAP, Dense])`` puts every backbone weight under the backbone's group, exactly
like Keras.  Loading matches weights BY NAME (robust to the freeze-dependent weight order, SURVEY
§2.6), and also accepts a bare backbone file (Keras ``*_notop.h5`` layout, flat layer groups).

Full state (``save_checkpoint`` / ``load_checkpoint``): every weight, the optimizer slots, epoch /
round counters and RNG state, stored with ``torch.save`` as plain tensors/primitives so it loads
with ``weights_only=True``.
"""
from __future__ import annotations

import os
from typing import Dict, List, Tuple

import numpy as np
import torch

KERAS_VERSION = b"2.2.4-tf"


def _h5():
    try:
        from ..utils.hostext import import_host_ext
        return import_host_ext("_idc_h5")
    except ImportError:
        import sys
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        sys.path.insert(0, root)
        from tools.build_native import build_h5
        build_h5(verbose=False)
        from .. import _idc_h5
        return _idc_h5


def _layer_entries(layer) -> List[Tuple[str, torch.Tensor]]:
    """(Keras weight name, tensor) pairs of a top-level layer in Keras ``weights`` order."""
    names = layer.keras_weight_names()
    return list(zip(names, layer.weights))


def save_weights(net, path: str) -> None:
    h5 = _h5()
    top = [l for l in net.layers] if hasattr(net, "layers") else [net]
    attrs, dsets = [], []
    layer_names = []
    for l in top:
        if getattr(l, "keras_class", "") == "InputLayer":
            continue
        layer_names.append(l.name.encode())
        entries = _layer_entries(l)
        attrs.append((f"/{l.name}", "weight_names", [n.encode() for n, _ in entries], False))
        for n, t in entries:
            dsets.append((f"/{l.name}/{n}", t.detach().float().cpu().numpy()))
        if not entries:
            # Keras still writes an (empty) group for weightless layers
            attrs[-1] = (f"/{l.name}", "weight_names", [], False)
            dsets.append((f"/{l.name}/.keep", np.zeros((0,), np.float32)))
    attrs.append(("/", "layer_names", layer_names, False))
    attrs.append(("/", "backend", [b"tensorflow"], True))
    attrs.append(("/", "keras_version", [KERAS_VERSION], True))
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    h5.write(path, attrs, dsets)


def read_weights(path: str) -> Dict[str, np.ndarray]:
    """``{'<top layer>/<sublayer>/<var>:0': array}`` from a Keras-layout HDF5 file."""
    attrs, dsets = _h5().read(path)
    out = {}
    for k, v in dsets.items():
        if k.endswith("/.keep"):
            continue
        out[k.lstrip("/")] = np.asarray(v)
    return out


def _name_map(net) -> Dict[str, torch.Tensor]:
    """Every weight tensor of ``net`` under all the names a file may use for it."""
    m = {}
    top = net.layers if hasattr(net, "layers") else [net]
    for l in top:
        for n, t in _layer_entries(l):
            m[f"{l.name}/{n}"] = t   # nested layout: model/sublayer/var:0 or layer/layer/var:0
            m[n] = t                 # flat layout (bare backbone file): sublayer/var:0
            if "/" not in n.split(":")[0] or n.count("/") == 1:
                m[f"{n.split('/')[0]}/{n}"] = t  # Keras flat-group layout: layer/layer/var:0
    return m


def load_weights(net, path: str, strict: bool = False) -> List[str]:
    """Load by name; returns the list of model weights that were NOT found in the file."""
    data = read_weights(path)
    names = _name_map(net)
    loaded = set()
    with torch.no_grad():
        for k, arr in data.items():
            t = names.get(k)
            if t is None:
                # strip a leading group that is not ours (e.g. a differently named backbone)
                parts = k.split("/", 1)
                if len(parts) == 2:
                    t = names.get(parts[1])
            if t is None:
                continue
            a = torch.from_numpy(np.ascontiguousarray(arr))
            if tuple(a.shape) != tuple(t.shape):
                raise ValueError(f"shape mismatch for {k}: file {tuple(a.shape)} vs model {tuple(t.shape)}")
            t.copy_(a.to(t.device, t.dtype))
            loaded.add(id(t))
    missing = [n for n, t in names.items() if id(t) not in loaded and "/" in n]
    if strict and missing:
        raise KeyError(f"weights missing from {path}: {missing[:5]}...")
    return missing


def save_checkpoint(model, path: str, extra=None) -> None:
    net = model.net
    state = {"weights": [t.detach().cpu() for t in net.weight_tensors()],
             "trainable": [bool(l.trainable) for l in _all_layers(net)],
             "epoch": int((extra or {}).get("epoch", 0)),
             "extra": {k: v for k, v in (extra or {}).items() if isinstance(v, (int, float, str, bool))},
             "rng_cpu": torch.get_rng_state()}
    if model.optimizer is not None:
        state["optimizer"] = {"name": model.optimizer.name,
                              "iterations": int(model.optimizer.iterations),
                              "slots": {k: v.detach().cpu() for k, v in model.optimizer.state_tensors().items()
                                        if v is not None}}
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    torch.save(state, path)


def load_checkpoint(model, path: str) -> dict:
    state = torch.load(path, map_location="cpu", weights_only=True)
    net = model.net
    with torch.no_grad():
        for t, v in zip(net.weight_tensors(), state["weights"]):
            t.copy_(v.to(t.device))
    opt = state.get("optimizer")
    if opt and model.optimizer is not None and opt["name"] == model.optimizer.name:
        model.optimizer.iterations = opt["iterations"]
        for k, v in opt["slots"].items():
            cur = model.optimizer.state_tensors().get(k)
            if cur is not None and cur.shape == v.shape:
                cur.copy_(v.to(cur.device))
    if "rng_cpu" in state:
        torch.set_rng_state(state["rng_cpu"])
    return {"epoch": state.get("epoch", 0), **state.get("extra", {})}


def _all_layers(net):
    for l in getattr(net, "layers", []):
        yield l
        if hasattr(l, "layers") and l is not net:
            yield from _all_layers(l)
