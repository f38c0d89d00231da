"""Training-curve plot, reproducing the reference ``log`` helper.

Reference: ``dist_model_tf_vgg.py:67-101`` (also mobile/dense): concatenate the phase-1 and
phase-2 histories (acc, val_acc, loss, val_loss), draw a two-panel figure with a "Start Fine
Tuning" marker at ``initial_epochs-1``, save ``{path}/logs/plot_dev{num_devices}.png`` and print
both history dicts.  ``ylim`` is applied for mobile/dense (``dist_model_tf_mobile.py:84,93``).
"""
from __future__ import annotations

import os
from typing import Optional, Tuple


def log(path: str, history, history_fine, num_devices: int, initial_epochs: int = 10,
        ylim: Optional[Tuple[Tuple[float, float], Tuple[float, float]]] = None,
        acc_key: str = "accuracy", printer=print) -> str:
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    h1, h2 = history.history, history_fine.history
    acc = list(h1.get(acc_key, [])) + list(h2.get(acc_key, []))
    val_acc = list(h1.get("val_" + acc_key, [])) + list(h2.get("val_" + acc_key, []))
    loss = list(h1.get("loss", [])) + list(h2.get("loss", []))
    val_loss = list(h1.get("val_loss", [])) + list(h2.get("val_loss", []))

    fig = plt.figure(figsize=(8, 8))
    plt.subplot(2, 1, 1)
    plt.plot(acc, label="Training Accuracy")
    plt.plot(val_acc, label="Validation Accuracy")
    if ylim:
        plt.ylim(list(ylim[0]))
    plt.plot([initial_epochs - 1, initial_epochs - 1], plt.ylim(), label="Start Fine Tuning")
    plt.legend(loc="lower right")
    plt.title("Training and Validation Accuracy")
    plt.subplot(2, 1, 2)
    plt.plot(loss, label="Training Loss")
    plt.plot(val_loss, label="Validation Loss")
    if ylim:
        plt.ylim(list(ylim[1]))
    plt.plot([initial_epochs - 1, initial_epochs - 1], plt.ylim(), label="Start Fine Tuning")
    plt.legend(loc="upper right")
    plt.title("Training and Validation Loss")
    plt.xlabel("epoch")
    os.makedirs(os.path.join(path, "logs"), exist_ok=True)
    out = os.path.join(path, "logs", f"plot_dev{num_devices}.png")
    plt.savefig(out)
    plt.close(fig)
    if printer is not None:
        printer(h1)
        printer(h2)
    return out
