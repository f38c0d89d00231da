"""Streaming metrics (device-resident accumulators, one host sync per epoch).

* ``'accuracy'`` / ``BinaryAccuracy`` — ``dist_model_tf_vgg.py:132``, ``fed_model.py:128``.  Keras
  thresholds the *logits* at 0.5 (it does not know the loss is from logits; quirk Q11).  The
  default here is the correct logit-0 threshold; ``keras_compat=True`` reproduces Keras.
* ``AUC`` — ``secure_fed_model.py:81-82`` computes sklearn ``roc_auc_score`` per batch and
  averages it.  Default here is the exact epoch-level AUC (Mann-Whitney U with tie correction);
  ``mode='per_batch'`` reproduces the reference's batch-mean (skipping single-class batches,
  which crash sklearn in the reference, quirk Q18).
* ``Mean`` — the loss tracker.

Accumulators are torch tensors on the model's device, so a data-parallel ``reduce`` is one
packed all-reduce per epoch.
"""
from __future__ import annotations

from typing import List, Optional

import torch


class Metric:
    name = "metric"

    def reset(self):
        raise NotImplementedError

    def update(self, logits: torch.Tensor, y: torch.Tensor, loss: Optional[torch.Tensor] = None):
        raise NotImplementedError

    def result(self) -> float:
        raise NotImplementedError

    # packed state for cross-replica reduction (sum semantics)
    def state(self) -> List[torch.Tensor]:
        return []

    def set_state(self, tensors: List[torch.Tensor]):
        pass


class Mean(Metric):
    def __init__(self, name="loss", device=None):
        self.name = name
        self.device = device
        self.reset()

    def reset(self):
        self.total = torch.zeros((), dtype=torch.float64, device=self.device)
        self.count = torch.zeros((), dtype=torch.float64, device=self.device)

    def update_value(self, value: torch.Tensor, n: int):
        self.total = self.total + value.detach().double() * n
        self.count = self.count + n

    def update(self, logits, y, loss=None):
        if loss is not None:
            self.update_value(loss, logits.shape[0])

    def result(self):
        c = float(self.count)
        return float(self.total) / c if c else 0.0

    def state(self):
        return [self.total.reshape(1), self.count.reshape(1)]

    def set_state(self, t):
        self.total, self.count = t[0].reshape(()), t[1].reshape(())


class Accuracy(Metric):
    """Binary (1 logit) or categorical (argmax) accuracy."""

    def __init__(self, name="accuracy", threshold: Optional[float] = None, keras_compat=False,
                 device=None):
        self.name = name
        self.threshold = threshold if threshold is not None else (0.5 if keras_compat else 0.0)
        self.device = device
        self.reset()

    def reset(self):
        self.correct = torch.zeros((), dtype=torch.float64, device=self.device)
        self.count = torch.zeros((), dtype=torch.float64, device=self.device)

    def update(self, logits, y, loss=None):
        logits = logits.detach().float()
        if logits.dim() == 1 or logits.shape[-1] == 1:
            pred = (logits.reshape(-1) > self.threshold)
            truth = y.reshape(-1) > 0.5
        else:
            pred = logits.argmax(-1)
            truth = y.argmax(-1) if (y.dim() == 2 and y.shape[-1] == logits.shape[-1]) else y.reshape(-1)
            truth = truth.to(pred.device).long()
        self.correct = self.correct + (pred == truth.to(pred.device)).sum().double()
        self.count = self.count + pred.numel()

    def result(self):
        c = float(self.count)
        return float(self.correct) / c if c else 0.0

    def state(self):
        return [self.correct.reshape(1), self.count.reshape(1)]

    def set_state(self, t):
        self.correct, self.count = t[0].reshape(()), t[1].reshape(())


def exact_auc(scores: torch.Tensor, labels: torch.Tensor) -> float:
    """ROC AUC = P(score_pos > score_neg) + 0.5 P(tie) via average ranks (Mann-Whitney)."""
    s = scores.detach().double().reshape(-1).cpu()
    l = (labels.detach().reshape(-1).cpu() > 0.5)
    npos = int(l.sum())
    nneg = l.numel() - npos
    if npos == 0 or nneg == 0:
        return float("nan")
    order = torch.argsort(s)
    ss = s[order]
    ranks = torch.empty_like(ss)
    n = ss.numel()
    i = 0
    # average ranks over ties
    uniq, inv, counts = torch.unique_consecutive(ss, return_inverse=True, return_counts=True)
    ends = torch.cumsum(counts, 0).double()
    starts = ends - counts.double() + 1
    avg = (starts + ends) / 2
    ranks = avg[inv]
    rank_of = torch.empty(n, dtype=torch.float64)
    rank_of[order] = ranks
    rpos = rank_of[l].sum().item()
    return (rpos - npos * (npos + 1) / 2) / (npos * nneg)


class AUC(Metric):
    def __init__(self, name="auc", mode: str = "exact", device=None):
        self.name = name
        self.mode = mode
        self.device = device
        self.reset()

    def reset(self):
        self.scores: List[torch.Tensor] = []
        self.labels: List[torch.Tensor] = []
        self.batch_aucs: List[float] = []

    def update(self, logits, y, loss=None):
        # a copy: the fused backend returns VIEWS of its output buffer, rewritten by the next step
        s = logits.detach().float().reshape(-1).clone()
        l = y.detach().reshape(-1).float()
        if self.mode == "per_batch":
            a = exact_auc(s, l)
            if a == a:
                self.batch_aucs.append(a)
        else:
            self.scores.append(s)
            self.labels.append(l.to(s.device))

    def result(self):
        if self.mode == "per_batch":
            return sum(self.batch_aucs) / len(self.batch_aucs) if self.batch_aucs else float("nan")
        if not self.scores:
            return float("nan")
        return exact_auc(torch.cat(self.scores), torch.cat(self.labels))

    def gather_arrays(self):
        if not self.scores:
            return None, None
        return torch.cat(self.scores), torch.cat(self.labels)


def get(identifier, keras_compat: bool = False, device=None) -> Metric:
    if isinstance(identifier, Metric):
        return identifier
    name = str(identifier).lower()
    if name in ("accuracy", "acc", "binary_accuracy", "categorical_accuracy"):
        return Accuracy("accuracy", keras_compat=keras_compat, device=device)
    if name in ("auc", "auroc"):
        return AUC("auc", device=device)
    raise ValueError(f"unknown metric {identifier!r}")


class BinaryAccuracy(Accuracy):
    def __init__(self, name="binary_accuracy", threshold=None, keras_compat=False, device=None):
        super().__init__(name, threshold, keras_compat, device)
