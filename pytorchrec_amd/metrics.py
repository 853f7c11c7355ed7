"""CTR metrics: the reference's IMetric family is
ranking-only with a hard-coded 99-sample layout (torchrec/metric/IMetric.py:17-26,
metrics.py:13-15), so CTR evaluation needs AUC and log-loss.  Each metric is a
callable ``m(prediction_logits, target) -> float`` with a ``name`` (what
``IModel.evaluate`` records), computed on the host in float64."""
from __future__ import annotations

import numpy as np


class AUC:
    name = "auc"

    def __call__(self, prediction, target) -> float:
        p = np.asarray(prediction, np.float64).reshape(-1)
        y = np.asarray(target, np.float64).reshape(-1) > 0.5
        n_pos, n_neg = int(y.sum()), int((~y).sum())
        if n_pos == 0 or n_neg == 0:
            return float("nan")
        order = np.argsort(p, kind="mergesort")
        ranks = np.empty(len(p), np.float64)
        sp = p[order]
        i = 0
        while i < len(sp):  # average ranks over ties
            j = i
            while j + 1 < len(sp) and sp[j + 1] == sp[i]:
                j += 1
            ranks[order[i:j + 1]] = (i + j) / 2.0 + 1.0
            i = j + 1
        return float((ranks[y].sum() - n_pos * (n_pos + 1) / 2.0) / (n_pos * n_neg))


class LogLoss:
    name = "logloss"

    def __call__(self, prediction, target) -> float:
        z = np.asarray(prediction, np.float64).reshape(-1)
        y = np.asarray(target, np.float64).reshape(-1)
        if z.size == 0:
            return float("nan")
        return float(np.mean(np.maximum(z, 0) - z * y + np.log1p(np.exp(-np.abs(z)))))


_metric_classes = {"auc": AUC, "logloss": LogLoss}


def get_metric(name: str):
    n = name.strip().lower()
    if n not in _metric_classes:
        raise ValueError(f"unknown metric {name!r}; choose from {sorted(_metric_classes)}")
    return _metric_classes[n]()
