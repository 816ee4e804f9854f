"""Evaluation metrics of the reference trainer/evaluator.

* ``auc`` — exact rank-based ROC AUC (Mann-Whitney U, average ranks for ties): the primary
  parity estimator, identical on both sides.
* ``keras_auc`` — ``tf.keras.metrics.AUC()`` defaults (train.py:101, evaluate.py:45): ROC over 200
  thresholds, trapezoidal interpolation.
Host-side numpy (metric computation is off the timed path).
"""

from __future__ import annotations

import numpy as np


def auc(labels, scores) -> float:
    y = np.asarray(labels, dtype=np.float64).reshape(-1)
    s = np.asarray(scores, dtype=np.float64).reshape(-1)
    order = np.argsort(s, kind='mergesort')
    ss = s[order]
    n = len(s)
    # average ranks for ties
    ranks = np.empty(n)
    boundaries = np.nonzero(np.diff(ss))[0] + 1
    starts = np.concatenate([[0], boundaries])
    ends = np.concatenate([boundaries, [n]])
    for a, b in zip(starts, ends):
        ranks[order[a:b]] = 0.5 * (a + b - 1) + 1.0
    pos = y > 0.5
    npos, nneg = pos.sum(), n - pos.sum()
    if npos == 0 or nneg == 0:
        return float('nan')
    return float((ranks[pos].sum() - npos * (npos + 1) / 2.0) / (npos * nneg))


def keras_auc(labels, probs, num_thresholds: int = 200) -> float:
    eps = 1e-7
    thr = np.array([0.0 - eps] + [(i + 1) / (num_thresholds - 1) for i in range(num_thresholds - 2)] + [1.0 + eps])
    y = np.asarray(labels).reshape(-1) > 0.5
    p = np.asarray(probs, dtype=np.float64).reshape(-1)
    ps = np.sort(p)
    # counts of predictions > thr via searchsorted (O(n log n))
    gt = len(p) - np.searchsorted(ps, thr, side='right')
    pos_sorted = np.sort(p[y])
    tp = len(pos_sorted) - np.searchsorted(pos_sorted, thr, side='right')
    fp = gt - tp
    P, N = y.sum(), (~y).sum()
    fn, tn = P - tp, N - fp
    rec = np.divide(tp, tp + fn, out=np.zeros(len(thr)), where=(tp + fn) > 0)
    fpr = np.divide(fp, fp + tn, out=np.zeros(len(thr)), where=(fp + tn) > 0)
    return float(np.sum((fpr[:-1] - fpr[1:]) * (rec[:-1] + rec[1:]) / 2.0))
