"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restated Keras/TF 2.12 primitives used by the reference model and trainer, and the
counter-based dropout mask the build uses (so dropout-on runs are reproducible on
both sides).  numpy versions; torch versions live in onetrans_ref.py.
"""

from __future__ import annotations

import numpy as np

KERAS_EPSILON = 1e-7          # tf.keras.backend.epsilon()
RMS_EPS = 1e-6                # RMSNorm eps, model.py:14


def fmix32(h: np.ndarray) -> np.ndarray:
    """murmur3 finaliser on uint32 (wrapping arithmetic)."""
    h = h.astype(np.uint32)
    h ^= h >> np.uint32(16)
    h = (h * np.uint32(0x85EBCA6B)).astype(np.uint32)
    h ^= h >> np.uint32(13)
    h = (h * np.uint32(0xC2B2AE35)).astype(np.uint32)
    h ^= h >> np.uint32(16)
    return h


def dropout_keep(seed: int, site: int, index: np.ndarray, rate: float) -> np.ndarray:
    """Build dropout mask: element ``index`` (flat (b*I + p)*d + n within a layer's
    [B, I, d] residual branch) of dropout site ``site`` (2*layer + {0: attention,
    1: FFN}, model.py:193,198) is kept iff fmix32(index*0x9E3779B1 + seed ^ site*0x85EBCA77)
    >= rate * 2^32.  Kept values are scaled by 1/(1-rate) like tf.nn.dropout."""
    with np.errstate(over='ignore'):
        idx = index.astype(np.uint64) & np.uint64(0xFFFFFFFF)
        h = (idx * np.uint64(0x9E3779B1) + np.uint64(seed & 0xFFFFFFFF)) & np.uint64(0xFFFFFFFF)
        h = h.astype(np.uint32) ^ np.uint32((site * 0x85EBCA77) & 0xFFFFFFFF)
        h = fmix32(h)
    thr = np.uint64(min(int(round(rate * 4294967296.0)), 4294967295))
    return h.astype(np.uint64) >= thr


def dropout_threshold(rate: float) -> int:
    return min(int(round(rate * 4294967296.0)), 4294967295)


def keras_bce(y: np.ndarray, p: np.ndarray) -> float:
    """tf.keras.losses.BinaryCrossentropy(from_logits=False), SUM_OVER_BATCH_SIZE
    (train.py:84-87; TF backend clips p to [eps, 1-eps] then adds eps inside the logs)."""
    eps = KERAS_EPSILON
    pc = np.clip(p, eps, 1.0 - eps)
    bce = -(y * np.log(pc + eps) + (1.0 - y) * np.log(1.0 - pc + eps))
    return float(np.mean(bce))


def keras_bce_logits(y: np.ndarray, z: np.ndarray) -> float:
    """The same loss on a sigmoid head's output in Keras 2.12 (the cached ``_keras_logits`` path):
    tf.nn.sigmoid_cross_entropy_with_logits = max(z, 0) - z y + log(1 + exp(-|z|)), SUM_OVER_BATCH_SIZE."""
    return float(np.mean(np.maximum(z, 0.0) - z * y + np.log1p(np.exp(-np.abs(z)))))


def clip_by_norm(g: np.ndarray, clip: float) -> np.ndarray:
    """tf.clip_by_norm (train.py:135): g * clip / max(||g||_2, clip)."""
    l2 = np.sqrt(np.sum(g * g))
    return g * clip / max(l2, clip)


def rmsprop_update(w, g, v, m, lr, rho, eps, momentum):
    """Keras 2.12 RMSprop.update_step, centered=False: v = rho v + (1-rho) g^2;
    inc = lr g rsqrt(v + eps); momentum: m = mom m + inc, w -= m; else w -= inc."""
    v = rho * v + (1.0 - rho) * g * g
    inc = lr * g / np.sqrt(v + eps)
    if momentum > 0:
        m = momentum * m + inc
        w = w - m
    else:
        w = w - inc
    return w, v, m


def adagrad_sparse_update(w, acc, rows, g_rows, lr, eps):
    """Keras 2.12 Adagrad on a de-duplicated IndexedSlices gradient:
    acc[r] += g^2; w[r] -= lr g / sqrt(acc[r] + eps)."""
    acc = acc.copy(); w = w.copy()
    acc[rows] += g_rows * g_rows
    w[rows] -= lr * g_rows / np.sqrt(acc[rows] + eps)
    return w, acc


def auc_exact(y: np.ndarray, s: np.ndarray) -> float:
    """Rank-based ROC AUC (Mann-Whitney U with average ranks for ties) — the
    sklearn.metrics.roc_auc_score estimator."""
    y = np.asarray(y).reshape(-1).astype(np.float64)
    s = np.asarray(s).reshape(-1).astype(np.float64)
    order = np.argsort(s, kind='mergesort')
    ss = s[order]
    ranks = np.empty(len(s))
    i = 0
    n = len(s)
    while i < n:
        j = i
        while j + 1 < n and ss[j + 1] == ss[i]:
            j += 1
        ranks[order[i:j + 1]] = 0.5 * (i + j) + 1.0
        i = j + 1
    npos = y.sum()
    nneg = n - npos
    if npos == 0 or nneg == 0:
        return float('nan')
    return float((ranks[y > 0.5].sum() - npos * (npos + 1) / 2.0) / (npos * nneg))


def auc_keras(y: np.ndarray, p: np.ndarray, num_thresholds: int = 200) -> float:
    """tf.keras.metrics.AUC() default (train.py:101): ROC, 200 thresholds,
    summation_method='interpolation' (trapezoid)."""
    eps = KERAS_EPSILON
    thr = [(i + 1) * 1.0 / (num_thresholds - 1) for i in range(num_thresholds - 2)]
    thr = np.array([0.0 - eps] + thr + [1.0 + eps])
    y = np.asarray(y).reshape(-1) > 0.5
    p = np.asarray(p).reshape(-1)
    pred = p[None, :] > thr[:, None]
    tp = (pred & y[None]).sum(1).astype(np.float64)
    fp = (pred & ~y[None]).sum(1).astype(np.float64)
    fn = (~pred & y[None]).sum(1).astype(np.float64)
    tn = (~pred & ~y[None]).sum(1).astype(np.float64)
    rec = np.divide(tp, tp + fn, out=np.zeros_like(tp), where=(tp + fn) > 0)
    fpr = np.divide(fp, fp + tn, out=np.zeros_like(fp), where=(fp + tn) > 0)
    heights = (rec[:-1] + rec[1:]) / 2.0
    return float(np.sum((fpr[:-1] - fpr[1:]) * heights))
