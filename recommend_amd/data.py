"""Synthetic input batches (SURVEY §8d "Synthetic inputs").

* ``create_sample_batch`` — the reference's input contract
  (``data_loader.py:301-329``): user features int U[0,100), item features int
  U[0,1000), context features float U[0,1), each ``[B,1]``; every sequence
  ``[B, L_i, 64]`` U[0,1).  Differences, all recorded in DESIGN.md: the NS
  ints are returned as float32 (defect D3: the reference concatenates int32 with
  float32 at ``model.py:253``), the sequence lengths are given instead of drawn
  per call (``data_loader.py:319``), and labels are Bernoulli draws from a fixed
  teacher instead of uniform floats (defect D7, ``data_loader.py:327``).
* ``criteo_batch`` — the Criteo-shape workload of BASELINE.json configs 2-5:
  13 dense floats ``log1p(lognormal(0,1))``, 26 categorical ids
  ``Zipf(1.1) mod cardinality`` and 3 item-id sequences.

All generators are numpy ``Generator(PCG64)``: same seed => same batch, here and
on the GPU box.
"""

from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import numpy as np

from .config import OneTransConfig

Batch = Tuple[Dict[str, np.ndarray], Dict[str, np.ndarray], Dict[str, np.ndarray]]


def _teacher_labels(rng_seed: int, B: int, tasks: List[str], signal: np.ndarray) -> Dict[str, np.ndarray]:
    """Bernoulli(sigmoid(teacher logit)); the teacher is a fixed function of the inputs
    (seed 7) so AUC after training is meaningful (> 0.5)."""
    rng = np.random.Generator(np.random.PCG64(rng_seed))
    labels = {}
    for ti, t in enumerate(tasks):
        z = signal[:, ti % signal.shape[1]]
        p = 1.0 / (1.0 + np.exp(-z))
        labels[t] = (rng.random(B) < p).astype(np.float32).reshape(B, 1)
    return labels


def create_sample_batch(batch_size: int, config: OneTransConfig, seq_lens: Optional[List[int]] = None,
                        seed: int = 1000) -> Batch:
    """data_loader.py:301-329 with the deviations listed in the module docstring."""
    rng = np.random.Generator(np.random.PCG64(seed))
    B = batch_size
    fc = config.feature_config
    ns: Dict[str, np.ndarray] = {}
    for name in fc['user_features']:
        ns[name] = rng.integers(0, 100, size=(B, 1)).astype(np.float32)
    for name in fc['item_features']:
        ns[name] = rng.integers(0, 1000, size=(B, 1)).astype(np.float32)
    for name in fc['context_features']:
        ns[name] = rng.random((B, 1), dtype=np.float32)
    seq: Dict[str, np.ndarray] = {}
    lens = seq_lens or getattr(config, '_seq_lens', None) or [10] * len(fc['sequence_features'])
    for name, L in zip(fc['sequence_features'], lens):
        seq[name] = rng.random((B, L, config.seq_feature_dim), dtype=np.float32)
    trng = np.random.Generator(np.random.PCG64(7))
    nsmat = np.concatenate([ns[n] for n in config.ns_feature_names() if n in ns], axis=1)
    a = trng.normal(size=(nsmat.shape[1], 2)) / np.sqrt(nsmat.shape[1])
    z = (nsmat / np.maximum(nsmat.max(axis=0, keepdims=True), 1.0)) @ a
    z = 3.0 * (z - z.mean(axis=0))
    labels = _teacher_labels(seed + 1, B, config.tasks, z)
    return ns, seq, labels


def criteo_batch(batch_size: int, config: OneTransConfig, seq_lens: Optional[List[int]] = None,
                 seed: int = 1000, teacher: str = 'ids') -> Batch:
    """Criteo-shape batch: dense I* float32 [B,1]; sparse C* int64 [B,1]; seqs int64 [B,L_i].

    ``teacher`` picks the label signal: 'ids' (default; every feature, the sparse ids through a hashed
    per-id effect — learnable only by memorising ids) or 'dense' (the 13 dense features alone, 4x the
    weight: a signal a few hundred steps of training pick up, for tests that need a model that has
    learned)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    B = batch_size
    fc = config.feature_config
    ns: Dict[str, np.ndarray] = {}
    trng = np.random.Generator(np.random.PCG64(7))
    signal = np.zeros((B, 2))
    dense_signal = np.zeros((B, 2))
    for name in config.ns_feature_names():
        if name in config.sparse_features:
            card = config.sparse_features[name]
            ids = (rng.zipf(1.1, size=(B, 1)) - 1) % card
            ns[name] = ids.astype(np.int64)
            u = trng.normal(size=(1024, 2)) * 0.3
            signal += u[(ids[:, 0] * 2654435761) % 1024]
        else:
            v = np.log1p(rng.lognormal(0.0, 1.0, size=(B, 1))).astype(np.float32)
            ns[name] = v
            w = trng.normal(size=(1, 2)) * 0.3
            signal += v * w
            dense_signal += v * w * 4.0
    seq: Dict[str, np.ndarray] = {}
    lens = seq_lens or getattr(config, '_seq_lens', None)
    vocab = config.seq_item_vocab
    for name, L in zip(fc['sequence_features'], lens):
        seq[name] = ((rng.zipf(1.1, size=(B, L)) - 1) % vocab).astype(np.int64)
    if teacher == 'dense':
        signal = dense_signal
    elif teacher != 'ids':
        raise ValueError(f"teacher {teacher!r}: 'ids' or 'dense'")
    labels = _teacher_labels(seed + 1, B, config.tasks, signal - signal.mean(axis=0))
    return ns, seq, labels


def make_batch(batch_size: int, config: OneTransConfig, seed: int = 1000,
               seq_lens: Optional[List[int]] = None, teacher: str = 'ids') -> Batch:
    """Dispatch on the config: Criteo-shape when embedding tables are configured (``teacher``: criteo_batch)."""
    if config.sparse_features or config.seq_item_vocab:
        return criteo_batch(batch_size, config, seq_lens, seed, teacher)
    return create_sample_batch(batch_size, config, seq_lens, seed)
