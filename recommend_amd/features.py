"""Feature pipeline: the reference's host-side preprocessing and batching, restated.

Reference: ``practice/data_loader.py``
* ``FeatureProcessor`` (:13-68): per-feature mean/std/min/max fitted on a table; numerical features
  z-scored with ``(x - mean) / (std + 1e-8)`` and clipped to [-3, 3]; categorical vocab = max + 1
  (the reference one-hot encodes, :61-68; the build feeds ids to the embedding tables instead,
  ``one_hot=True`` reproduces the reference output).
* ``SequenceProcessor`` (:71-101): keep the most recent ``max_seq_len`` events, left-pad with zeros;
  an empty sequence becomes zeros ``[max_seq_len, 64]``.
* ``OneTransDataset`` / ``DataLoader`` (:104-297): per-sample processing and a tf.data generator whose
  output signature does not match what it yields (a defect: :220-231) — replaced by vectorised batch
  assembly in the model's input format (dicts of ``[B, 1]`` features, ``[B, L, 64]`` sequences,
  ``{task: [B, 1]}`` labels).
* ``DevicePrefetcher`` (build): the MI355X side of ``dataset.prefetch`` (:232) — the next batch is
  copied host→HBM from pinned memory on a separate HIP stream while the current step runs.
"""

from __future__ import annotations

from typing import Dict, Iterator, List, Optional, Sequence

import numpy as np

from .config import OneTransConfig

Batch = tuple


class FeatureProcessor:
    """data_loader.py:13-68."""

    def __init__(self, config: OneTransConfig, numerical: Optional[Sequence[str]] = None,
                 categorical: Optional[Sequence[str]] = None):
        self.config = config
        self.numerical = list(numerical) if numerical is not None else ['price', 'age', 'ctr']      # :40-42
        self.categorical = (list(categorical) if categorical is not None
                            else ['user_id', 'item_id', 'category', 'brand', 'location', 'device'])  # :44-46
        self.feature_stats: Dict[str, Dict[str, float]] = {}
        self.vocab_sizes: Dict[str, int] = {}

    def fit(self, data) -> 'FeatureProcessor':
        """:22-37.  ``data``: a pandas DataFrame or a dict of 1-D arrays (pandas std is ddof=1)."""
        cols = data.columns if hasattr(data, 'columns') else data.keys()
        for f in self.numerical:
            if f in cols:
                v = np.asarray(data[f], dtype=np.float64)
                self.feature_stats[f] = {'mean': float(v.mean()), 'std': float(v.std(ddof=1)),
                                         'min': float(v.min()), 'max': float(v.max())}
        for f in self.categorical:
            if f in cols:
                self.vocab_sizes[f] = int(np.asarray(data[f]).max() + 1)
        return self

    def process_numerical_feature(self, name: str, values: np.ndarray) -> np.ndarray:
        """:48-58: z-score, clip to [-3, 3]; unfitted features pass through."""
        if name not in self.feature_stats:
            return values
        st = self.feature_stats[name]
        return np.clip((np.asarray(values, dtype=np.float64) - st['mean']) / (st['std'] + 1e-8), -3, 3)

    def process_categorical_feature(self, name: str, values: np.ndarray, one_hot: bool = False) -> np.ndarray:
        """:60-68.  Default: int64 ids for the embedding gather (an id >= vocab raises, like the reference's
        one_hot would silently zero it — ids out of the table are an input error here); ``one_hot``:
        the reference's one-hot rows."""
        if name not in self.vocab_sizes:
            return values
        ids = np.asarray(values).astype(np.int64)
        V = self.vocab_sizes[name]
        if one_hot:
            out = np.zeros(ids.shape + (V,), dtype=np.float32)
            ok = (ids >= 0) & (ids < V)
            out[ok, ids[ok]] = 1.0
            return out
        if ids.size and (ids.min() < 0 or ids.max() >= V):
            raise ValueError(f'{name}: id outside the fitted vocabulary [0, {V})')
        return ids


class SequenceProcessor:
    """data_loader.py:71-101."""

    def __init__(self, config: OneTransConfig, width: int = 64):
        self.max_seq_len = config.max_seq_len
        self.width = width

    def process_sequence(self, seq: np.ndarray) -> np.ndarray:
        """:79-94: keep the last max_seq_len events, left-pad with zeros."""
        seq = np.asarray(seq)
        L = self.max_seq_len
        if len(seq) == 0:
            return np.zeros((L, self.width), dtype=np.float32)
        if len(seq) >= L:
            return seq[-L:]
        pad = [(L - len(seq), 0)] + [(0, 0)] * (seq.ndim - 1)
        return np.pad(seq, pad, mode='constant')

    def pad_batch(self, seqs: Sequence[np.ndarray], dtype=np.float32) -> np.ndarray:
        """process_sequence over a batch, vectorised into one [B, max_seq_len, ...] array (event
        features [., width] or item ids [.])."""
        L = self.max_seq_len
        tail = None
        for s in seqs:
            s = np.asarray(s)
            if len(s):
                tail = s.shape[1:]
                break
        tail = tail if tail is not None else (self.width,)
        out = np.zeros((len(seqs), L) + tuple(tail), dtype=dtype)
        for b, s in enumerate(seqs):
            s = np.asarray(s)
            n = min(len(s), L)
            if n:
                out[b, L - n:] = s[len(s) - n:]
        return out


class OneTransDataset:
    """data_loader.py:104-233 in the model's input format.  ``non_seq``: {name: [N] array},
    ``seq``: {name: list of N per-sample arrays}, ``labels``: {task: [N]}."""

    def __init__(self, config: OneTransConfig, non_seq: Dict[str, np.ndarray], seq: Dict[str, List[np.ndarray]],
                 labels: Dict[str, np.ndarray], processor: Optional[FeatureProcessor] = None):
        self.config = config
        self.non_seq, self.seq, self.labels = non_seq, seq, labels
        self.features = processor or FeatureProcessor(config).fit(non_seq)
        self.sequences = SequenceProcessor(config)

    def __len__(self) -> int:
        return len(next(iter(self.non_seq.values()))) if self.non_seq else 0

    def batch(self, idx: np.ndarray) -> Batch:
        fp = self.features
        ns = {}
        for name, v in self.non_seq.items():
            x = np.asarray(v)[idx]
            if name in fp.vocab_sizes:
                ns[name] = fp.process_categorical_feature(name, x).reshape(-1, 1)
            else:
                ns[name] = fp.process_numerical_feature(name, x).astype(np.float32).reshape(-1, 1)
        seq = {name: self.sequences.pad_batch([lst[i] for i in idx]) for name, lst in self.seq.items()}
        lab = {t: np.asarray(v, dtype=np.float32)[idx].reshape(-1, 1) for t, v in self.labels.items()}
        return ns, seq, lab

    def batches(self, batch_size: int, shuffle: bool = True, seed: int = 0, drop_last: bool = False) -> Iterator[Batch]:
        """:213-233 (generator + shuffle + batch): whole batches assembled at once."""
        order = np.random.default_rng(seed).permutation(len(self)) if shuffle else np.arange(len(self))
        stop = len(order) - (len(order) % batch_size if drop_last else 0)
        for s in range(0, stop, batch_size):
            yield self.batch(order[s:s + batch_size])


class DevicePrefetcher:
    """Overlap the host→HBM copy of batch i+1 with step i (``dataset.prefetch``, data_loader.py:232):
    batches are staged in pinned host memory and copied on a dedicated HIP stream; the consumer's
    stream waits on that copy only when it takes the batch."""

    def __init__(self, batches: Iterator[Batch], device):
        import torch
        self.torch = torch
        self.it = iter(batches)
        self.device = torch.device(device)
        self.stream = torch.cuda.Stream(device=self.device)
        self.next = None
        self._preload()

    def _to_dev(self, d: Dict[str, np.ndarray]):
        torch = self.torch
        return {k: torch.from_numpy(np.ascontiguousarray(v)).pin_memory().to(self.device, non_blocking=True)
                for k, v in d.items()}

    def _preload(self):
        try:
            ns, seq, lab = next(self.it)
        except StopIteration:
            self.next = None
            return
        with self.torch.cuda.stream(self.stream):
            self.next = (self._to_dev(ns), self._to_dev(seq), self._to_dev(lab))
            self.event = self.torch.cuda.Event()
            self.event.record(self.stream)

    def __iter__(self):
        return self

    def __next__(self) -> Batch:
        if self.next is None:
            raise StopIteration
        cur = self.torch.cuda.current_stream(self.device)
        cur.wait_event(self.event)
        out = self.next
        for d in out:                       # the tensors are now used on the consumer's stream
            for t in d.values():
                t.record_stream(cur)
        self._preload()
        return out
