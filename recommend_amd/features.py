"""Feature pipeline: the reference's host-side preprocessing and batching, restated.

Reference: ``practice/data_loader.py``
* ``FeatureProcessor`` (:13-68): per-feature mean/std/min/max fitted on a table; numerical features
  z-scored with ``(x - mean) / (std + 1e-8)`` and clipped to [-3, 3]; categorical vocab = max + 1
  (one-hot by default, as the reference :61-68; the dataset's batches opt in to int64 ids for the
  embedding tables with ``one_hot=False``).
* ``SequenceProcessor`` (:71-101): keep the most recent ``max_seq_len`` events, left-pad with zeros;
  an empty sequence becomes zeros ``[max_seq_len, 64]``.
* ``OneTransDataset`` / ``DataLoader`` (:104-297): the reference surface (per-sample ``__getitem__``,
  ``load_datasets`` / ``get_*_dataset`` / ``get_data_info``); its tf.data generator, whose output
  signature does not match what it yields (a defect: :220-231), is replaced by vectorised batch
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

    def process_categorical_feature(self, name: str, values: np.ndarray, one_hot: bool = True) -> np.ndarray:
        """:60-68.  Default: the reference's one-hot rows (``tf.one_hot``: an id outside [0, vocab) gives
        an all-zero row).  ``one_hot=False`` is the build's explicit opt-in for the embedding path: int64
        ids, and an id outside the fitted vocabulary raises (it would address no table row)."""
        if name not in self.vocab_sizes:
            return values
        ids = np.asarray(values).astype(np.int64)
        V = self.vocab_sizes[name]
        if one_hot:
            out = np.zeros(ids.shape + (V,), dtype=np.float32)
            ok = (ids >= 0) & (ids < V)
            out[ok, ids[ok]] = 1.0
            return out
        return self.process_categorical_ids(name, ids)

    def process_categorical_ids(self, name: str, values: np.ndarray) -> np.ndarray:
        """Embedding-path categorical encoding (build extension): int64 ids checked against the vocab."""
        ids = np.asarray(values).astype(np.int64)
        V = self.vocab_sizes.get(name)
        if V is not None and ids.size and (ids.min() < 0 or ids.max() >= V):
            raise ValueError(f'{name}: id outside the fitted vocabulary [0, {V})')
        return ids


class SequenceProcessor:
    """data_loader.py:71-101."""

    def __init__(self, config: OneTransConfig, width: int = 64):
        self.max_seq_len = config.max_seq_len
        self.width = width

    def process_sequence(self, sequence_data: np.ndarray, sequence_type: Optional[str] = None) -> np.ndarray:
        """:75-94: keep the last max_seq_len events, left-pad with zeros (an empty sequence: float64
        zeros [max_seq_len, 64], as the reference).  ``sequence_type`` is accepted and unused, like the
        reference's."""
        seq = np.asarray(sequence_data)
        L = self.max_seq_len
        if len(seq) == 0:
            return np.zeros((L, self.width))
        if len(seq) >= L:
            return seq[-L:]
        pad = [(L - len(seq), 0)] + [(0, 0)] * (seq.ndim - 1)
        return np.pad(seq, pad, mode='constant')

    def process_multi_sequences(self, sequences: Dict[str, np.ndarray]) -> Dict[str, np.ndarray]:
        """:96-101: process_sequence on each behaviour sequence, keyed by its type."""
        return {t: self.process_sequence(s, t) for t, s in sequences.items()}

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
    """data_loader.py:104-233.

    Reference form ``OneTransDataset(config, data_path)``: ``load_data`` fills the dataset with the
    reference's synthetic sample (:119-154: 1000 samples, ``user_id``/``item_id``/``price``/``category``/
    ``time``, one random-length ``[n, 64]`` sequence per configured sequence feature, 0/1 labels; the
    reference defines no file format) and the feature processor stays unfitted, so ``__getitem__``
    passes values through exactly as the reference's does.  Build form: ``non_seq`` ({name: [N]}),
    ``seq`` ({name: list of N per-sample arrays}) and ``labels`` ({task: [N]}) given directly; the
    processor is then fitted on ``non_seq`` (``fit_processor``) and categorical features become
    embedding ids.  ``batch`` / ``batches`` / ``get_dataset`` assemble whole batches in the model's
    input format (dicts of ``[B, 1]`` features, ``[B, L, 64]`` sequences, ``{task: [B, 1]}`` labels)."""

    CATEGORICAL = ('user_id', 'item_id', 'category')          # :164

    def __init__(self, config: OneTransConfig, data_path: Optional[str] = None,
                 non_seq: Optional[Dict[str, np.ndarray]] = None, seq: Optional[Dict[str, List[np.ndarray]]] = None,
                 labels: Optional[Dict[str, np.ndarray]] = None, processor: Optional[FeatureProcessor] = None,
                 fit_processor: Optional[bool] = None):
        self.config = config
        self.feature_processor = processor or FeatureProcessor(config)
        self.sequence_processor = SequenceProcessor(config)
        self.non_seq_data: Dict[str, np.ndarray] = dict(non_seq or {})
        self.seq_data: Dict[str, List[np.ndarray]] = dict(seq or {})
        self.labels: Dict[str, np.ndarray] = dict(labels or {})
        if data_path:
            self.load_data(data_path)
        if fit_processor is None:
            fit_processor = processor is None and non_seq is not None
        if fit_processor and self.non_seq_data:
            self.feature_processor.fit(self.non_seq_data)

    # reference attribute names (:107-115) and the build's short ones
    features = property(lambda self: self.feature_processor)
    sequences = property(lambda self: self.sequence_processor)

    def load_data(self, data_path: str) -> None:
        """:119-123 -> _create_sample_data (the reference loads no file)."""
        self._create_sample_data()

    def _create_sample_data(self, num_samples: int = 1000) -> None:
        """:125-154 (numpy's global generator, as the reference)."""
        self.non_seq_data = {
            'user_id': np.random.randint(0, 1000, num_samples),
            'item_id': np.random.randint(0, 5000, num_samples),
            'price': np.random.uniform(0, 1000, num_samples),
            'category': np.random.randint(0, 50, num_samples),
            'time': np.random.randint(0, 24, num_samples)}
        self.seq_data = {}
        for t in self.config.feature_config['sequence_features']:
            self.seq_data[t] = [np.random.randn(np.random.randint(1, self.config.max_seq_len + 1), 64)
                                for _ in range(num_samples)]
        self.labels = {'ctr': np.random.randint(0, 2, num_samples).astype(np.float32),
                       'cvr': np.random.randint(0, 2, num_samples).astype(np.float32)}

    def __len__(self) -> int:
        return len(next(iter(self.non_seq_data.values()))) if self.non_seq_data else 0

    def _process_features(self, idx: int):
        """:156-185, one sample (categorical: the one-hot default of the processor)."""
        fp, sp = self.feature_processor, self.sequence_processor
        ns = {}
        for name, v in self.non_seq_data.items():
            if isinstance(v, np.ndarray):
                x = np.array([v[idx]])
                ns[name] = (fp.process_categorical_feature(name, x) if name in self.CATEGORICAL
                            else fp.process_numerical_feature(name, x))[0]
        seq = {t: sp.process_sequence(lst[idx], t) for t, lst in self.seq_data.items() if idx < len(lst)}
        return ns, seq

    def __getitem__(self, idx: int):
        """:193-204."""
        ns, seq = self._process_features(idx)
        lab = {t: v[idx] for t, v in self.labels.items() if idx < len(v)}
        return ns, seq, lab

    def batch(self, idx: np.ndarray) -> Batch:
        fp = self.feature_processor
        ns = {}
        for name, v in self.non_seq_data.items():
            x = np.asarray(v)[idx]
            if name in fp.vocab_sizes:
                ns[name] = fp.process_categorical_feature(name, x, one_hot=False).reshape(-1, 1)
            else:
                ns[name] = np.asarray(fp.process_numerical_feature(name, x), dtype=np.float32).reshape(-1, 1)
        seq = {name: self.sequence_processor.pad_batch([lst[i] for i in idx]) for name, lst in self.seq_data.items()}
        lab = {t: np.asarray(v, dtype=np.float32)[idx].reshape(-1, 1) for t, v in self.labels.items()}
        return ns, seq, lab

    def batches(self, batch_size: int, shuffle: bool = True, seed: int = 0, drop_last: bool = False) -> Iterator[Batch]:
        """:213-233 (generator + shuffle + batch): whole batches assembled at once."""
        order = np.random.default_rng(seed).permutation(len(self)) if shuffle else np.arange(len(self))
        stop = len(order) - (len(order) % batch_size if drop_last else 0)
        for s in range(0, stop, batch_size):
            yield self.batch(order[s:s + batch_size])

    def get_dataset(self, batch_size: int = 32, shuffle: bool = True, seed: int = 0) -> List[Batch]:
        """get_tf_dataset (:206-233) without TensorFlow: the list of (non_seq, seq, labels) batches the
        trainer's train_step takes (the reference's generator signature does not match what it yields)."""
        return list(self.batches(batch_size, shuffle=shuffle, seed=seed))

    get_tf_dataset = get_dataset


class DataLoader:
    """data_loader.py:236-297: train / val / test datasets."""

    def __init__(self, config: OneTransConfig):
        self.config = config
        self.train_dataset: Optional[OneTransDataset] = None
        self.val_dataset: Optional[OneTransDataset] = None
        self.test_dataset: Optional[OneTransDataset] = None

    def load_datasets(self, train_path: str, val_path: str, test_path: str) -> None:
        """:245-254."""
        self.train_dataset = OneTransDataset(self.config, train_path)
        self.val_dataset = OneTransDataset(self.config, val_path)
        self.test_dataset = OneTransDataset(self.config, test_path)

    def _get(self, ds, which: str, batch_size, shuffle: bool):
        if batch_size is None:
            batch_size = self.config.batch_size
        if ds is None:
            raise ValueError(f'{which} dataset not loaded')          # :262, :272, :282
        return ds.get_dataset(batch_size, shuffle=shuffle)

    def get_train_dataset(self, batch_size: Optional[int] = None):
        return self._get(self.train_dataset, 'train', batch_size, True)

    def get_val_dataset(self, batch_size: Optional[int] = None):
        return self._get(self.val_dataset, 'validation', batch_size, False)

    def get_test_dataset(self, batch_size: Optional[int] = None):
        return self._get(self.test_dataset, 'test', batch_size, False)

    def get_data_info(self) -> Dict:
        """:286-297."""
        info = {}
        if self.train_dataset:
            info['train_samples'] = len(self.train_dataset)
        if self.val_dataset:
            info['val_samples'] = len(self.val_dataset)
        if self.test_dataset:
            info['test_samples'] = len(self.test_dataset)
        return info


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
