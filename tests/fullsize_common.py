"""Shared by tests/golden/make_fullsize_golden.py (writes the golden files in the build container,
oracle on the host cores) and tests/test_fullsize_train_gpu.py (the HIP path on the GPU box):
one full training step at a BASELINE configuration's full size, compared on

* the batch's probabilities (training mode, dropout on), the loss,
* every dense gradient bank (a fixed sample of entries plus the bank's L2 norm),
* the sparse table gradients (the summed gradient of a fixed sample of touched rows + the L2 norm
  over all touched rows),
* the parameters after the optimizer (dense: RMSprop after per-variable clip; tables: clipped
  Adagrad) on the same samples.

Embedding tables are BASELINE-sized on the GPU (C2: 32.4M x 16 + 1M x 64; C4: + a 100M x 64 item
table).  Their values are a hash of the element index that is exactly representable in fp32
(``table_values``), so the GPU fills the full tables and the oracle builds only the rows the batch
touches — remapped to a compact table (``compact_problem``) — with bit-identical contents.
"""

from __future__ import annotations

from typing import Dict, Tuple

import numpy as np

TABLE_SEED = {'emb.ns': 0x1234567, 'emb.seq_item': 0x7654321}
SAMPLES_PER_BANK = 2048
SAMPLE_ROWS = 1024


def _mix(h, xp):
    """murmur3 fmix32 on int64 holding uint32 values (numpy or torch; wraps mod 2^32)."""
    m = 0xFFFFFFFF
    h = h ^ (h >> 16)
    h = (h * 0x85EBCA6B) & m
    h = h ^ (h >> 13)
    h = (h * 0xC2B2AE35) & m
    h = h ^ (h >> 16)
    return h


def table_values_np(rows: np.ndarray, E: int, seed: int) -> np.ndarray:
    """Table rows ``rows`` (global row ids) -> float32 [n, E]: ((hash >> 8) - 2^23) * 2^-27, an exact
    fp32 value in [-1/16, 1/16)."""
    idx = rows.astype(np.int64)[:, None] * E + np.arange(E, dtype=np.int64)[None, :]
    h = ((idx & 0xFFFFFFFF) * 0x9E3779B1 + seed) & 0xFFFFFFFF
    h = _mix(h ^ ((idx >> 32) * 0x85EBCA77 & 0xFFFFFFFF), np)
    return (((h >> 8) - (1 << 23)).astype(np.float32) * np.float32(2.0 ** -27))


def fill_table_device(t, seed: int, chunk_rows: int = 1 << 22, row0: int = 0, row_stride: int = 1,
                      nrows: int = -1) -> None:
    """The same values for every row of the device table ``t`` [rows, E] (torch int64 arithmetic;
    the products are masked to 32 bits, so two's-complement wrap-around does not matter).  Local row
    j holds global row ``row0 + j * row_stride`` (a row-sharded table: row0 = rank, stride = world),
    for the first ``nrows`` rows (all when negative)."""
    import torch
    rows, E = t.shape
    if nrows >= 0:
        rows = nrows
    col = torch.arange(E, device=t.device, dtype=torch.int64)[None, :]
    for r0 in range(0, rows, chunk_rows):
        r = torch.arange(r0, min(rows, r0 + chunk_rows), device=t.device, dtype=torch.int64)[:, None]
        r = r * row_stride + row0
        idx = r * E + col
        h = ((idx & 0xFFFFFFFF) * 0x9E3779B1 + seed) & 0xFFFFFFFF
        h = _mix(h ^ ((idx >> 32) * 0x85EBCA77 & 0xFFFFFFFF), torch)
        t[r0:r0 + r.shape[0]] = ((h >> 8) - (1 << 23)).to(torch.float32) * (2.0 ** -27)


def compact_problem(cfg, batch) -> Tuple[object, tuple, Dict[str, np.ndarray], Dict[str, np.ndarray]]:
    """Oracle view of a batch: ids remapped to the rows it touches.

    Returns (ocfg, obatch, tables, rowmap): ``ocfg`` = cfg with every sparse field's cardinality and
    the item vocabulary shrunk to the touched ids; ``obatch`` = the batch with remapped ids;
    ``tables`` = compact 'emb.ns' / 'emb.seq_item' (float64) with the full tables' values;
    ``rowmap[name][j]`` = full-table row of compact row j."""
    ocfg, obatches, tables, rowmap = compact_problem_multi(cfg, [batch])
    return ocfg, obatches[0], tables, rowmap


def compact_problem_multi(cfg, batches) -> Tuple[object, list, Dict[str, np.ndarray], Dict[str, np.ndarray]]:
    """compact_problem over several batches sharing ONE compact table (the union of the rows any of them
    touches): a multi-step oracle run.  Rows no batch touches never receive a gradient, and Adagrad
    leaves zero-gradient rows (and the tables' clip norms) unchanged, so training on the compact
    tables is training on the full ones."""
    import copy
    from recommend_amd.params import ns_table_offsets
    ocfg = copy.deepcopy(cfg)
    full_off = ns_table_offsets(cfg)
    obatches = [(dict(ns), dict(seq), lab) for (ns, seq, lab) in batches]
    rows_ns, card = [], {}
    for name in cfg.ns_feature_names():
        if name in cfg.sparse_features and any(name in b[0] for b in batches):
            u = np.unique(np.concatenate([b[0][name].reshape(-1) for b in batches if name in b[0]]))
            for ob in obatches:
                if name in ob[0]:
                    ob[0][name] = np.searchsorted(u, ob[0][name]).astype(np.int64)
            card[name] = len(u)
            rows_ns.append(full_off[name] + u)
    ocfg.sparse_features = {k: card.get(k, 1) for k in cfg.sparse_features}
    rowmap, tables = {}, {}
    if rows_ns:
        rowmap['emb.ns'] = np.concatenate(rows_ns)
        tables['emb.ns'] = table_values_np(rowmap['emb.ns'], cfg.ns_embedding_dim, TABLE_SEED['emb.ns']).astype(np.float64)
    if cfg.seq_item_vocab and any(b[1] for b in batches):
        u = np.unique(np.concatenate([v.reshape(-1) for b in batches for v in b[1].values()]))
        for ob in obatches:
            for k, v in ob[1].items():
                ob[1][k] = np.searchsorted(u, v).astype(np.int64)
        ocfg.seq_item_vocab = len(u)
        rowmap['emb.seq_item'] = u
        tables['emb.seq_item'] = table_values_np(u, cfg.seq_feature_dim, TABLE_SEED['emb.seq_item']).astype(np.float64)
    return ocfg, obatches, tables, rowmap


def bank_samples(name: str, size: int) -> np.ndarray:
    """Fixed sample of flat indices of a dense bank (every entry for small banks)."""
    if size <= SAMPLES_PER_BANK:
        return np.arange(size)
    seed = sum(ord(c) * (i + 1) for i, c in enumerate(name))
    return np.sort(np.random.default_rng(seed).choice(size, SAMPLES_PER_BANK, replace=False))


def row_samples(name: str, n: int) -> np.ndarray:
    """Fixed sample of positions into a table's sorted touched-row list."""
    if n <= SAMPLE_ROWS:
        return np.arange(n)
    seed = sum(ord(c) * (i + 3) for i, c in enumerate(name))
    return np.sort(np.random.default_rng(seed).choice(n, SAMPLE_ROWS, replace=False))


def setup_config(name: str):
    """The workload config as the golden step runs it (BASELINE shape; parity-test optimizer settings:
    a smaller dense lr and momentum so one step moves the weights without saturating RMSprop)."""
    from recommend_amd.config import workload_config
    cfg = workload_config(name)
    cfg.optimizer_config = dict(cfg.optimizer_config, dense_lr=0.001, momentum=0.9)
    return cfg


# The reduced-precision training test's trajectory (tests/test_train_lowprec_gpu.py, golden train_T.npz): labels
# from the dense features (data.criteo_batch teacher='dense') and RMSprop at dense lr 1e-4 with momentum 0.9 (an
# optimizer_config the reference's trainer accepts, train.py:60-66), on which the T model learns within 20 steps
# (held-out AUC 0.82 / 0.68, logit std 1.2 / 0.36; tools/lowprec_sweep.py, profiles/r05/lowprec_sweep.log)
LOWPREC_TEACHER = 'dense'
LOWPREC_OPT = {'dense_lr': 1e-4, 'momentum': 0.9}


def lowprec_config():
    cfg = setup_config('T')
    cfg.optimizer_config = dict(cfg.optimizer_config, **LOWPREC_OPT)
    return cfg


BATCH_SEED = 424242
MODEL_SEED = 0


def dropout_seed(model_seed: int = MODEL_SEED, step: int = 1) -> int:
    """The dropout seed OneTransModel.forward_probs uses on its ``step``-th training forward."""
    return ((0x5EED0000 ^ model_seed) + 0x9E3779B9 * step) & 0xFFFFFFFF
