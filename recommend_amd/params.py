"""Canonical parameter layout + Keras-compatible initialisation.

Every trainable variable of the reference model (``model.py``) maps onto one slice
of a named bank below; Keras Dense kernels keep their ``[in, out]`` layout.

=====================  ===============================  ==============================================
name                   shape                            reference variable(s)
=====================  ===============================  ==============================================
tok.ns.kernel          [F_ns, L_NS*d]                   Tokenizer.ns_tokenizer Dense (model.py:211-214)
tok.ns.bias            [L_NS*d]                         "
tok.seq.kernel         [n_seq, E, d]                    Tokenizer.seq_projections[i] (model.py:217-219)
tok.seq.bias           [n_seq, d]                       "
tok.sep                [1, d]                           Tokenizer.sep_embedding (model.py:222)
blk.{l}.norm1/norm2    [d]                              OneTransBlock.norm1/norm2 scale (model.py:173-174)
blk.{l}.wqkv           [G, d, 3d]                       g=0: W{q,k,v}_shared, g=1+i: W{q,k,v}_dedicated[i]
                                                        (model.py:38-54); columns [q | k | v]
blk.{l}.wo             [d, d]                           MixedMHA.Wo (model.py:57)
blk.{l}.w1, b1         [G, d, f], [G, f]                MixedFFN ffn_shared / ffn_dedicated[i] Dense(f)
blk.{l}.w2, b2         [G, f, d], [G, d]                ... Dense(d) (model.py:136-147)
out_norm               [d]                              OneTransModel.output_norm (model.py:322)
head.w1, head.b1       [T, d, d/2], [T, d/2]            task_heads[task] Dense(d/2, gelu) (model.py:325-330)
head.w2, head.b2       [T, d/2], [T]                    task_heads[task] Dense(1, sigmoid)
emb.ns                 [sum(card), e]                   build extension: NS id -> row; the per-field tables
                                                        are concatenated (row offset ns_table_offsets())
emb.seq_item           [vocab, E]                       build extension: seq item id -> row
=====================  ===============================  ==============================================

``keras_variables(cfg)`` lists each reference variable as a 2-D strided view
``(bank, offset, rows, cols, row_stride)`` — the granularity of the per-tensor
``clip_by_norm`` in ``train.py:134-135``.
"""

from __future__ import annotations

from typing import Dict, List, Tuple

import numpy as np

from .config import OneTransConfig


def _glorot(rng: np.random.Generator, fan_in: int, fan_out: int) -> np.ndarray:
    """Keras glorot_uniform: U(-l, l), l = sqrt(6 / (fan_in + fan_out))."""
    lim = np.sqrt(6.0 / (fan_in + fan_out))
    return rng.uniform(-lim, lim, size=(fan_in, fan_out))


def dense_param_shapes(cfg: OneTransConfig, f_ns: int) -> Dict[str, Tuple[int, ...]]:
    d, f, G, L = cfg.hidden_dim, cfg.ffn_dim, cfg.num_groups, cfg.num_ns_tokens
    E = cfg.seq_feature_dim
    nseq = len(cfg.feature_config['sequence_features'])
    shapes = {
        'tok.ns.kernel': (f_ns, L * d), 'tok.ns.bias': (L * d,),
        'tok.seq.kernel': (nseq, E, d), 'tok.seq.bias': (nseq, d),
        'tok.sep': (1, d),
    }
    for l in range(cfg.num_layers):
        shapes.update({
            f'blk.{l}.norm1': (d,), f'blk.{l}.norm2': (d,),
            f'blk.{l}.wqkv': (G, d, 3 * d), f'blk.{l}.wo': (d, d),
            f'blk.{l}.w1': (G, d, f), f'blk.{l}.b1': (G, f),
            f'blk.{l}.w2': (G, f, d), f'blk.{l}.b2': (G, d),
        })
    shapes['out_norm'] = (d,)
    T = len(cfg.tasks)
    shapes.update({'head.w1': (T, d, d // 2), 'head.b1': (T, d // 2), 'head.w2': (T, d // 2), 'head.b2': (T,)})
    return shapes


def ns_table_offsets(cfg: OneTransConfig) -> Dict[str, int]:
    """Row offset of every NS id feature inside the concatenated 'emb.ns' table."""
    off, out = 0, {}
    for name in cfg.ns_feature_names():
        if name in cfg.sparse_features:
            out[name] = off
            off += cfg.sparse_features[name]
    out['__total__'] = off
    return out


def init_params(cfg: OneTransConfig, f_ns: int, seed: int = 0, perturb: bool = False,
                with_tables: bool = True) -> Dict[str, np.ndarray]:
    """Keras default init in a fixed draw order (float64 host arrays).

    ``perturb=True`` additionally randomises biases (+-0.1) and norm scales (1 +- 0.1) so
    parity tests exercise every parameter (Keras zero biases / unit scales would hide
    bias-path bugs)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    d, f, G, L = cfg.hidden_dim, cfg.ffn_dim, cfg.num_groups, cfg.num_ns_tokens
    E = cfg.seq_feature_dim
    nseq = len(cfg.feature_config['sequence_features'])
    P: Dict[str, np.ndarray] = {}
    P['tok.ns.kernel'] = _glorot(rng, f_ns, L * d)
    P['tok.ns.bias'] = np.zeros(L * d)
    P['tok.seq.kernel'] = np.stack([_glorot(rng, E, d) for _ in range(nseq)])
    P['tok.seq.bias'] = np.zeros((nseq, d))
    P['tok.sep'] = rng.uniform(-0.05, 0.05, size=(1, d))       # Keras Embedding init
    for l in range(cfg.num_layers):
        P[f'blk.{l}.norm1'] = np.ones(d)
        P[f'blk.{l}.norm2'] = np.ones(d)
        wqkv = np.empty((G, d, 3 * d))
        for part in range(3):                                  # q, k, v: shared then dedicated
            for g in range(G):
                wqkv[g, :, part * d:(part + 1) * d] = _glorot(rng, d, d)
        P[f'blk.{l}.wqkv'] = wqkv
        P[f'blk.{l}.wo'] = _glorot(rng, d, d)
        P[f'blk.{l}.w1'] = np.stack([_glorot(rng, d, f) for _ in range(G)])
        P[f'blk.{l}.b1'] = np.zeros((G, f))
        P[f'blk.{l}.w2'] = np.stack([_glorot(rng, f, d) for _ in range(G)])
        P[f'blk.{l}.b2'] = np.zeros((G, d))
    P['out_norm'] = np.ones(d)
    T = len(cfg.tasks)
    P['head.w1'] = np.empty((T, d, d // 2)); P['head.b1'] = np.zeros((T, d // 2))
    P['head.w2'] = np.empty((T, d // 2)); P['head.b2'] = np.zeros(T)
    for ti in range(T):
        P['head.w1'][ti] = _glorot(rng, d, d // 2)
        P['head.w2'][ti] = _glorot(rng, d // 2, 1)[:, 0]
    if perturb:
        for k in list(P):
            if k.endswith(('bias', '.b1', '.b2')):
                P[k] = P[k] + rng.uniform(-0.1, 0.1, size=P[k].shape)
            elif k.endswith(('norm1', 'norm2', 'out_norm')):
                P[k] = P[k] + rng.uniform(-0.1, 0.1, size=P[k].shape)
    if with_tables:
        P.update(init_tables(cfg, seed + 1))
    return P


def init_tables(cfg: OneTransConfig, seed: int) -> Dict[str, np.ndarray]:
    """Embedding tables, Keras Embedding init U(-0.05, 0.05) (host float64; small configs only)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    T = {}
    if cfg.sparse_features:
        total = ns_table_offsets(cfg)['__total__']
        T['emb.ns'] = rng.uniform(-0.05, 0.05, size=(total, cfg.ns_embedding_dim))
    if cfg.seq_item_vocab:
        T['emb.seq_item'] = rng.uniform(-0.05, 0.05, size=(cfg.seq_item_vocab, cfg.seq_feature_dim))
    return T


def keras_variables(cfg: OneTransConfig, shapes: Dict[str, Tuple[int, ...]],
                    f_ns: int = None) -> List[Tuple[str, int, int, int, int]]:
    """Reference variables as 2-D strided views (bank, elem_offset, rows, cols, row_stride).

    Each entry is one ``tf.Variable`` of the reference model, i.e. one ``clip_by_norm`` unit
    (train.py:134-135)."""
    d, f, G = cfg.hidden_dim, cfg.ffn_dim, cfg.num_groups
    out = []

    def whole(name):
        shp = shapes[name]
        n = int(np.prod(shp))
        cols = shp[-1]
        out.append((name, 0, n // cols, cols, cols))

    F = shapes['tok.ns.kernel'][0] if f_ns is None else f_ns      # real rows (bank may be padded)
    out.append(('tok.ns.kernel', 0, F, shapes['tok.ns.kernel'][1], shapes['tok.ns.kernel'][1]))
    whole('tok.ns.bias')
    nseq, E, _ = shapes['tok.seq.kernel']
    for i in range(nseq):
        out.append(('tok.seq.kernel', i * E * d, E, d, d))
        out.append(('tok.seq.bias', i * d, 1, d, d))
    whole('tok.sep')
    for l in range(cfg.num_layers):
        whole(f'blk.{l}.norm1')
        for part in range(3):
            for g in range(G):
                out.append((f'blk.{l}.wqkv', g * d * 3 * d + part * d, d, d, 3 * d))
        whole(f'blk.{l}.wo')
        for g in range(G):
            out.append((f'blk.{l}.w1', g * d * f, d, f, f))
            out.append((f'blk.{l}.b1', g * f, 1, f, f))
            out.append((f'blk.{l}.w2', g * f * d, f, d, d))
            out.append((f'blk.{l}.b2', g * d, 1, d, d))
        whole(f'blk.{l}.norm2')
    whole('out_norm')
    dh = d // 2
    for ti in range(len(cfg.tasks)):
        out.append(('head.w1', ti * d * dh, d, dh, dh))
        out.append(('head.b1', ti * dh, 1, dh, dh))
        out.append(('head.w2', ti * dh, 1, dh, dh))
        out.append(('head.b2', ti, 1, 1, 1))
    return out
