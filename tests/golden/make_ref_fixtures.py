#!/usr/bin/env python3
"""Golden fixtures produced by the REFERENCE's own code, run in the build container (never on the GPU
box; /root/reference does not travel):

    python tests/golden/make_ref_fixtures.py        # writes tests/golden/reference_fixtures.npz

The reference package imports TensorFlow at module top (config.py:6, model.py:6, data_loader.py:6),
which is not installed.  The parts pinned here never call TensorFlow, so a placeholder module is
installed under that name: it provides the two base classes the class statements need
(tf.keras.layers.Layer, tf.keras.Model) and raises on ANY call, so a fixture can only come from code
paths that do not touch TensorFlow.  The package __init__ (which imports train/evaluate and their
plotting stack) is bypassed: config.py, model.py and data_loader.py are loaded as submodules of a bare
package object.  No bytecode is written under /root/reference.

Pinned (reference file:line -> build function, checked in tests/test_reference_fixtures.py):
* get_model_config presets + OneTransConfig defaults   config.py:9-117     -> recommend_amd.config
* PyramidScheduler.get_layer_config                     model.py:280-302    -> OneTransConfig.pyramid_schedule
* FeatureProcessor.fit / process_numerical_feature      data_loader.py:13-58 -> recommend_amd.features
* SequenceProcessor.process_sequence / _multi_sequences data_loader.py:71-101 -> recommend_amd.features
* OneTransDataset sample data + __getitem__             data_loader.py:104-204 -> recommend_amd.features
* DataLoader errors / get_data_info                     data_loader.py:236-297 -> recommend_amd.features
"""

import hashlib
import importlib.util
import json
import os
import sys
import types

import numpy as np

REF = '/root/reference/rank/scaling_up/oneTrans/practice'
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'reference_fixtures.npz')


class _Absent:
    """Any TensorFlow attribute: callable-looking (typing accepts it in annotations) but raising."""

    def __init__(self, path):
        self._path = path

    def __getattr__(self, name):
        return _Absent(f'{self._path}.{name}')

    def __call__(self, *a, **k):
        raise RuntimeError(f'TensorFlow is not installed: {self._path}() was called')


class _TFModule(types.ModuleType):
    def __getattr__(self, name):
        return _Absent(f'tf.{name}')


class _Namespace(_Absent):
    """tf.keras / tf.keras.layers: the listed real classes, every other attribute absent."""

    def __init__(self, path, **real):
        super().__init__(path)
        self.__dict__.update(real)


def load_reference():
    sys.dont_write_bytecode = True
    tf = _TFModule('tensorflow')
    tf.keras = _Namespace('tf.keras', layers=_Namespace('tf.keras.layers', Layer=type('Layer', (), {})),
                          Model=type('Model', (), {}))
    sys.modules['tensorflow'] = tf
    pkg = types.ModuleType('refpractice')
    pkg.__path__ = [REF]
    sys.modules['refpractice'] = pkg
    mods = {}
    for name in ('config', 'model', 'data_loader'):
        spec = importlib.util.spec_from_file_location(f'refpractice.{name}', os.path.join(REF, f'{name}.py'))
        m = importlib.util.module_from_spec(spec)
        sys.modules[spec.name] = m
        spec.loader.exec_module(m)
        mods[name] = m
    return mods


def main():
    ref = load_reference()
    cfgm, modm, dlm = ref['config'], ref['model'], ref['data_loader']
    out = {}
    # ---- config presets (config.py:85-117) and defaults
    presets = {name: cfgm.get_model_config(name).to_dict() for name in ('small', 'default', 'large')}
    out['presets_json'] = np.array(json.dumps(presets, sort_keys=True, default=str))
    # ---- pyramid (model.py:287-302) with the reference's default ratios, at the configs' lengths
    cfg = cfgm.OneTransConfig()
    sched = modm.PyramidScheduler(cfg)
    rows = []
    for L0 in (40, 140, 524, 1036):
        for layer in range(len(cfg.pyramid_ratios) + 1):
            c = sched.get_layer_config(layer, L0)
            q = c['query_indices']
            rows.append((L0, layer, c.get('keep_len', -1), q[0] if q else -1, q[-1] if q else -1,
                         len(q) if q else 0))
    out['pyramid'] = np.array(rows, dtype=np.int64)      # L0, layer, keep_len, first, last, count
    out['pyramid_ratios'] = np.array(cfg.pyramid_ratios, dtype=np.float64)
    # ---- FeatureProcessor (data_loader.py:13-58) on a seeded table
    import pandas as pd
    rng = np.random.default_rng(20261016)
    n = 257
    df = pd.DataFrame({'price': np.concatenate([rng.lognormal(3, 1, n - 2), [5000.0, 0.0]]),
                       'age': rng.integers(18, 80, n).astype(np.float64),
                       'ctr': rng.beta(2, 30, n),
                       'user_id': rng.integers(0, 1000, n), 'item_id': rng.integers(0, 5000, n),
                       'category': rng.integers(0, 50, n)})
    fp = dlm.FeatureProcessor(cfg)
    fp.fit(df)
    probe = np.array([-100.0, 0.0, 1.0, 17.5, 40.0, 100.0, 1e4])
    for f in ('price', 'age', 'ctr'):
        out[f'feat_in_{f}'] = df[f].to_numpy()
        out[f'feat_out_{f}'] = np.asarray(fp.process_numerical_feature(f, probe), dtype=np.float64)
        st = fp.feature_stats[f]
        out[f'feat_stats_{f}'] = np.array([st['mean'], st['std'], st['min'], st['max']], dtype=np.float64)
    for f in ('user_id', 'item_id', 'category'):
        out[f'feat_in_{f}'] = df[f].to_numpy()
        out[f'feat_vocab_{f}'] = np.array(fp.vocab_sizes[f])
    out['feat_probe'] = probe
    # ---- SequenceProcessor (data_loader.py:71-94)
    cfg.max_seq_len = 24                                    # small fixture (the rule does not depend on it)
    sp = dlm.SequenceProcessor(cfg)
    L = cfg.max_seq_len
    out['seq_max_len'] = np.array(L)
    for i, n_ev in enumerate((0, 1, 7, L, L + 9)):
        s = rng.standard_normal((n_ev, 64)).astype(np.float32)
        out[f'seq_in_{i}'] = s
        out[f'seq_out_{i}'] = np.asarray(sp.process_sequence(s, 'click_seq'))
    # ---- SequenceProcessor.process_multi_sequences (data_loader.py:96-101)
    multi = {'click_seq': out['seq_in_2'], 'cart_seq': out['seq_in_0'], 'purchase_seq': out['seq_in_4']}
    got = sp.process_multi_sequences(multi)
    out['multi_keys'] = np.array(list(got))
    for k, v in got.items():
        out[f'multi_out_{k}'] = np.asarray(v)
    # ---- OneTransDataset (data_loader.py:104-204): the reference's synthetic sample (numpy's global
    # generator, seeded here) and its per-sample __getitem__ (unfitted processor: TF-free)
    cfg.max_seq_len = 12
    np.random.seed(7)
    ds = dlm.OneTransDataset(cfg, 'train')
    for k, v in ds.non_seq_data.items():
        out[f'ds_ns_{k}'] = np.asarray(v)
    for t, lst in ds.seq_data.items():
        out[f'ds_seqlen_{t}'] = np.array([len(q) for q in lst])
        # the events themselves (float64 randn) only as a digest: 1000 samples x 3 sequences is ~10 MB
        out[f'ds_seqsha_{t}'] = np.array(hashlib.sha256(np.ascontiguousarray(np.concatenate(lst))).hexdigest())
    for t, v in ds.labels.items():
        out[f'ds_lab_{t}'] = np.asarray(v)
    out['ds_len'] = np.array(len(ds))
    for i in (0, 1, 999):
        ns_i, seq_i, lab_i = ds[i]
        for k, v in ns_i.items():
            out[f'ds_item{i}_ns_{k}'] = np.asarray(v)
        for k, v in seq_i.items():
            out[f'ds_item{i}_seq_{k}'] = np.asarray(v)
        for k, v in lab_i.items():
            out[f'ds_item{i}_lab_{k}'] = np.asarray(v)
    # ---- DataLoader (data_loader.py:236-297): ValueError before loading, info after
    dl = dlm.DataLoader(cfg)
    errs = []
    for get in (dl.get_train_dataset, dl.get_val_dataset, dl.get_test_dataset):
        try:
            get(8)
            errs.append('none')
        except ValueError:
            errs.append('ValueError')
    out['dl_errors'] = np.array(errs)
    out['dl_info_empty'] = np.array(json.dumps(dl.get_data_info()))
    np.savez_compressed(OUT, **out)
    print(f'wrote {OUT}: {len(out)} arrays')


if __name__ == '__main__':
    main()
