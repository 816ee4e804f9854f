"""CPU: the build's restatements against fixtures produced by the reference's own code
(tests/golden/make_ref_fixtures.py runs config.py / model.py / data_loader.py of the reference in the
build container; TensorFlow-free code paths only)."""

import json
import os

import numpy as np
import pytest

from recommend_amd.config import OneTransConfig, get_model_config
from recommend_amd.features import FeatureProcessor, SequenceProcessor

FIX = np.load(os.path.join(os.path.dirname(__file__), 'golden', 'reference_fixtures.npz'))


@pytest.mark.parametrize('name', ['small', 'default', 'large'])
def test_presets_match_reference(name):
    """config.py:85-117: every reference hyper-parameter of every preset."""
    ref = json.loads(str(FIX['presets_json']))[name]
    got = get_model_config(name).to_dict()
    for k, v in ref.items():
        assert got[k] == v, (name, k, got.get(k), v)


def test_pyramid_matches_reference_scheduler():
    """model.py:287-302 run by the reference: layer 0 keeps the same tail; from layer 1 on the
    reference's indices (against L0) fall outside the pruned tensor (D2) and the build keeps
    min(keep_len, I_l) tail tokens of the current layer instead."""
    cfg = OneTransConfig()
    np.testing.assert_allclose(FIX['pyramid_ratios'], cfg.pyramid_ratios)
    rows = FIX['pyramid']
    for L0 in np.unique(rows[:, 0]):
        sched = cfg.pyramid_schedule(int(L0))
        cur = int(L0)
        for (_, layer, keep_len, first, last, count) in rows[rows[:, 0] == L0]:
            if layer >= cfg.num_layers:
                continue
            if keep_len < 0:                                       # past the ratio list: no pruning
                assert sched[layer]['keep'] == sched[layer]['in_len']
                continue
            assert (first, last, count) == (L0 - keep_len, L0 - 1, keep_len)   # indices against L0
            assert sched[layer]['in_len'] == cur
            assert sched[layer]['keep'] == min(keep_len, cur)
            if layer > 0:
                assert last >= cur           # D2: the reference gathers past the end of the pruned tensor
            cur = sched[layer]['keep']
    bad = OneTransConfig()
    bad.pyramid_fix = False
    with pytest.raises(IndexError):                                 # TF-CPU raises on the same gather
        bad.pyramid_schedule(140)


def test_feature_processor_matches_reference():
    """data_loader.py:22-58: fitted stats and z-score/clip outputs of the reference's FeatureProcessor."""
    data = {f: FIX[f'feat_in_{f}'] for f in ('price', 'age', 'ctr', 'user_id', 'item_id', 'category')}
    fp = FeatureProcessor(OneTransConfig()).fit(data)
    for f in ('price', 'age', 'ctr'):
        st = fp.feature_stats[f]
        np.testing.assert_allclose([st['mean'], st['std'], st['min'], st['max']], FIX[f'feat_stats_{f}'],
                                   rtol=1e-12)
        np.testing.assert_allclose(fp.process_numerical_feature(f, FIX['feat_probe']), FIX[f'feat_out_{f}'],
                                   rtol=1e-12, atol=1e-15)
    for f in ('user_id', 'item_id', 'category'):
        assert fp.vocab_sizes[f] == int(FIX[f'feat_vocab_{f}'])


def test_sequence_processor_matches_reference():
    """data_loader.py:79-94: the reference's truncation / left padding, lengths 0 .. max+9."""
    cfg = OneTransConfig()
    cfg.max_seq_len = int(FIX['seq_max_len'])
    sp = SequenceProcessor(cfg)
    ins = [FIX[f'seq_in_{i}'] for i in range(5)]
    for i, s in enumerate(ins):
        np.testing.assert_array_equal(sp.process_sequence(s), FIX[f'seq_out_{i}'])
    pb = sp.pad_batch(ins)
    for i in range(5):
        np.testing.assert_array_equal(pb[i], FIX[f'seq_out_{i}'])
