"""CPU: the feature pipeline (recommend_amd/features.py) against data_loader.py:13-233's rules."""

import numpy as np
import pandas as pd
import pytest

from recommend_amd.config import OneTransConfig
from recommend_amd.features import FeatureProcessor, OneTransDataset, SequenceProcessor


def test_zscore_clip_matches_pandas():
    """data_loader.py:22-58: pandas mean/std (ddof=1), (x - mean)/(std + 1e-8), clip [-3, 3]."""
    rng = np.random.default_rng(0)
    df = pd.DataFrame({'price': np.concatenate([rng.normal(50, 10, 200), [500.0, -400.0]]),
                       'user_id': rng.integers(0, 37, 202)})
    fp = FeatureProcessor(OneTransConfig()).fit(df)
    st = fp.feature_stats['price']
    assert st['mean'] == pytest.approx(df['price'].mean()) and st['std'] == pytest.approx(df['price'].std())
    assert st['min'] == df['price'].min() and st['max'] == df['price'].max()
    z = fp.process_numerical_feature('price', df['price'].values)
    want = np.clip((df['price'] - df['price'].mean()) / (df['price'].std() + 1e-8), -3, 3).values
    np.testing.assert_allclose(z, want, rtol=1e-12)
    assert z.max() == 3 and z.min() == -3                           # the two outliers are clipped
    assert fp.vocab_sizes['user_id'] == df['user_id'].max() + 1
    assert np.array_equal(fp.process_numerical_feature('age', np.array([7.0])), [7.0])   # unfitted: as is


def test_categorical_one_hot_default_and_ids():
    fp = FeatureProcessor(OneTransConfig()).fit({'item_id': np.array([0, 3, 4])})
    oh = fp.process_categorical_feature('item_id', np.array([4, 1, 9]))              # data_loader.py:60-68
    assert oh.shape == (3, 5) and oh[0, 4] == 1 and oh[1, 1] == 1 and oh.sum() == 2   # id 9: all-zero row
    ids = fp.process_categorical_feature('item_id', np.array([4, 0]), one_hot=False)  # embedding-path opt-in
    assert ids.dtype == np.int64 and ids.tolist() == [4, 0]
    with pytest.raises(ValueError):
        fp.process_categorical_feature('item_id', np.array([5]), one_hot=False)


def test_sequence_pad_truncate():
    """data_loader.py:79-94: keep the most recent max_seq_len events, left-pad with zeros."""
    cfg = OneTransConfig()
    cfg.max_seq_len = 4
    sp = SequenceProcessor(cfg, width=2)
    s = np.arange(12, dtype=np.float32).reshape(6, 2)
    assert np.array_equal(sp.process_sequence(s), s[-4:])
    short = sp.process_sequence(s[:1])
    assert np.array_equal(short, np.array([[0, 0], [0, 0], [0, 0], [0, 1]]))
    assert np.array_equal(sp.process_sequence(np.zeros((0, 2))), np.zeros((4, 2)))
    seqs = [s, s[:1], s[:0], s[:4]]
    pb = sp.pad_batch(seqs)
    assert pb.shape == (4, 4, 2)
    for b, q in enumerate(seqs):
        assert np.array_equal(pb[b], sp.process_sequence(q))
    ids = sp.pad_batch([np.array([5, 6, 7, 8, 9]), np.array([3])], dtype=np.int64)    # item-id sequences
    assert ids.tolist() == [[6, 7, 8, 9], [0, 0, 0, 3]]


def test_dataset_batches():
    cfg = OneTransConfig()
    cfg.max_seq_len = 8
    rng = np.random.default_rng(1)
    N = 50
    non_seq = {'user_id': rng.integers(0, 100, N), 'price': rng.uniform(0, 10, N)}
    seq = {'click_seq': [rng.standard_normal((int(rng.integers(0, 12)), 64)) for _ in range(N)]}
    labels = {'ctr': rng.integers(0, 2, N), 'cvr': rng.integers(0, 2, N)}
    ds = OneTransDataset(cfg, non_seq=non_seq, seq=seq, labels=labels)
    bs = list(ds.batches(16, shuffle=True, seed=3))
    assert [b[0]['user_id'].shape[0] for b in bs] == [16, 16, 16, 2]
    ns, sq, lab = bs[0]
    assert ns['user_id'].dtype == np.int64 and ns['user_id'].shape == (16, 1)
    assert ns['price'].dtype == np.float32 and np.abs(ns['price']).max() <= 3
    assert sq['click_seq'].shape == (16, 8, 64) and lab['ctr'].shape == (16, 1)
    again = list(ds.batches(16, shuffle=True, seed=3))
    assert all(np.array_equal(a[1]['click_seq'], b[1]['click_seq']) for a, b in zip(bs, again))
    seen = np.concatenate([b[0]['user_id'][:, 0] for b in ds.batches(16, shuffle=False)])
    assert np.array_equal(seen, non_seq['user_id'])
    assert sum(1 for _ in ds.batches(16, drop_last=True)) == 3


def test_dataloader_surface():
    """data_loader.py:236-297: unloaded datasets raise ValueError; load_datasets fills the reference's
    1000-sample synthetic sets; batches feed the trainer's (non_seq, seq, labels) form."""
    from recommend_amd import DataLoader
    cfg = OneTransConfig()
    cfg.max_seq_len = 6
    dl = DataLoader(cfg)
    for get in (dl.get_train_dataset, dl.get_val_dataset, dl.get_test_dataset):
        with pytest.raises(ValueError):
            get()
    assert dl.get_data_info() == {}
    np.random.seed(0)
    dl.load_datasets('train', 'val', 'test')
    assert dl.get_data_info() == {'train_samples': 1000, 'val_samples': 1000, 'test_samples': 1000}
    bs = dl.get_val_dataset(batch_size=256)
    assert [b[0]['user_id'].shape[0] for b in bs] == [256, 256, 256, 232]
    ns, seq, lab = bs[0]
    assert set(seq) == set(cfg.feature_config['sequence_features'])
    assert seq['click_seq'].shape == (256, 6, 64) and lab['ctr'].shape == (256, 1)
    ns1, seq1, lab1 = dl.val_dataset[0]
    assert ns1['user_id'] == dl.val_dataset.non_seq_data['user_id'][0]      # unfitted processor: as is
    assert seq1['click_seq'].shape == (6, 64)
