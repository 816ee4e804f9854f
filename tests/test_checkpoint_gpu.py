"""Checkpoint format (train.py:281-338: model weights + config.json + training_history.json) and the
device prefetcher of the feature pipeline (data_loader.py:232)."""

import json

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from recommend_amd.data import make_batch
from recommend_amd.features import DevicePrefetcher
from recommend_amd.model import OneTransModel
from recommend_amd.params import init_params
from recommend_amd.trainer import OneTransTrainer

from test_model_gpu import ns_t, small_criteo


def test_save_load_roundtrip(dev, tmp_path):
    cfg = small_criteo('tail', pyramid=True, layers=3)
    P = init_params(cfg, cfg.ns_input_width(), seed=0, perturb=True)
    tr = OneTransTrainer(cfg, model_dir=str(tmp_path), model=OneTransModel(cfg, device=dev, init=P))
    batch = make_batch(16, cfg, seed=7)
    tr.train_step(batch)
    tr.history['train_loss'].append(1.25)
    tr.save_model('ckpt')
    d = tmp_path / 'ckpt'
    assert {p.name for p in d.iterdir()} == {'model_weights.npz', 'config.json', 'training_history.json'}
    assert json.load(open(d / 'config.json'))['hidden_dim'] == cfg.hidden_dim
    tr2 = OneTransTrainer(cfg, model_dir=str(tmp_path), model=OneTransModel(cfg, device=dev, seed=5))
    tr2.load_model(str(d))
    a, b = tr.model.param_dict(), tr2.model.param_dict()
    assert set(a) == set(b)
    for k in a:
        assert np.array_equal(a[k], b[k]), k
    assert tr2.history['train_loss'] == [1.25]
    assert tr2.optimizer.steps_done == tr.optimizer.steps_done == 1     # the warm-up ramp resumes
    assert 'optimizer_steps' not in tr2.history
    ns, seq, _ = batch
    with torch.no_grad():
        pa = tr.model((ns_t(ns, dev), ns_t(seq, dev)))
        pb = tr2.model((ns_t(ns, dev), ns_t(seq, dev)))
    for t in cfg.tasks:
        assert torch.equal(pa[t], pb[t])


def test_evaluate_reports_regression_tasks(dev):
    """evaluate(): AUC for the BCE tasks, mse / mae for a task trained with MSE (train.py:106,
    evaluate.py:52-54)."""
    cfg = small_criteo('head')
    cfg.tasks = ['ctr', 'watch_time']
    tr = OneTransTrainer(cfg, model=OneTransModel(cfg, device=dev, seed=0))
    batches = [make_batch(24, cfg, seed=300 + i) for i in range(2)]
    for b in batches:
        b[2]['watch_time'] = np.linspace(0.0, 1.0, 24, dtype=np.float32).reshape(-1, 1)
    res = tr.evaluate(batches)
    assert set(res) == {'ctr_auc', 'ctr_keras_auc', 'watch_time_mse', 'watch_time_mae'}
    with torch.no_grad():
        p = torch.cat([tr.val_step(b)['probs'][1].cpu() for b in batches]).double().numpy()
    y = np.concatenate([b[2]['watch_time'].reshape(-1) for b in batches]).astype(np.float64)
    assert abs(res['watch_time_mse'] - np.mean((p - y) ** 2)) < 1e-9
    assert abs(res['watch_time_mae'] - np.mean(np.abs(p - y))) < 1e-9


def test_device_prefetcher_feeds_training(dev):
    cfg = small_criteo('head')
    batches = [make_batch(12, cfg, seed=100 + i) for i in range(3)]
    got = list(DevicePrefetcher(iter(batches), dev))
    assert len(got) == 3
    for (ns, seq, lab), (ns2, seq2, lab2) in zip(batches, got):
        for src, dst in ((ns, ns2), (seq, seq2), (lab, lab2)):
            for k in src:
                assert dst[k].device.type == 'cuda'
                assert np.array_equal(np.asarray(src[k]), dst[k].cpu().numpy())
    tr = OneTransTrainer(cfg, model=OneTransModel(cfg, device=dev, seed=0))
    for b in DevicePrefetcher(iter(batches), dev):
        out = tr.train_step(b)
    assert torch.isfinite(out['total_loss']).item()
