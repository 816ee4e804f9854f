"""Two-stage cached serving (recommend_amd/serving.py, paper §3.5.1) vs the full forward: every
candidate's probabilities equal OneTransModel.forward on the expanded batch (the candidate's NS
features with its request's sequences) and the CPU oracle's."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from recommend_amd.data import make_batch
from recommend_amd.model import OneTransModel
from recommend_amd.params import init_params
from recommend_amd.serving import OneTransServer
from oracle import onetrans_ref as R

from test_model_gpu import c1, ns_t, small_criteo

CASES = {
    'criteo_head': lambda: small_criteo('head'),
    'criteo_tail': lambda: small_criteo('tail'),
    'criteo_tail_pyramid': lambda: small_criteo('tail', pyramid=True, layers=3),
    'criteo_head_pyramid': lambda: small_criteo('head', pyramid=True, layers=3),
    'criteo_d128': lambda: small_criteo('head', d=128, H=4, f=256, Lns=12, seq_lens=(20, 20, 20)),
    # deep pyramid: later layers keep fewer tokens than there are NS tokens (S side dropped)
    'criteo_deep_pyramid': lambda: _deep(small_criteo('tail', pyramid=True, layers=4, Lns=6)),
    'c1_head': lambda: c1('head'),
}


def _deep(cfg):
    cfg.pyramid_ratios = [0.5, 0.2, 0.1, 0.05]
    return cfg


def expand(seq, req):
    return {k: v[req] for k, v in seq.items()}


@pytest.mark.parametrize('case', list(CASES))
def test_cached_serving_matches_forward(dev, case):
    cfg = CASES[case]()
    Rq, C = 5, 23
    P = init_params(cfg, cfg.ns_input_width(), seed=0, perturb=True)
    model = OneTransModel(cfg, device=dev, init=P)
    ns_r, seq_r, _ = make_batch(Rq, cfg, seed=2000)            # request side: sequences
    ns_c, _, _ = make_batch(C, cfg, seed=3000)                 # candidate side: NS features
    req = np.random.default_rng(1).integers(0, Rq, C)
    req[:Rq] = np.arange(Rq)                                   # every request has a candidate
    srv = OneTransServer(model)
    cache = srv.encode_requests(ns_t(seq_r, dev))
    got = srv.score(cache, torch.from_numpy(req), ns_t(ns_c, dev))
    seq_full = expand(seq_r, req)
    with torch.no_grad():
        full = model((ns_t(ns_c, dev), ns_t(seq_full, dev)), training=False)
    ref = R.forward(R.to_torch(P), cfg, R.to_torch(ns_c), R.to_torch(seq_full), training=False)
    for t in cfg.tasks:
        a = got[t].double().cpu().numpy()
        np.testing.assert_allclose(a, full[t].double().cpu().numpy(), atol=2e-6, rtol=0)
        np.testing.assert_allclose(a, ref['probs'][t].numpy(), atol=5e-5, rtol=0)


def test_cache_reuse_across_calls(dev):
    """One stage-I cache scores several candidate batches (stage II only) with identical results."""
    cfg = small_criteo('tail', pyramid=True, layers=3)
    P = init_params(cfg, cfg.ns_input_width(), seed=0, perturb=True)
    model = OneTransModel(cfg, device=dev, init=P)
    _, seq_r, _ = make_batch(3, cfg, seed=5)
    ns_c, _, _ = make_batch(12, cfg, seed=6)
    srv = OneTransServer(model)
    cache = srv.encode_requests(ns_t(seq_r, dev))
    req = torch.tensor([0, 1, 2] * 4)
    a = srv.score(cache, req, ns_t(ns_c, dev))
    b = srv.score(cache, req[:6], ns_t({k: v[:6] for k, v in ns_c.items()}, dev))
    for t in cfg.tasks:
        torch.testing.assert_close(a[t][:6], b[t], rtol=0, atol=0)


def test_norm_select_refused(dev):
    cfg = small_criteo('tail', pyramid=True, layers=3)
    cfg.pyramid_select = 'norm'
    model = OneTransModel(cfg, device=dev, init=init_params(cfg, cfg.ns_input_width(), seed=0))
    with pytest.raises(ValueError):
        OneTransServer(model)
