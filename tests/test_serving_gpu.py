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
    check_serving(CASES[case](), 5, 23, dev)


@pytest.mark.parametrize('Rq,C', [(1, 1), (2, 129)])
def test_serving_edge_sizes(dev, Rq, C):
    """One request with one candidate; two requests sharing a ragged 129-candidate batch."""
    check_serving(CASES['criteo_tail_pyramid'](), Rq, C, dev)


def check_serving(cfg, Rq, C, dev):
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


def test_bad_request_index_refused(dev):
    """A request index outside [0, R) is refused on the host before the cached-attention launch."""
    cfg = small_criteo('tail', pyramid=True, layers=3)
    model = OneTransModel(cfg, device=dev, init=init_params(cfg, cfg.ns_input_width(), seed=0))
    _, seq_r, _ = make_batch(3, cfg, seed=5)
    ns_c, _, _ = make_batch(4, cfg, seed=6)
    srv = OneTransServer(model)
    cache = srv.encode_requests(ns_t(seq_r, dev))
    for bad in ([0, 1, 2, 3], [0, -1, 1, 2]):
        with pytest.raises(ValueError):
            srv.score(cache, torch.tensor(bad), ns_t(ns_c, dev))
        with pytest.raises(ValueError):
            srv.score(cache, torch.tensor(bad, device=dev), ns_t(ns_c, dev))


def test_norm_select_refused(dev):
    cfg = small_criteo('tail', pyramid=True, layers=3)
    cfg.pyramid_select = 'norm'
    model = OneTransModel(cfg, device=dev, init=init_params(cfg, cfg.ns_input_width(), seed=0))
    with pytest.raises(ValueError):
        OneTransServer(model)


@pytest.mark.parametrize('dedicated', ['head', 'tail'])
def test_extend_requests_matches_reencode(dev, dedicated):
    """Cross-request reuse: appending events to the last sequence computes only the new tokens and
    gives the cache a full re-encode would (scores equal, and equal to the full forward)."""
    cfg = small_criteo(dedicated)
    P = init_params(cfg, cfg.ns_input_width(), seed=0, perturb=True)
    model = OneTransModel(cfg, device=dev, init=P)
    Rq, C, dL = 3, 9, 4
    _, seq_r, _ = make_batch(Rq, cfg, seed=41)
    ns_c, _, _ = make_batch(C, cfg, seed=42)
    last = cfg.feature_config['sequence_features'][-1]
    new = np.random.default_rng(5).integers(0, cfg.seq_item_vocab, (Rq, dL))
    full = dict(seq_r)
    full[last] = np.concatenate([seq_r[last], new], 1)
    req = torch.tensor([0, 1, 2, 2, 1, 0, 0, 1, 2])
    srv = OneTransServer(model)
    ext = srv.extend_requests(srv.encode_requests(ns_t(seq_r, dev)), last, torch.from_numpy(new).to(dev))
    ref_cache = srv.encode_requests(ns_t(full, dev))
    assert ext.L_S == ref_cache.L_S
    a = srv.score(ext, req, ns_t(ns_c, dev))
    b = srv.score(ref_cache, req, ns_t(ns_c, dev))
    with torch.no_grad():
        f = model((ns_t(ns_c, dev), ns_t(expand(full, req.numpy()), dev)), training=False)
    for t in cfg.tasks:
        np.testing.assert_allclose(a[t].cpu().numpy(), b[t].cpu().numpy(), atol=2e-6, rtol=0)
        np.testing.assert_allclose(a[t].cpu().numpy(), f[t].cpu().numpy(), atol=2e-6, rtol=0)
    with pytest.raises(ValueError):                      # an earlier sequence would shift later positions
        srv.extend_requests(ext, cfg.feature_config['sequence_features'][0], torch.from_numpy(new).to(dev))


def test_extend_refused_under_pyramid(dev):
    cfg = small_criteo('tail', pyramid=True, layers=3)
    model = OneTransModel(cfg, device=dev, init=init_params(cfg, cfg.ns_input_width(), seed=0))
    _, seq_r, _ = make_batch(2, cfg, seed=3)
    srv = OneTransServer(model)
    cache = srv.encode_requests(ns_t(seq_r, dev))
    last = cfg.feature_config['sequence_features'][-1]
    with pytest.raises(ValueError):
        srv.extend_requests(cache, last, torch.zeros(2, 3, dtype=torch.int64, device=dev))


def test_inference_engine(dev, tmp_path):
    """The reference engine surface (examples/inference_example.py): a saved model directory, single and
    batch inference, and the two-stage score_candidates path agreeing with them."""
    from recommend_amd.serving import OneTransInferenceEngine
    from recommend_amd.trainer import OneTransTrainer
    cfg = small_criteo('head')
    cfg.max_seq_len = 12
    P = init_params(cfg, cfg.ns_input_width(), seed=0, perturb=True)
    tr = OneTransTrainer(cfg, model_dir=str(tmp_path), model=OneTransModel(cfg, device=dev, init=P))
    tr.save_model('m')
    eng = OneTransInferenceEngine(str(tmp_path / 'm'), device=dev)
    ns_c, seq, _ = make_batch(4, cfg, seed=9)
    names = list(ns_c)
    user = {k: ns_c[k][0] for k in names[:5]}
    cands = [{k: ns_c[k][i] for k in names[5:]} for i in range(4)]
    seq1 = {k: v[0] for k, v in seq.items()}                      # one user's sequences (unpadded)
    batch = [(user, c, {}, seq1) for c in cands]
    got = eng.batch_inference(batch)
    single = eng.single_inference(user, cands[2], {}, seq1)
    fast = eng.score_candidates(user, seq1, cands)
    for t in cfg.tasks:
        assert abs(single[t] - got[2][t]) < 2e-6
        for i in range(4):
            assert abs(fast[i][t] - got[i][t]) < 2e-6
    st = eng.get_stats()
    assert st['total_requests'] == 5 and st['success_rate'] == 100.0
    with pytest.raises(FileNotFoundError):
        OneTransInferenceEngine(str(tmp_path / 'missing'))
