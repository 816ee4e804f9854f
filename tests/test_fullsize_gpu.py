"""Parity at BASELINE.json's full sizes through a size-independent property: samples are independent
in the forward pass (no batch coupling anywhere in model.py), so the logits the HIP path computes for a
few samples of a full-size batch must equal the oracle's logits for those samples alone.  Full model
shapes, full batches, full embedding tables (C4's 100M-row table excepted: 25 GB to copy to the host)."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from recommend_amd.config import workload_config
from recommend_amd.data import make_batch
from recommend_amd.model import OneTransModel
from oracle import onetrans_ref as R

from test_model_gpu import LOGIT_TOL, ns_t


def _sub(d, idx):
    return {k: np.ascontiguousarray(v[idx]) for k, v in d.items()}


@pytest.mark.parametrize('name,nsub', [('C2', 6), ('T', 3), ('C3', 2), ('C5', 1)])
def test_fullsize_rows_match_oracle(dev, name, nsub):
    cfg = workload_config(name)
    B = cfg._batch
    model = OneTransModel(cfg, device=dev, seed=0)
    ns, seq, _ = make_batch(B, cfg, seed=77)
    with torch.no_grad():
        model((ns_t(ns, dev), ns_t(seq, dev)), training=False)
    logits = model._last_logits.double().cpu().numpy()             # [T, B]
    assert np.isfinite(logits).all()
    pick = np.unique(np.concatenate([[0, B - 1], np.random.default_rng(3).choice(B, nsub, replace=False)]))
    P = {k: (torch.from_numpy(v) if k.startswith('emb.') else torch.from_numpy(v).double())
         for k, v in model.param_dict().items()}                    # tables stay f32 (host memory)
    ref = R.forward(P, cfg, R.to_torch(_sub(ns, pick)), R.to_torch(_sub(seq, pick)), training=False)
    for i, t in enumerate(cfg.tasks):
        np.testing.assert_allclose(logits[i, pick], ref['logits'][t].numpy()[:, 0], atol=LOGIT_TOL, rtol=0)
