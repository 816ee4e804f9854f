"""Serving throughput: two-stage cached inference (recommend_amd/serving.py) vs one full forward per
(request, candidate) sample (the reference engine's batch_inference, examples/inference_example.py:131).

    python3 tools/serve_bench.py [--config C2] [--requests 64] [--cands 64] [--iters 20]

Prints one JSON line: candidates/s of both paths (HIP-event timed, inputs resident on the GPU), the
stage-I / stage-II split, and the max |prob| difference between the two paths.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from recommend_amd.config import workload_config
from recommend_amd.data import make_batch
from recommend_amd.model import OneTransModel
from recommend_amd.serving import OneTransServer

ap = argparse.ArgumentParser()
ap.add_argument('--config', default='C2')
ap.add_argument('--requests', type=int, default=64)
ap.add_argument('--cands', type=int, default=64, help='candidates per request')
ap.add_argument('--iters', type=int, default=20)
a = ap.parse_args()

dev = torch.device('cuda')
cfg = workload_config(a.config)
model = OneTransModel(cfg, device=dev, seed=0)
Rq, C = a.requests, a.requests * a.cands
ns_r, seq_r, _ = make_batch(Rq, cfg, seed=11)
ns_c, _, _ = make_batch(C, cfg, seed=12)
req = np.repeat(np.arange(Rq), a.cands)
to = lambda d: {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in d.items()}
seq_r_d, ns_c_d = to(seq_r), to(ns_c)
seq_full_d = to({k: v[req] for k, v in seq_r.items()})
req_d = torch.from_numpy(req.astype(np.int32)).to(dev)
srv = OneTransServer(model)


def timed(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        out = fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / a.iters, out


with torch.no_grad():
    t_full, p_full = timed(lambda: model((ns_c_d, seq_full_d), training=False))
    t_cached, p_cached = timed(lambda: srv.score(srv.encode_requests(seq_r_d), req_d, ns_c_d))
    t_s1, cache = timed(lambda: srv.encode_requests(seq_r_d))
    t_s2, _ = timed(lambda: srv.score(cache, req_d, ns_c_d))
diff = max(float((p_full[t] - p_cached[t]).abs().max()) for t in cfg.tasks)
print(json.dumps({
    'config': a.config, 'requests': Rq, 'candidates': C, 'L_S': cache.L_S, 'L_NS': cfg.num_ns_tokens,
    'full_forward': {'ms': round(t_full, 3), 'candidates_per_s': round(C / t_full * 1e3, 1)},
    'cached': {'ms': round(t_cached, 3), 'candidates_per_s': round(C / t_cached * 1e3, 1),
               'stage1_ms': round(t_s1, 3), 'stage2_ms': round(t_s2, 3)},
    'speedup': round(t_full / t_cached, 2), 'max_abs_prob_diff': diff}))
