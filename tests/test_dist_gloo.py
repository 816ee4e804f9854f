"""CPU, world_size 2 over gloo: the data-parallel exchange (recommend_amd.dist) reproduces the
single-process gradient of the full batch (dense all-reduce mean; sparse all-gather / world)."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from recommend_amd import dist as otdist
        from recommend_amd.config import workload_config
        from recommend_amd.data import make_batch
        from recommend_amd.params import init_params
        from oracle import onetrans_ref as R
        cfg = workload_config('C2')
        cfg.hidden_dim, cfg.num_heads, cfg.ffn_dim, cfg.num_layers, cfg.num_ns_tokens = 16, 2, 32, 1, 2
        cfg.sparse_features = {k: 10 for k in cfg.sparse_features}
        cfg.seq_item_vocab = 20
        cfg._seq_lens = [3, 2, 3]
        P = init_params(cfg, cfg.ns_input_width(), seed=0, perturb=True)
        ns, seq, lab = make_batch(8, cfg, seed=5)
        sl = slice(4 * rank, 4 * rank + 4)
        part = lambda d: {k: v[sl] for k, v in d.items()}
        _, g, _ = R.loss_and_grads(R.to_torch(P), cfg, R.to_torch(part(ns)), R.to_torch(part(seq)),
                                   R.to_torch(part(lab)), training=False)
        names = [k for k in g if not k.startswith('emb.')]
        flat = torch.cat([g[k].reshape(-1) for k in names]).float()
        otdist.allreduce_dense(flat, bucket_elems=1000)
        # sparse: rows touched by this rank's batch (keys + gradient rows), exchanged
        gt = g['emb.seq_item']
        keys = torch.nonzero(gt.abs().sum(1) > 0)[:, 0]
        keys = torch.cat([keys, torch.full((64 - keys.numel(),), -1, dtype=torch.long)])
        rows = torch.where((keys >= 0)[:, None], gt[keys.clamp(min=0)], torch.zeros(1, gt.shape[1], dtype=gt.dtype))
        k_all, g_all = otdist.allgather_sparse(keys, rows.float())
        dense = torch.zeros(gt.shape)
        ok = k_all >= 0
        dense.index_add_(0, k_all[ok], g_all[ok].double().float())
        if rank == 0:
            _, gf, _ = R.loss_and_grads(R.to_torch(P), cfg, R.to_torch(ns), R.to_torch(seq), R.to_torch(lab),
                                        training=False)
            ref = torch.cat([gf[k].reshape(-1) for k in names]).float()
            q.put((float((flat - ref).abs().max()), float((dense - gf['emb.seq_item'].float()).abs().max())))
    finally:
        dist.destroy_process_group()


def test_dp_exchange_equals_full_batch():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    dense_err, sparse_err = q.get(timeout=10)
    assert dense_err < 1e-6
    assert sparse_err < 1e-6
