"""Row-sharded embedding table (recommend_amd/sharded.py) on the data-parallel path, world_size 2.

Both ranks share the one GPU of the box and talk over gloo (RCCL refuses two ranks on one device;
the exchange code is the same, gloo stages the all-to-alls through host memory).  Checks:
* lookup through route -> all-to-all -> gather -> all-to-all -> unpermute == full_table[ids]
  (zeros for out-of-range ids), and apply_gradient == the oracle's de-duplicated, globally clipped
  Keras Adagrad (oracle/onetrans_ref.py train_step, sparse part) on the full table;
* three training steps of OneTransModel with 'emb.seq_item' row-sharded over 2 ranks (each rank on
  half the batch) == the oracle's full-batch train_step, every parameter and the logical table;
* a checkpoint of the row-sharded model (collective save_weights) loads into a fresh sharded model
  bit-identically, and the loaded model's predictions are identical."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import release_device_cache

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _lookup_update(rank, world, dev):
    from recommend_amd.sharded import ShardedTable
    num_rows, E = 301, 32
    rng = np.random.default_rng(7)
    full = rng.uniform(-0.05, 0.05, (num_rows, E)).astype(np.float32)
    st = ShardedTable('t', num_rows, E, world, rank, dev, full_init=full)
    # ids of each rank: Zipf-ish with repeats, plus out-of-range ids
    ids_all = [np.concatenate([rng.integers(0, num_rows, 200), rng.integers(0, 5, 50), [-1, num_rows, 3]])
               for _ in range(world)]
    grads_all = [rng.standard_normal((len(i), E)).astype(np.float32) * 0.1 for i in ids_all]
    ids = torch.from_numpy(ids_all[rank]).to(dev)
    got = st.lookup(ids).cpu().numpy()
    exp = np.where(((ids_all[rank] >= 0) & (ids_all[rank] < num_rows))[:, None],
                   full[np.clip(ids_all[rank], 0, num_rows - 1)], 0.0)
    err_lookup = float(np.abs(got - exp).max())
    acc = torch.full((st.table.shape[0], E), 0.1, device=dev)
    lr, eps, clip = 0.05, 1e-7, 0.5
    st.apply_gradient(st.last_route, torch.from_numpy(grads_all[rank]).to(dev), acc, lr, eps, clip)
    new = st.full_table().cpu().numpy()
    # expected: dense gradient of mean-over-ranks, invalid ids dropped, clip by global norm, Adagrad
    g = np.zeros((num_rows, E), np.float64)
    for i, gr in zip(ids_all, grads_all):
        ok = (i >= 0) & (i < num_rows)
        np.add.at(g, i[ok], gr[ok].astype(np.float64) / world)
    l2 = np.sqrt((g * g).sum())
    g = g * clip / max(l2, clip)
    a = 0.1 + g * g
    ref = full - lr * g / np.sqrt(a + eps)
    return err_lookup, float(np.abs(new - ref).max())


def _worker(rank, world, port, q, sharding='row'):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    os.environ['ONETRANS_TABLE_SHARDING'] = 'none' if sharding.startswith('none') else 'row'
    # 'row-nodedup': every id routed (no de-duplication before the all-to-all)
    os.environ['ONETRANS_SHARD_DEDUP'] = '0' if sharding == 'row-nodedup' else '1'
    # 'none-compact': the replicated table's gradient exchanged as the union of touched rows only
    os.environ['ONETRANS_COMPACT_EXCHANGE'] = '1' if sharding == 'none-compact' else '0'
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        dev = torch.device('cuda:0')
        res = {}
        res['lookup'], res['adagrad'] = _lookup_update(rank, world, dev)

        from recommend_amd.data import make_batch
        from recommend_amd.model import OneTransModel
        from recommend_amd.params import init_params, keras_variables
        from recommend_amd.trainer import OneTransTrainer
        from oracle import onetrans_ref as R
        from test_model_gpu import small_criteo
        cfg = small_criteo('head', d=64, H=4, f=128, Lns=4, seq_lens=(5, 9, 7))
        cfg.dropout_rate = 0.0
        cfg.optimizer_config = dict(cfg.optimizer_config, dense_lr=0.001, momentum=0.9)
        P = init_params(cfg, cfg.ns_input_width(), seed=0, perturb=True)
        model = OneTransModel(cfg, device=dev, init=P)
        if sharding.startswith('row'):
            assert 'emb.seq_item' in model.sharded
            assert model.sharded['emb.seq_item'].dedup == (sharding == 'row')
            assert model.sharded['emb.seq_item'].local_rows == (cfg.seq_item_vocab - rank + 1) // 2
        else:                                            # replicated: dense-gradient all-reduce exchange
            assert not model.sharded
        tr = OneTransTrainer(cfg, model=model)
        B = 40
        Pt = R.to_torch(P)
        st = R.init_state(Pt, cfg)
        kv = keras_variables(cfg, {k: v.shape for k, v in P.items() if not k.startswith('emb.')})
        losses = []
        sl = slice(rank * B // world, (rank + 1) * B // world)
        part = lambda d: {k: v[sl] for k, v in d.items()}
        batches = [make_batch(B, cfg, seed=3000 + step) for step in range(3)]
        parts = [tuple(part(x) for x in b) for b in batches]
        for step in range(3):
            ns, seq, lab = batches[step]
            # the row-sharded runs route the next step's ids during this step (look-ahead, trainer.route_ahead)
            nxt = parts[step + 1] if step + 1 < 3 and sharding == 'row' else None
            out = tr.train_step(parts[step], next_batch=nxt)
            loss = out['total_loss'].detach().reshape(1).cpu()
            dist.all_reduce(loss)
            losses.append(float(loss) / world)
            Pt, st, rl, _ = R.train_step(Pt, st, cfg, kv, R.to_torch(ns), R.to_torch(seq), R.to_torch(lab), seed=0)
            res[f'loss{step}'] = abs(losses[-1] - float(rl))
        got = model.param_dict()
        res['params'] = {k: float(np.abs(got[k] - v.detach().numpy()).max()) for k, v in Pt.items()}
        if sharding == 'row':
            # checkpoint round trip with the table row-sharded: save_weights is collective (rank 0
            # writes), load_weights fills each rank's shard, and the loaded model predicts the same
            import tempfile
            path = os.path.join(tempfile.gettempdir(), f'ot_shard_ckpt_{os.environ["MASTER_PORT"]}.npz')
            model.save_weights(path)
            dist.barrier()
            fresh = OneTransModel(cfg, device=dev, seed=123)
            fresh.load_weights(path)
            assert fresh.tables['emb.seq_item'] is fresh.sharded['emb.seq_item'].table
            back = fresh.param_dict()
            res['ckpt'] = max(float(np.abs(back[k] - got[k]).max()) for k in got)
            ns, seq, _ = make_batch(B, cfg, seed=4000)
            sl = slice(rank * B // world, (rank + 1) * B // world)
            tdev = lambda d: {k: torch.from_numpy(v[sl]).to(dev) for k, v in d.items()}
            with torch.no_grad():
                a = model.forward_probs(tdev(ns), tdev(seq), training=False)
                b = fresh.forward_probs(tdev(ns), tdev(seq), training=False)
            res['ckpt_fwd'] = float((a - b).abs().max())
            dist.barrier()
            if rank == 0:
                os.remove(path)
        if rank == 0:
            q.put(res)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('sharding', ['row', 'row-nodedup', 'none', 'none-compact'])
def test_row_sharded_table_two_ranks(sharding):
    """'row': the item table row-sharded over the ranks; 'none': replicated, exchanged as a dense
    all-reduced gradient ('none-compact': only the rows some rank touched are all-reduced).  Either way three DP steps equal the oracle's full-batch steps (and the
    dense gradients are all-reduced per block during the backward)."""
    release_device_cache()             # the ranks' tables need the memory this process's allocator still caches
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    env_pp = os.environ.get('PYTHONPATH', '')
    here = os.path.dirname(os.path.abspath(__file__))
    os.environ['PYTHONPATH'] = os.pathsep.join([here, os.path.dirname(here)] + ([env_pp] if env_pp else []))
    try:
        procs = [ctx.Process(target=_worker, args=(r, 2, port, q, sharding)) for r in range(2)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(300)
    finally:
        os.environ['PYTHONPATH'] = env_pp
    for p in procs:
        if p.exitcode is None:
            p.kill()
        assert p.exitcode == 0, p.exitcode
    res = q.get(timeout=10)
    assert res['lookup'] == 0.0
    assert res['adagrad'] < 1e-6, res['adagrad']
    for step in range(3):
        assert res[f'loss{step}'] < 2e-4, (step, res[f'loss{step}'])
    bad = {k: v for k, v in res['params'].items() if v >= 2e-4}
    assert not bad, bad
    if sharding == 'row':
        assert res['ckpt'] == 0.0 and res['ckpt_fwd'] == 0.0, (res['ckpt'], res['ckpt_fwd'])


@pytest.mark.parametrize('world', [1, 3, 8])
@pytest.mark.parametrize("n", [0, 1, 5000, 300000])
def test_shard_route_unique_kernel(world, n):
    """ot_shard_route_unique / ot_segment_rows_sum against numpy: distinct ids in (owner, local row)
    order, every invalid id merged into one entry at owner 0, per-owner counts, the inverse map, and
    the per-distinct-id gradient sums (fixed order: equal to a float64 sum within f32 rounding)."""
    from recommend_amd import kernels as K
    dev = torch.device('cuda:0')
    num_rows, E = 100_003, 16
    rng = np.random.default_rng(n + world)
    ids = ((rng.zipf(1.2, n) - 1) % num_rows).astype(np.int64)
    if n > 2:
        ids[:3] = [-5, num_rows, num_rows + 7]                 # invalid ids
    t = torch.from_numpy(ids).to(dev)
    uniq_local = torch.full((max(1, n),), -99, dtype=torch.int64, device=dev)
    inv = torch.empty(max(1, n), dtype=torch.int64, device=dev)
    order = torch.empty(max(1, n), dtype=torch.int32, device=dev)
    run_start = torch.empty(n + 1, dtype=torch.int32, device=dev)
    counts = torch.full((world,), -1, dtype=torch.int32, device=dev)
    K.shard_route_unique(t, n, num_rows, world, uniq_local, inv, order, run_start, counts)
    ok = (ids >= 0) & (ids < num_rows)
    owner = np.where(ok, ids % world, 0)
    loc = np.where(ok, ids // world, -1)
    keys = sorted(set(zip(owner.tolist(), loc.tolist())))
    U = len(keys)
    c = counts.cpu().numpy()
    assert c.sum() == U
    assert c.tolist() == [sum(1 for o, _ in keys if o == r) for r in range(world)]
    assert uniq_local[:U].cpu().numpy().tolist() == [l for _, l in keys]
    pos = {k: u for u, k in enumerate(keys)}
    assert inv[:n].cpu().numpy().tolist() == [pos[(o, l)] for o, l in zip(owner.tolist(), loc.tolist())]
    rs = run_start.cpu().numpy()
    assert rs[U] == n and (np.diff(rs[:U + 1]) > 0).all()
    grads = rng.standard_normal((n, E)).astype(np.float32)
    out = torch.empty(max(1, U), E, device=dev)
    K.segment_rows_sum(torch.from_numpy(grads).to(dev) if n else torch.zeros(1, E, device=dev), order, run_start,
                       U, E, out)
    exp = np.zeros((U, E))
    mag = np.zeros((U, E))
    inv_np = inv[:n].cpu().numpy()
    np.add.at(exp, inv_np, grads.astype(np.float64))
    np.add.at(mag, inv_np, np.abs(grads).astype(np.float64))
    if U:
        # f32 summation (pieces of 64 positions, then the pieces in order): within 1e-6 of sum |g| per entry
        assert (np.abs(out[:U].cpu().numpy() - exp) <= 1e-5 + 1e-6 * mag).all()
