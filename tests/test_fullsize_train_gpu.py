"""One full training step at BASELINE size through the HIP path vs the oracle's golden step.

C2 = the headline configuration (B=4096, 4L d128, L0=140, 32.4M x 16 + 1M x 64 tables), C3 = the
pyramid stress configuration (B=2048, 6L d256, L0=524, keep 0.5 per layer: 524 -> 262 -> 131 -> ...)
and C4's shape (B=2048, 8L d256, the 100M-row x 64 item table): the exact kernels, row maps, wgrad
chunk tables and XCD tile remaps the bench runs.  C4 runs twice: replicated on one GPU, and AS STATED
in BASELINE configs[3] — the item table row-sharded (id % world) over 2 data-parallel ranks, each on
half of the batch, the lookup and the sparse update over all-to-alls (both ranks on the box's one GPU,
collectives over gloo: RCCL refuses two ranks per device; the exchange code is the one RCCL runs).
The golden values come from tests/golden/make_fullsize_golden.py (float64 oracle on the host cores of
the build container, the batch in slices, only the touched table rows — see tests/fullsize_common.py);
nothing here reads the reference.

Compared (tolerances as the small-shape parity tests, tests/test_model_gpu.py):
* probabilities of all B samples (training mode, dropout on): |dp| < 1e-4 (a logit error of at most
  ~4e-4, inside north_star's 1e-3); loss: |dL| < 1e-4;
* every dense gradient bank on a fixed sample of entries: max error / max|g| of the bank < 2e-4, and
  the bank's L2 norm within 2e-4 relative;
* each table's de-duplicated gradient: touched-row count exact, L2 norm within 2e-4 relative, a
  fixed sample of rows within 2e-4 of the table's max |g|;
* the update (clip + RMSprop(momentum) dense, clipped Adagrad sparse) on the same samples: the
  parameter change within 2e-4 of the bank's largest change, plus for dense banks the first RMSprop
  step's slope at that element times the gradient band (2e-4 max|g|)."""

import os
import socket

import numpy as np
import pytest
import torch

from conftest import release_device_cache

pytestmark = pytest.mark.gpu

from fullsize_common import BATCH_SEED, MODEL_SEED, TABLE_SEED, dropout_seed, fill_table_device, setup_config, \
    table_values_np
from recommend_amd.data import make_batch
from recommend_amd.model import OneTransModel, keras_bce_loss
from recommend_amd.params import init_params
from recommend_amd.trainer import OneTransTrainer, stack_labels

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')
TOL = 2e-4


def _rel(a, b, scale):
    return float(np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64)).max() / max(scale, 1e-30))


def bank_summary(G, model, gbuf, k, f_ns):
    """(sampled gradient entries, gradient L2 norm, sampled parameter entries) of dense bank k, the
    samples at the golden's indices (gbuf: the gradient buffer, mean over the global batch)."""
    idx = G[f'g_idx.{k}']
    g, w = _flat_view(model, gbuf, k, f_ns), _flat_view(model, model.flat.data, k, f_ns)
    return g[idx], float(np.sqrt((g * g).sum())), w[idx]


def dense_errors(G, P, cfg, summary_of, errs):
    """Sampled gradient / updated-parameter entries of every dense bank vs the golden
    (``summary_of(k)`` = bank_summary's triple)."""
    lr, eps, rho = cfg.optimizer_config['dense_lr'], cfg.rmsprop_epsilon, cfg.rmsprop_rho
    for k in P:
        gi_got, gnorm, wi_got = summary_of(k)
        idx = G[f'g_idx.{k}']
        errs[f'g.{k}'] = _rel(gi_got, G[f'g.{k}'], float(G[f'g_max.{k}']))
        errs[f'gnorm.{k}'] = abs(gnorm / float(G[f'g_norm.{k}']) - 1.0) if G[f'g_norm.{k}'] > 0 else 0.0
        w0 = np.asarray(P[k]).reshape(-1)[idx]
        d_ref = G[f'w1.{k}'] - w0
        # the first RMSprop step u(g) = lr g / sqrt((1 - rho) g^2 + eps) has slope
        # lr eps / ((1 - rho) g^2 + eps)^1.5 (up to lr / sqrt(eps) at g ~ 0): a gradient inside its TOL
        # band moves element i's update by up to slope(g_i) * TOL * max|g|, on top of TOL * max|du|
        gi = G[f'g.{k}']
        slope = lr * eps / ((1 - rho) * gi * gi + eps) ** 1.5
        band = TOL * np.abs(d_ref).max() + slope * TOL * float(G[f'g_max.{k}'])
        errs[f'w.{k}'] = TOL * float((np.abs(wi_got - w0 - d_ref) / band).max())


def table_errors(G, k, u, gs, rows_after, E, errs):
    """Table k: ``u`` sorted distinct touched rows (global ids), ``gs`` [U, E] their de-duplicated
    gradient (mean over the global batch), ``rows_after`` the table rows G['t_rows.k'] after the step."""
    nz = np.abs(gs).sum(1) > 0
    assert int(nz.sum()) == int(G[f't_count.{k}']), (k, int(nz.sum()), int(G[f't_count.{k}']))
    errs[f'tnorm.{k}'] = abs(float(np.sqrt((gs * gs).sum())) / float(G[f't_norm.{k}']) - 1.0)
    rows = G[f't_rows.{k}']
    pos = np.searchsorted(u, rows)
    assert np.array_equal(u[pos], rows), k
    errs[f'tg.{k}'] = _rel(gs[pos], G[f't_g.{k}'], float(G[f't_max.{k}']))
    w0 = table_values_np(rows, E, TABLE_SEED[k]).astype(np.float64)
    d_ref = G[f't_w1.{k}'] - w0
    errs[f'tw.{k}'] = _rel(np.asarray(rows_after, np.float64) - w0, d_ref, np.abs(d_ref).max())


def dedup_rows(keys: torch.Tensor, grads: torch.Tensor):
    """(sorted distinct keys, summed float64 gradient rows) as host numpy."""
    u, inv = torch.unique(keys, return_inverse=True)
    gs = torch.zeros(u.numel(), grads.shape[1], dtype=torch.float64, device=grads.device).index_add_(0, inv,
                                                                                                    grads.double())
    return u.cpu().numpy(), gs.cpu().numpy()


def check(name, errs):
    print(f'{name}: worst ' + ', '.join(f'{k} {v:.1e}' for k, v in sorted(errs.items(), key=lambda kv: -kv[1])[:6]))
    assert errs['probs'] < 1e-4, errs['probs']
    assert errs['loss'] < 1e-4, errs['loss']
    bad = {k: v for k, v in errs.items() if k not in ('probs', 'loss') and v >= TOL}
    assert not bad, bad


def _flat_view(model, buf, k, f_ns):
    v = model.layout.view(buf, k)
    if k == 'tok.ns.kernel':
        v = v[:f_ns]
    return v.reshape(-1).double().cpu().numpy()


@pytest.mark.parametrize('name', ['C2', 'C3', 'C4'])
def test_fullsize_train_step(dev, name):
    path = os.path.join(GOLDEN, f'fullsize_{name}.npz')
    if not os.path.exists(path):
        pytest.skip(f'{path} not generated')
    G = np.load(path)
    cfg = setup_config(name)
    B = cfg._batch
    assert int(G['B']) == B
    f_ns = cfg.ns_input_width()
    P = init_params(cfg, f_ns, seed=MODEL_SEED, perturb=True, with_tables=False)
    model = OneTransModel(cfg, device=dev, seed=MODEL_SEED, init=P)
    for k, t in model.tables.items():
        fill_table_device(t, TABLE_SEED[k])
    tr = OneTransTrainer(cfg, model=model)
    ns, seq, lab = make_batch(B, cfg, seed=BATCH_SEED)
    tdev = lambda d: {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in d.items()}
    y = stack_labels(lab, cfg.tasks, dev)
    model.train()
    probs = model.forward_probs(tdev(ns), tdev(seq), training=True)
    assert dropout_seed() == int(G['seed'])
    loss = keras_bce_loss(y, probs, cfg.tasks)
    tr.optimizer.begin_backward()
    loss.backward()
    gflat = model.flat.grad.clone()
    sparse = [(k, dedup_rows(keys, g)) for (k, keys, g) in model._pending_sparse]
    tr.optimizer.step()
    torch.cuda.synchronize()

    errs = {'probs': float(np.abs(probs.detach().double().cpu().numpy() - G['probs']).max()),
            'loss': abs(float(loss.detach()) - float(G['loss']))}
    dense_errors(G, P, cfg, lambda k: bank_summary(G, model, gflat, k, f_ns), errs)
    for (k, (u, gs)) in sparse:
        rows = torch.from_numpy(G[f't_rows.{k}']).to(dev)
        table_errors(G, k, u, gs, model.tables[k][rows].double().cpu().numpy(), model.tables[k].shape[1], errs)
    assert {k for (k, _) in sparse} == {k[len('t_count.'):] for k in G.files if k.startswith('t_count.')}
    check(name, errs)


# ------------------------------------------------------------------ C4 as stated: row-sharded, 2 ranks
def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _sharded_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    os.environ['ONETRANS_TABLE_SHARDING'] = 'row'
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        dev = torch.device('cuda:0')
        G = np.load(os.path.join(GOLDEN, 'fullsize_C4.npz'))
        cfg = setup_config('C4')
        B = cfg._batch
        Bl = B // world
        sl = slice(rank * Bl, (rank + 1) * Bl)
        f_ns = cfg.ns_input_width()
        P = init_params(cfg, f_ns, seed=MODEL_SEED, perturb=True, with_tables=False)
        model = OneTransModel(cfg, device=dev, seed=MODEL_SEED, init=P)
        st = model.sharded['emb.seq_item']
        assert st.world == world and st.num_rows == cfg.seq_item_vocab
        fill_table_device(model.tables['emb.ns'], TABLE_SEED['emb.ns'])
        fill_table_device(st.table, TABLE_SEED['emb.seq_item'], row0=rank, row_stride=world, nrows=st.local_rows)
        tr = OneTransTrainer(cfg, model=model)
        ns, seq, lab = make_batch(B, cfg, seed=BATCH_SEED)
        part = lambda d: {k: torch.from_numpy(np.ascontiguousarray(v[sl])).to(dev) for k, v in d.items()}
        y = stack_labels({k: v[sl] for k, v in lab.items()}, cfg.tasks, dev)
        assert model.batch_offset(Bl) == rank * Bl       # dropout masks of the global batch's samples
        model.train()
        probs = model.forward_probs(part(ns), part(seq), training=True)
        loss = keras_bce_loss(y, probs, cfg.tasks)
        tr.optimizer.begin_backward()
        loss.backward()
        plan = next(iter(model._plans.values()))
        sparse = {}
        for (k, keys, g) in model._pending_sparse:
            ids = plan['seq_ids'] if k in model.sharded else keys   # a sharded table's keys are its route
            sparse[k] = dedup_rows(ids, g)
        tr.optimizer.step()
        torch.cuda.synchronize()
        res = {'probs': probs.detach().double().cpu().numpy(), 'loss': float(loss.detach()), 'sparse': sparse}
        if rank == 0:
            res['banks'] = {k: bank_summary(G, model, model.flat.grad, k, f_ns) for k in P}
            rows = torch.from_numpy(G['t_rows.emb.ns']).to(dev)
            res['ns_rows'] = model.tables['emb.ns'][rows].double().cpu().numpy()
        else:
            # replicas agree: the data-parallel dense step is identical on every rank
            res['param_digest'] = float(model.flat.data.double().sum())
        r = G['t_rows.emb.seq_item']
        mine = np.nonzero(r % world == rank)[0]
        res['item_rows'] = (mine, st.table[torch.from_numpy(r[mine] // world).to(dev)].double().cpu().numpy())
        res['sent'] = st.sent_rows
        if rank == 0:
            res['param_digest'] = float(model.flat.data.double().sum())
        q.put((rank, res))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_fullsize_train_step_c4_row_sharded():
    """BASELINE configs[3] as stated, on one GPU: the 100M x 64 item table row-sharded over 2 ranks
    (50M rows each), each rank training on its half of the golden batch; the step must equal the
    oracle's single full-batch step (tests/golden/fullsize_C4.npz)."""
    import torch.multiprocessing as mp
    G = np.load(os.path.join(GOLDEN, 'fullsize_C4.npz'))
    cfg = setup_config('C4')
    world = 2
    release_device_cache()             # the ranks' tables need the memory this process's allocator still caches
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    env_pp = os.environ.get('PYTHONPATH', '')
    here = os.path.dirname(os.path.abspath(__file__))
    os.environ['PYTHONPATH'] = os.pathsep.join([here, os.path.dirname(here)] + ([env_pp] if env_pp else []))
    try:
        procs = [ctx.Process(target=_sharded_worker, args=(r, world, port, q)) for r in range(world)]
        for p in procs:
            p.start()
        got = {}
        for _ in range(world):
            r, res = q.get(timeout=600)
            got[r] = res
        for p in procs:
            p.join(120)
    finally:
        os.environ['PYTHONPATH'] = env_pp
    for p in procs:
        if p.exitcode is None:
            p.kill()
        assert p.exitcode == 0, p.exitcode
    f_ns = cfg.ns_input_width()
    P = init_params(cfg, f_ns, seed=MODEL_SEED, perturb=True, with_tables=False)
    errs = {'probs': float(np.abs(np.concatenate([got[r]['probs'] for r in range(world)], 1) - G['probs']).max()),
            'loss': abs(sum(got[r]['loss'] for r in range(world)) / world - float(G['loss']))}
    assert got[0]['param_digest'] == got[1]['param_digest']
    dense_errors(G, P, cfg, lambda k: got[0]['banks'][k], errs)
    for k in ('emb.ns', 'emb.seq_item'):
        # the global de-duplicated gradient: each rank's rows summed, / world (the ranks' losses are
        # means over their local halves)
        us = [got[r]['sparse'][k][0] for r in range(world)]
        u = np.unique(np.concatenate(us))
        gs = np.zeros((len(u), got[0]['sparse'][k][1].shape[1]))
        for r in range(world):
            gs[np.searchsorted(u, us[r])] += got[r]['sparse'][k][1] / world
        if k == 'emb.ns':
            after = got[0]['ns_rows']
        else:
            after = np.zeros((len(G['t_rows.emb.seq_item']), gs.shape[1]))
            for r in range(world):
                idx, vals = got[r]['item_rows']
                after[idx] = vals
        table_errors(G, k, u, gs, after, gs.shape[1], errs)
    print(f'row-sharded C4: ids routed per rank {[got[r]["sent"] for r in range(world)]}')
    check('C4 row-sharded x2', errs)
