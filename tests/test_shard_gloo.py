"""CPU, world_size 4 over gloo: the host logic of the row-sharded table (recommend_amd/sharded.py) —
split sizes, the all-to-all exchanges, the route back, the global-norm clip — with peers that send
no ids and peers that own none of the ids in flight.

The device kernels the class calls (ot_shard_route[_unique], ot_gather_rows, ot_permute_rows,
ot_segment_rows_sum, ot_sparse_prepare/finish; their GPU parity is tests/test_sharded_gpu.py) are replaced here by small
torch stand-ins that follow their header contracts (include/onetrans_hip.h), so only the exchange
plumbing is under test."""

import os
import socket
import types

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


def _cpu_kernels():
    """Header-contract stand-ins of the shard kernels (CPU tensors)."""
    K = types.SimpleNamespace()

    def shard_route(ids, n, num_rows, world, perm, send_local, counts):
        ids = ids[:n]
        ok = (ids >= 0) & (ids < num_rows)
        owner = torch.where(ok, ids % world, torch.zeros_like(ids))     # invalid ids: owner 0
        order = torch.sort(owner, stable=True).indices
        perm[:n] = order.to(torch.int32)
        loc = torch.where(ok, ids // world, torch.full_like(ids, -1))
        send_local[:n] = loc[order]
        counts.copy_(torch.bincount(owner, minlength=world).to(torch.int32))

    def shard_route_unique(ids, n, num_rows, world, uniq_local, inv, order, run_start, counts):
        ids = ids[:n]
        ok = (ids >= 0) & (ids < num_rows)
        owner = torch.where(ok, ids % world, torch.zeros_like(ids))
        loc1 = torch.where(ok, ids // world + 1, torch.zeros_like(ids))     # invalid: (owner 0, 0)
        key = owner * (1 << 40) + loc1
        srt = torch.sort(key, stable=True)
        order[:n] = srt.indices.to(torch.int32)
        uk, u_of_sorted = torch.unique_consecutive(srt.values, return_inverse=True)
        U = len(uk)
        inv[srt.indices] = u_of_sorted
        uniq_local[:U] = (uk % (1 << 40)) - 1
        heads = torch.ones(n, dtype=torch.bool)
        heads[1:] = srt.values[1:] != srt.values[:-1]
        run_start[:U] = torch.nonzero(heads).reshape(-1).to(torch.int32)
        run_start[U] = n
        counts.copy_(torch.bincount(uk // (1 << 40), minlength=world).to(torch.int32))

    def segment_rows_sum(src, order, run_start, U, E, out):
        for u in range(U):
            acc = torch.zeros(E)
            for j in range(int(run_start[u]), int(run_start[u + 1])):
                acc += src[int(order[j])]
            out[u] = acc

    def gather_rows(table, E, idx, n, out):
        idx = idx[:n]
        out[:n] = torch.where((idx >= 0)[:, None], table[idx.clamp(min=0)], torch.zeros(1, E))

    def permute_rows(src, perm, n, E, inverse, dst):
        p = perm[:n].long()
        if inverse:
            dst[p] = src[:n]
        else:
            dst[:n] = src[p]

    def sparse_workspace(n, E, device):
        return {}

    def sparse_prepare(E, num_rows, keys, grads, n, sumsq_out, ws):
        keys, grads = keys[:n], grads[:n].double()
        ok = keys >= 0
        uk, inv = torch.unique(keys[ok], return_inverse=True)
        g = torch.zeros(len(uk), E, dtype=torch.float64).index_add_(0, inv, grads[ok])
        ws['keys'], ws['g'] = uk, g
        sumsq_out.fill_(float((g * g).sum()))

    def sparse_finish(table, accum, E, n, lr, eps, clip, sumsq_total, ws):
        uk, g = ws['keys'], ws['g']
        l2 = float(sumsq_total.sqrt())
        g = g * clip / max(l2, clip)
        a = accum[uk].double() + g * g
        accum[uk] = a.float()
        table[uk] = (table[uk].double() - lr * g / torch.sqrt(a + eps)).float()

    K.shard_route, K.gather_rows, K.permute_rows = shard_route, gather_rows, permute_rows
    K.shard_route_unique, K.segment_rows_sum = shard_route_unique, segment_rows_sum
    K.sparse_workspace, K.sparse_prepare, K.sparse_finish = sparse_workspace, sparse_prepare, sparse_finish
    return K


def _ids_of(rank, num_rows, world, rng):
    if rank == 2:
        return np.zeros(0, np.int64)                          # a peer that sends no ids
    # no id is owned by rank 3 (id % 4 != 3): a peer that receives no ids; repeats and invalid ids
    ids = rng.integers(0, num_rows, 40)
    ids = ids[ids % world != 3]
    return np.concatenate([ids, ids[:5], [-1, num_rows + 2]]).astype(np.int64)


def _worker(rank, world, port, q, dedup, lookahead=False):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from recommend_amd import sharded
        sharded.K = _cpu_kernels()
        num_rows, E = 203, 8
        rng = np.random.default_rng(11)
        full = rng.uniform(-0.05, 0.05, (num_rows, E)).astype(np.float32)
        st = sharded.ShardedTable('t', num_rows, E, world, rank, torch.device('cpu'), full_init=full, dedup=dedup)
        ids_all = [_ids_of(r, num_rows, world, np.random.default_rng(100 + r)) for r in range(world)]
        grads_all = [np.random.default_rng(200 + r).standard_normal((len(i), E)).astype(np.float32)
                     for r, i in enumerate(ids_all)]
        got = st.lookup(torch.from_numpy(ids_all[rank])).numpy()
        ids = ids_all[rank]
        ok = (ids >= 0) & (ids < num_rows)
        exp = np.where(ok[:, None], full[np.clip(ids, 0, num_rows - 1)], 0.0)
        err_lookup = float(np.abs(got - exp).max()) if len(ids) else 0.0
        route = st.last_route
        recv = route[5]
        acc = torch.full((st.table.shape[0], E), 0.1)
        lr, eps, clip = 0.05, 1e-7, 1.5
        nxt = None
        if lookahead:            # the next batch's ids routed before this step's update (trainer.route_ahead)
            ids2 = torch.from_numpy(_ids_of(rank, num_rows, world, np.random.default_rng(300 + rank)))
            nxt = st.route(ids2)
        st.apply_gradient(route, torch.from_numpy(grads_all[rank]), acc, lr, eps, clip)
        new = st.full_table().numpy()
        err_next = 0.0
        if lookahead:            # ... looked up after the update: the updated rows, through the look-ahead route
            got2 = st.lookup(ids2, routed=nxt).numpy()
            i2 = ids2.numpy()
            ok2 = (i2 >= 0) & (i2 < num_rows)
            exp2 = np.where(ok2[:, None], new[np.clip(i2, 0, num_rows - 1)], 0.0)
            err_next = float(np.abs(got2 - exp2).max()) if len(i2) else 0.0
        g = np.zeros((num_rows, E), np.float64)
        for i, gr in zip(ids_all, grads_all):
            v = (i >= 0) & (i < num_rows)
            np.add.at(g, i[v], gr[v].astype(np.float64) / world)
        l2 = np.sqrt((g * g).sum())
        g = g * clip / max(l2, clip)
        ref = full - lr * g / np.sqrt(0.1 + g * g + eps)
        distinct = len(np.unique(np.where(ok, ids, -1))) if len(ids) else 0
        q.put((rank, len(ids), recv, max(err_lookup, err_next), float(np.abs(new - ref).max()), st.sent_rows if not
               lookahead else distinct if dedup else len(ids), distinct))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('dedup,lookahead', [(True, False), (False, False), (True, True)])
def test_sharded_exchange_world4_with_empty_peers(dedup, lookahead):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    world = 4
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, dedup, lookahead)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    for p in procs:
        if p.exitcode is None:
            p.kill()
        assert p.exitcode == 0, p.exitcode
    out = [q.get(timeout=10) for _ in range(world)]
    res = {r: (n, recv, el, ea) for (r, n, recv, el, ea, _, _) in out}
    for (r, n, _, _, _, sent, distinct) in out:       # dedup: each distinct id (invalid ids: one) sent once
        assert sent == (distinct if dedup else n), (r, sent, distinct, n)
    assert res[2][0] == 0                         # rank 2 sent nothing
    assert res[3][1] == 0                         # rank 3 received nothing
    for r, (n, recv, el, ea) in res.items():
        assert el == 0.0, (r, el)
        assert ea < 1e-6, (r, ea)


def test_pending_route_identity():
    """A look-ahead route matches only the very id objects it was made from, unchanged: not a copy,
    not a tensor written in place since, not another table."""
    from recommend_amd.sharded import PendingRoute
    table = object()
    ids = torch.arange(10)
    pr = PendingRoute(table, [ids], None)
    assert pr.matches(table, [ids]) and pr.matches(table, ids)
    assert not pr.matches(table, [ids.clone()])
    assert not pr.matches(object(), [ids])
    assert not pr.matches(table, [ids, ids])
    ids.add_(1)                                   # same address, new contents
    assert not pr.matches(table, [ids])
    arr = np.arange(5)
    pr2 = PendingRoute(table, [arr], None)
    assert pr2.matches(table, [arr]) and not pr2.matches(table, [arr.copy()])
