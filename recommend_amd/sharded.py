"""Row-sharded embedding tables for the data-parallel stack.

A table of ``num_rows`` rows is split over the ``world`` ranks of a node: row ``id`` lives on rank
``id % world`` at local row ``id // world`` (the modulo spreads Zipf-hot ids over every GPU).  The
transformer stays data-parallel; only the table is partitioned:

* lookup:   route the batch's distinct ids by owner (``ot_shard_route_unique``: one sort by (owner,
  local row) merges repeats — Zipf batches repeat hot ids, ~3x at the C2/C4 shapes) -> RCCL
  all-to-all of the counts and of the local row indices -> each owner gathers its rows
  (``ot_gather_rows``) -> all-to-all of the rows back -> expanded to the batch's tokens through the
  inverse map (``ot_gather_rows`` again).  ``dedup=False`` (``ONETRANS_SHARD_DEDUP=0``) routes every
  id (``ot_shard_route`` + ``ot_permute_rows``).
* update:   the tokens' gradient rows are summed per distinct id (``ot_segment_rows_sum``, fixed
  order) and travel the same routes to their owners (all-to-all), are scaled by 1/world (each
  rank's loss is a mean over its local batch), de-duplicated across ranks, and applied with the
  sparse Keras Adagrad; the per-table ``clip_by_norm`` uses the global norm (an all-reduce of each
  owner's squared norm between ``ot_sparse_prepare`` and ``ot_sparse_finish``).

All bytes move on device; the only host traffic is the ``world`` split sizes the all-to-alls need.  That
one host wait is taken off the main stream: the ids are staged, routed and their per-owner counts
exchanged on the route stream — the model's communication stream (host ids are copied there; device ids
wait only for the event the caller names as their producer, ``ready``), so the host waits for those few
kernels — not for the previous step's backward and optimizer still queued on the main stream — and the GPU
keeps running them while it does (measured at world 1; at world > 1 the counts' all-to-all also queues
behind earlier collectives on RCCL's stream, unmeasured on hardware).  The gather that follows stays on the
main stream (it reads the table the previous step's sparse update wrote).  A fixed-capacity exchange with no
host sizes was considered: the only sound per-peer bound is the batch's id count n, and the rows coming
back would then move world x n x E x 4 bytes — ~20x the distinct rows at C4 / N = 8.
"""

from __future__ import annotations

from typing import Optional

import os

import time

import numpy as np
import torch
import torch.distributed as dist

from . import kernels as K


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class ShardedTable:
    def __init__(self, name: str, num_rows: int, E: int, world: int, rank: int, device, seed: int = 0,
                 full_init: Optional[np.ndarray] = None, lo: float = -0.05, hi: float = 0.05,
                 dedup: Optional[bool] = None, route_stream=None):
        if dedup is None:
            dedup = os.environ.get('ONETRANS_SHARD_DEDUP', '1') != '0'
        self.dedup = bool(dedup)
        self.name, self.num_rows, self.E = name, int(num_rows), int(E)
        self.world, self.rank, self.device = int(world), int(rank), device
        self.local_rows = (self.num_rows - self.rank + self.world - 1) // self.world
        # every rank allocates ceil(num_rows / world) rows (the same shape everywhere, so collectives
        # over the shard such as full_table's all-gather line up); the last row is padding on ranks
        # with fewer rows
        self.rows_alloc = max(1, (self.num_rows + self.world - 1) // self.world)
        self.table = torch.zeros(self.rows_alloc, self.E, device=device)
        if full_init is not None:           # the shard of a given logical table (tests, checkpoints)
            shard = np.asarray(full_init)[self.rank::self.world]
            self.table[:self.local_rows].copy_(torch.as_tensor(shard, dtype=torch.float32))
        else:
            K.hash_uniform_rows(self.table, self.local_rows, self.E, self.rank, self.world, seed, lo, hi)
        self.last_route = None
        self.sent_rows = 0         # ids (rows) the last lookup sent to their owners
        is_cuda = torch.device(device).type == 'cuda'
        # the stream the ids are staged / routed on: the owning model's communication stream (shared with the
        # dense gradient exchange, so a rank drives main + weight-gradient side + comm + RCCL's internal
        # stream = GPU_MAX_HW_QUEUES 4 hardware queues), or a stream of its own when used standalone
        self.route_stream = route_stream if route_stream is not None else (
            torch.cuda.Stream(device=device) if is_cuda else None)
        # split sizes land here (pinned); two buffers, so a look-ahead route (route()) of the next batch can be
        # in flight while this batch's are still being read
        self._counts_host = [torch.empty(2 * self.world, dtype=torch.int32, pin_memory=is_cuda) for _ in range(2)]
        self._counts_i = 0
        self.events = None        # diagnostics: a list collects HIP-event pairs around lookup / update
        self.route_wait_s = 0.0   # diagnostics: host seconds lookup() spent routing before its first gather launch

    def _mark(self):
        if self.events is None:
            return None
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return ev

    # -------------------------------------------------------------- all-to-all helpers
    def _a2a(self, out, inp, out_splits, in_splits):
        if self.world == 1:
            out.copy_(inp)
        elif dist.get_backend() == 'gloo':   # CPU rehearsal of the N>1 path: gloo exchanges host tensors
            o = torch.empty(out.shape, dtype=out.dtype)
            dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits)
            out.copy_(o)
        else:
            dist.all_to_all_single(out, inp, out_splits, in_splits)

    def route(self, ids, ready=None, srcs=None) -> 'PendingRoute':
        """Look-ahead routing: stage ``ids`` and issue their routing (sort by owner, the split-size all-to-all,
        the split sizes' copy to the host) on the route stream now, and return without waiting; ``lookup(ids,
        routed=<the result>)`` later takes the routed ids (its host wait then finds the sizes already there).
        The trainer routes step i + 1's ids during step i (OneTransTrainer.train_step(next_batch=...)), so at
        N > 1 the split-size exchange overlaps step i's backward instead of stalling step i + 1's start."""
        return PendingRoute(self, ids if srcs is None else srcs, *self._issue_route(ids, ready))

    def _route(self, ids, ready):
        """Stage ``ids`` (a tensor or a list concatenated in order; host or device) and route them by owner
        on the route stream; returns (ids on the device, route buffers, send splits, recv splits) after the
        host has waited for that stream alone (the split sizes)."""
        return self._finish_route(*self._issue_route(ids, ready))

    def _issue_route(self, ids, ready):
        dev, rs = self.device, self.route_stream
        parts = list(ids) if isinstance(ids, (list, tuple)) else [ids]
        host = all(t.device.type == 'cpu' for t in parts)
        if rs is not None and not host:
            if ready is None:
                rs.wait_stream(torch.cuda.current_stream(dev))     # producer unknown: after the main stream
            elif ready is not True:
                rs.wait_event(ready)                                # the named producer event only
        ctx = torch.cuda.stream(rs) if rs is not None else _nullctx()
        with ctx:
            if host:
                h = torch.cat([t.reshape(-1).to(torch.int64) for t in parts])
                ids_d = (h.pin_memory() if rs is not None else h).to(dev, non_blocking=True)
            else:
                ids_d = torch.cat([t.reshape(-1).to(dev, torch.int64) for t in parts])
            n = ids_d.numel()
            counts = torch.empty(self.world, dtype=torch.int32, device=dev)
            if self.dedup:
                send_local = torch.empty(max(1, n), dtype=torch.int64, device=dev)
                inv = torch.empty(max(1, n), dtype=torch.int64, device=dev)
                order = torch.empty(max(1, n), dtype=torch.int32, device=dev)
                run_start = torch.empty(n + 1, dtype=torch.int32, device=dev)
                K.shard_route_unique(ids_d, n, self.num_rows, self.world, send_local, inv, order, run_start, counts)
                bufs = (send_local, inv, order, run_start)
            else:
                perm = torch.empty(max(1, n), dtype=torch.int32, device=dev)
                send_local = torch.empty(max(1, n), dtype=torch.int64, device=dev)
                K.shard_route(ids_d, n, self.num_rows, self.world, perm, send_local, counts)
                bufs = (send_local, perm)
            recv_counts = torch.empty_like(counts)
            self._a2a(recv_counts, counts, None, None)
            both = torch.cat([counts, recv_counts])
            host_counts = self._counts_host[self._counts_i]
            self._counts_i ^= 1
            host_counts.copy_(both, non_blocking=rs is not None)
            done = None
            if rs is not None:
                done = torch.cuda.Event()
                done.record(rs)
        return ids_d, bufs, host_counts, done

    def _finish_route(self, ids_d, bufs, host_counts, done):
        if done is not None:
            done.synchronize()                       # the one host wait: this stream's few kernels only
            main = torch.cuda.current_stream(self.device)
            main.wait_stream(self.route_stream)
            for t in (ids_d, *bufs):                 # allocated on the route stream, used on the main one
                t.record_stream(main)
        both = host_counts.tolist()
        return ids_d, bufs, both[:self.world], both[self.world:]

    def lookup(self, ids, ready=None, routed: 'PendingRoute' = None, srcs=None) -> torch.Tensor:
        """Rows of ``ids`` (int64 [n], or a list of id tensors taken in order; host or device) -> [n, E] fp32
        (zeros for ids outside the table); the staged device ids are kept in ``last_ids``.  ``ready``:
        for device ids, the HIP event after which they are valid (True: already complete, e.g. resident
        batches; None: wait for the current stream).  ``routed``: these ids' look-ahead ``route()``, made from
        ``srcs`` (the caller's id objects, when ``ids`` are tensors made from them; default ``ids``)."""
        ev0 = self._mark()
        E, dev = self.E, self.device
        t0 = time.perf_counter()
        if routed is not None:
            if not routed.matches(self, ids if srcs is None else srcs):
                raise ValueError(f'{self.name}: lookup with a look-ahead route of other ids')
            ids_d, bufs, send_splits, recv_splits = self._finish_route(*routed.parts)
        else:
            ids_d, bufs, send_splits, recv_splits = self._route(ids, ready)
        self.route_wait_s += time.perf_counter() - t0
        n = ids_d.numel()
        S = sum(send_splits)                  # ids this rank sends: distinct ids (dedup) or n
        R = sum(recv_splits)
        send_local = bufs[0]
        recv_local = torch.empty(max(1, R), dtype=torch.int64, device=dev)
        self._a2a(recv_local[:R], send_local[:S], recv_splits, send_splits)
        rows = torch.empty(max(1, R), E, device=dev)
        K.gather_rows(self.table, E, recv_local, R, rows)
        back = torch.empty(max(1, S), E, device=dev)
        self._a2a(back[:S], rows[:R], send_splits, recv_splits)
        out = torch.empty(n, E, device=dev)
        if self.dedup:
            _, inv, order, run_start = bufs
            K.gather_rows(back, E, inv, n, out)          # token i <- its distinct id's row
            self.last_route = (n, ('dedup', order, run_start, S), send_splits, recv_splits, recv_local, R)
        else:
            perm = bufs[1]
            K.permute_rows(back, perm, n, E, True, out)
            self.last_route = (n, perm, send_splits, recv_splits, recv_local, R)
        self.last_ids = ids_d
        self.sent_rows = S
        if ev0 is not None:
            self.events.append((ev0, self._mark()))
        return out

    def apply_gradient(self, route, grads: torch.Tensor, accum: torch.Tensor, lr: float, eps: float,
                       clip: float) -> None:
        """Sparse Adagrad on the owners for ``grads`` (rows in the order of the ids of the ``lookup``
        that produced ``route`` = its ``last_route``)."""
        if route is None:
            raise RuntimeError(f'{self.name}: apply_gradient without a lookup route')
        n, perm, send_splits, recv_splits, recv_local, R = route
        if grads.shape[0] != n:
            raise ValueError(f'{self.name}: {grads.shape[0]} gradient rows for a route of {n} ids')
        E, dev = self.E, self.device
        ev0 = self._mark()
        if isinstance(perm, tuple):                      # de-duplicated route: sum repeats first
            _, order, run_start, S = perm
            send = torch.empty(max(1, S), E, device=dev)
            K.segment_rows_sum(grads.contiguous(), order, run_start, S, E, send)
        else:
            S = n
            send = torch.empty(max(1, n), E, device=dev)
            K.permute_rows(grads.contiguous(), perm, n, E, False, send)
        recv = torch.empty(max(1, R), E, device=dev)
        self._a2a(recv[:R], send[:S], recv_splits, send_splits)
        if self.world > 1:
            recv.mul_(1.0 / self.world)
        ws = K.sparse_workspace(R, E, dev)
        sumsq = torch.zeros(1, device=dev)
        K.sparse_prepare(E, self.local_rows, recv_local, recv, R, sumsq, ws)
        if self.world > 1:
            if dist.get_backend() == 'gloo':
                h = sumsq.cpu()
                dist.all_reduce(h)
                sumsq.copy_(h)
            else:
                dist.all_reduce(sumsq)
        K.sparse_finish(self.table, accum, E, R, lr, eps, clip, sumsq, ws)
        if ev0 is not None:
            self.events.append((ev0, self._mark()))

    def full_table(self) -> torch.Tensor:
        """Gather the logical table on every rank (tests / checkpoints of small tables)."""
        if self.world == 1:
            return self.table[:self.local_rows].clone()
        gloo = dist.get_backend() == 'gloo'
        src = self.table.cpu() if gloo else self.table
        parts = [torch.empty_like(src) for _ in range(self.world)]
        dist.all_gather(parts, src)
        parts = [q.to(self.device) for q in parts]
        out = torch.empty(self.num_rows, self.E, device=self.device)
        for r in range(self.world):
            lr_ = (self.num_rows - r + self.world - 1) // self.world
            out[r::self.world] = parts[r][:lr_]
        return out


class PendingRoute:
    """A look-ahead route (ShardedTable.route): the staged ids' routing issued on the route stream, not yet
    waited for.  Identified by the id objects it was made from (tensors or host arrays), which it keeps alive:
    ``matches`` requires the very same objects, and for tensors an unchanged version counter, so a loader that
    reuses a buffer's address for new ids (a new tensor) or writes new ids into it through torch is refused.
    (Writes that bypass torch — into a numpy array that was routed — cannot be seen: a loader must not refill a
    batch it has passed as ``next_batch``.)"""

    def __init__(self, table, srcs, *parts):
        self.table = table
        self.srcs = list(srcs) if isinstance(srcs, (list, tuple)) else [srcs]
        self.versions = [t._version if isinstance(t, torch.Tensor) else None for t in self.srcs]
        self.parts = parts

    def matches(self, table, srcs) -> bool:
        srcs = list(srcs) if isinstance(srcs, (list, tuple)) else [srcs]
        return (table is self.table and len(srcs) == len(self.srcs)
                and all(a is b for a, b in zip(srcs, self.srcs))
                and all(v is None or b._version == v for b, v in zip(self.srcs, self.versions)))
