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

All bytes move on device; the only host traffic is the ``world`` split sizes the all-to-alls need.
"""

from __future__ import annotations

from typing import Optional

import os

import numpy as np
import torch
import torch.distributed as dist

from . import kernels as K


class ShardedTable:
    def __init__(self, name: str, num_rows: int, E: int, world: int, rank: int, device, seed: int = 0,
                 full_init: Optional[np.ndarray] = None, lo: float = -0.05, hi: float = 0.05,
                 dedup: Optional[bool] = None):
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
        self.events = None        # diagnostics: a list collects HIP-event pairs around lookup / update

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

    def _splits(self, counts):
        recv_counts = torch.empty_like(counts)
        self._a2a(recv_counts, counts, None, None)
        both = torch.cat([counts, recv_counts]).cpu().tolist()      # the one host sync: split sizes
        return both[:self.world], both[self.world:]

    def lookup(self, ids: torch.Tensor) -> torch.Tensor:
        """Rows of ``ids`` (int64 [n]) in order -> [n, E] fp32 (zeros for ids outside the table)."""
        ev0 = self._mark()
        ids = ids.reshape(-1).contiguous()
        n, E, dev = ids.numel(), self.E, self.device
        counts = torch.empty(self.world, dtype=torch.int32, device=dev)
        if self.dedup:
            send_local = torch.empty(max(1, n), dtype=torch.int64, device=dev)
            inv = torch.empty(max(1, n), dtype=torch.int64, device=dev)
            order = torch.empty(max(1, n), dtype=torch.int32, device=dev)
            run_start = torch.empty(n + 1, dtype=torch.int32, device=dev)
            K.shard_route_unique(ids, n, self.num_rows, self.world, send_local, inv, order, run_start, counts)
        else:
            perm = torch.empty(max(1, n), dtype=torch.int32, device=dev)
            send_local = torch.empty(max(1, n), dtype=torch.int64, device=dev)
            K.shard_route(ids, n, self.num_rows, self.world, perm, send_local, counts)
        send_splits, recv_splits = self._splits(counts)
        S = sum(send_splits)                  # ids this rank sends: distinct ids (dedup) or n
        R = sum(recv_splits)
        recv_local = torch.empty(max(1, R), dtype=torch.int64, device=dev)
        self._a2a(recv_local[:R], send_local[:S], recv_splits, send_splits)
        rows = torch.empty(max(1, R), E, device=dev)
        K.gather_rows(self.table, E, recv_local, R, rows)
        back = torch.empty(max(1, S), E, device=dev)
        self._a2a(back[:S], rows[:R], send_splits, recv_splits)
        out = torch.empty(n, E, device=dev)
        if self.dedup:
            K.gather_rows(back, E, inv, n, out)          # token i <- its distinct id's row
            self.last_route = (n, ('dedup', order, run_start, S), send_splits, recv_splits, recv_local, R)
        else:
            K.permute_rows(back, perm, n, E, True, out)
            self.last_route = (n, perm, send_splits, recv_splits, recv_local, R)
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
