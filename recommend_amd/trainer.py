"""OneTransTrainer — mirrors the reference trainer (``practice/train.py:19-374``).

``train_step`` is the metric's "fwd+bwd" unit (train.py:111-155): forward (tuple call
convention, train.py:118) -> Σ_task Keras BCE (train.py:124-128) -> backward (train.py:131) ->
per-variable clip_by_norm (train.py:134-135) -> RMSprop(momentum) (train.py:138) -> sparse Adagrad
on the embedding rows touched (build extension).  Defect D5 mapping: the trainer reads
``gradient_clip_norm`` (the reference reads the absent ``gradient_clip``) and
``optimizer_config['dense_lr']`` (the reference reads the absent ``learning_rate``); mixed
precision is not enabled (the reference reads the absent ``system_config``) — the HIP path
computes in fp32 like the Keras default policy.
"""

from __future__ import annotations

import json
import os
import time
from pathlib import Path
from typing import Dict, Optional

import numpy as np
import torch

from . import dist as otdist
from . import kernels as K
from .config import OneTransConfig, get_model_config
from .metrics import auc, keras_auc
from .model import BINARY_TASKS, OneTransModel, keras_bce_loss


def _to_dev(d: Dict, dev) -> Dict[str, torch.Tensor]:
    out = {}
    for k, v in d.items():
        t = v if isinstance(v, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(v))
        out[k] = t.to(dev, non_blocking=True)
    return out


def _seq_inputs(model, seq: Dict, dev) -> Dict:
    """Sequence features for forward_probs: with a row-sharded item table the id sequences stay as the caller
    gave them (host arrays or tensors) — the lookup copies them on the table's route stream, off the main stream
    (sharded.py), and a look-ahead route (route_ahead) is matched against these very objects."""
    if not getattr(model, 'sharded', None):
        return _to_dev(seq, dev)
    return dict(seq)


def label_rank(labels) -> int:
    """Rank of the caller's per-task labels: 1 for [B] (get_tf_dataset's batched scalars), 2 for [B, 1]
    (create_sample_batch) and for an already stacked [T, B] tensor.  It picks the BCE form (keras_bce_loss)."""
    if isinstance(labels, torch.Tensor):
        return 2
    return min(2, max(np.ndim(v) for v in labels.values()))


def stack_labels(labels: Dict, tasks, dev) -> torch.Tensor:
    """{task: [B,1]} -> [T, B] float32 on device."""
    return torch.stack([torch.as_tensor(labels[t]).reshape(-1).to(dev, torch.float32) for t in tasks])


class OneTransOptimizer:
    """Dense: clip_by_norm per reference variable + Keras RMSprop(momentum) on the flat buffer,
    one fused multi-segment launch (ot_clip_rmsprop).  Sparse: Keras Adagrad on the de-duplicated
    rows of each embedding table (ot_sparse_adagrad)."""

    def __init__(self, model: OneTransModel, config: OneTransConfig):
        self.model = model
        oc = config.optimizer_config
        self.lr = float(oc.get('dense_lr', config.learning_rate))
        # linear warm-up of the dense learning rate over config.warmup_steps (config.py:36; the
        # reference defines warmup_steps but never applies it, so this is opt-in: apply_warmup)
        self.warmup = int(config.warmup_steps) if getattr(config, 'apply_warmup', False) else 0
        self.steps_done = 0
        self.momentum = float(oc.get('momentum', 0.0))
        self.rho = float(config.rmsprop_rho)
        self.eps = float(config.rmsprop_epsilon)
        self.clip = float(config.gradient_clip_norm)
        self.sparse_lr = float(oc.get('sparse_lr', 0.1))
        self.sparse_eps = float(config.adagrad_epsilon)
        self.sparse_clip = float(config.sparse_clip_norm)
        dev = model.flat.device
        self.v = torch.zeros_like(model.flat.data)
        self.m = torch.zeros_like(model.flat.data)
        self.segs = torch.from_numpy(model.layout.segments.reshape(-1)).to(dev)
        self.nseg = model.layout.segments.shape[0]
        self.acc = {k: torch.full_like(t, float(config.adagrad_initial_accumulator)) for k, t in model.tables.items()}
        # data-parallel exchange of replicated tables: dense all-reduce up to this size, else all-gather
        self.dense_exchange_bytes = int(float(os.environ.get('ONETRANS_DENSE_EXCHANGE_MB', '512')) * 2 ** 20)
        # ... and of those, all-reduce only the rows some rank touched (the union, from a 1-byte-per-row
        # max all-reduce) when it is under 60% of a >= 128 MB table ('auto'), always ('1') or never ('0')
        self.compact_exchange = os.environ.get('ONETRANS_COMPACT_EXCHANGE', 'auto')
        self._dense_grad: Dict[str, torch.Tensor] = {}
        self._mask_buf: Dict[str, torch.Tensor] = {}
        self._masks: Dict = {}
        self._mask_stream = None
        self._mask_count: Dict[str, torch.Tensor] = {}
        # diagnostics (bench.py, N > 1): when a list, every step appends HIP-event pairs bracketing the
        # main stream's waits for the gradient exchange, i.e. the exchange time NOT hidden by backward
        self.exchange_events = None

    def current_lr(self) -> float:
        """Dense learning rate of the step being applied (``steps_done`` counts it): lr * min(1, step /
        warmup_steps) under ``apply_warmup``, else lr."""
        if self.warmup > 0:
            return self.lr * min(1.0, self.steps_done / self.warmup)
        return self.lr

    def _mark(self):
        if self.exchange_events is None:
            return None
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return ev

    def exposed_exchange_ms(self) -> float:
        """Sum over the recorded steps of the exposed exchange time (ms); clears the record."""
        if not self.exchange_events:
            return 0.0
        torch.cuda.synchronize()
        ms = sum(a.elapsed_time(b) for (a, b) in self.exchange_events)
        self.exchange_events = []
        return ms

    # ---------------------------------------------------------------- DP exchange overlapped with backward
    def bank_ranges(self):
        """Flat-buffer ranges that become final together in backward: 'head' (out_norm + heads), each
        block l, and the tokenizer remainder (layout order: tok.*, blk.0 .. blk.L-1, out_norm, head.*)."""
        lay, cfg = self.model.layout, self.model.config
        off = lay.offsets
        starts = [off[f'blk.{l}.norm1'] for l in range(cfg.num_layers)] + [off['out_norm']]
        r = {l: (starts[l], starts[l + 1]) for l in range(cfg.num_layers)}
        r['head'] = (off['out_norm'], lay.total)
        r['tok'] = (0, starts[0])
        return r

    def begin_backward(self) -> None:
        """Arm the per-bank all-reduce hooks for the next backward (world > 1, no accumulation): each
        block's gradient range is all-reduced on a communication stream as soon as its dgrad chain and
        its side-stream weight gradients are issued, overlapping the earlier layers' backward."""
        m = self.model
        if otdist.world() == 1 or m.accumulate_grads:
            m.grad_ready = None
            return
        if not hasattr(self, '_ranges'):
            self._ranges = self.bank_ranges()
            self._comm = m.comm_stream()
        self._works = []
        m.grad_ready = self._launch

    def _launch(self, key) -> None:
        m = self.model
        lo, hi = self._ranges[key]
        self._comm.wait_stream(torch.cuda.current_stream(m.flat.device))
        if m._side is not None:
            self._comm.wait_stream(m._side)              # this block's wgrads run on the side stream
        with torch.cuda.stream(self._comm):
            for s0 in range(lo, hi, otdist.BUCKET_ELEMS):          # 32 MiB buckets (one for a C2 block)
                self._works.append(otdist.allreduce_sum_async(m.flat.grad[s0:min(hi, s0 + otdist.BUCKET_ELEMS)]))

    def _compact(self, table: torch.Tensor) -> bool:
        """Exchange this replicated table's gradient as the union of touched rows (ONETRANS_COMPACT_EXCHANGE: '1'
        always, 'auto' for tables of >= 128 MB — each compaction costs a mask all-reduce and a host sync)?"""
        return self.compact_exchange == '1' or (self.compact_exchange == 'auto' and table.numel() * 4 >= 2 ** 27)

    def prepare_table_exchange(self) -> None:
        """Between the forward and the backward (OneTransTrainer.train_step): for each replicated table exchanged
        as the union of touched rows, build this rank's touched-row mask from the forward's ids, MAX-all-reduce it
        and count the union, all on a stream of its own that depends on the forward only; the count goes to pinned
        host memory.  step() then waits for that stream's event — long complete by the time the host has issued the
        backward — and takes the union's rows with ``torch.nonzero_static`` (no device sync), so the optimizer
        step has no host gap (the mask used to be built, reduced and ``torch.nonzero``-ed in step(), a sync on the
        whole queued backward)."""
        m = self.model
        self._masks = {}
        if otdist.world() == 1:
            return
        import torch.distributed as dist
        for name, ids in getattr(m, 'last_table_ids', {}).items():
            table = m.tables.get(name)
            if (ids is None or table is None or name in m.sharded or table.numel() * 4 > self.dense_exchange_bytes
                    or not self._compact(table)):
                continue
            rows = table.shape[0]
            mask = self._mask_buf.get(name)
            if mask is None:
                mask = self._mask_buf[name] = torch.zeros(rows, dtype=torch.uint8, device=table.device)
            if self._mask_stream is None:
                self._mask_stream = torch.cuda.Stream(device=table.device)
            cnt = self._mask_count.get(name)
            if cnt is None:
                cnt = self._mask_count[name] = torch.zeros(1, dtype=torch.int64, pin_memory=True)
            ms = self._mask_stream
            ms.wait_stream(torch.cuda.current_stream(table.device))      # the forward staged the ids
            with torch.cuda.stream(ms):
                mask.zero_()
                k = ids.reshape(-1)
                mask[k[(k >= 0) & (k < rows)]] = 1
                work = dist.all_reduce(mask, op=dist.ReduceOp.MAX, async_op=True)
                if dist.get_backend() == 'gloo':
                    # (the CPU rehearsal: gloo's wait blocks the host, so it and the count wait for step())
                    self._masks[name] = (mask, work, None)
                    continue
                work.wait()                              # RCCL: a stream dependency, no host wait
                cnt.copy_(torch.count_nonzero(mask).reshape(1), non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(ms)
            self._masks[name] = (mask, None, ev)

    def _start_table_exchange(self, g: torch.Tensor, keys: torch.Tensor, name: str = None):
        """Start the sum over ranks of a replicated table's dense gradient ``g``.  C2's 1M-row item table
        is 256 MB, but a rank's batch touches ~1/6 of its rows: the ranks first agree on the union of
        touched rows (uint8 mask, max all-reduce, 1 B per row) and all-reduce only those rows
        (``ONETRANS_COMPACT_EXCHANGE``).  Rows outside the union are zero on every rank, so the result
        is the dense all-reduce's.  Returns (g, work, union rows or None, compact rows or None)."""
        import torch.distributed as dist
        rows = g.shape[0]
        if self._compact(g):
            pending = self._masks.pop(name, None) if name is not None else None
            if pending is not None:                      # built from the forward's ids, reduced during the backward
                mask, work, ev = pending
                if work is not None:                     # gloo: wait and count here
                    work.wait()
                    torch.cuda.current_stream(g.device).wait_stream(self._mask_stream)
                    idx = torch.nonzero(mask).reshape(-1)
                else:
                    ev.synchronize()                     # (the mask stream's work, not the queued backward)
                    torch.cuda.current_stream(g.device).wait_event(ev)
                    idx = torch.nonzero_static(mask, size=int(self._mask_count[name].item())).reshape(-1)
            else:
                mask = torch.zeros(rows, dtype=torch.uint8, device=g.device)
                k = keys.reshape(-1)
                mask[k[(k >= 0) & (k < rows)]] = 1
                dist.all_reduce(mask, op=dist.ReduceOp.MAX)
                idx = torch.nonzero(mask).reshape(-1)    # host sync: the union's size
            if self.compact_exchange == '1' or idx.numel() < 0.6 * rows:
                cg = g.index_select(0, idx)
                return g, otdist.allreduce_sum_async(cg), idx, cg
        return g, otdist.allreduce_sum_async(g), None, None

    def step(self) -> None:
        m = self.model
        # replicated tables small enough to exchange densely: scatter the de-duplicated gradient and
        # start its all-reduce first, so the dense optimizer below runs while it is in flight
        early = {}
        ev_a = self._mark() if otdist.world() > 1 else None
        if otdist.world() > 1:
            for (name, keys, grads) in m._pending_sparse:
                table = m.tables[name]
                if name in m.sharded or table.numel() * 4 > self.dense_exchange_bytes:
                    continue
                rows, E = table.shape
                g = self._dense_grad.get(name)
                if g is None:
                    g = self._dense_grad[name] = torch.zeros_like(table)
                else:
                    g.zero_()
                K.sparse_grad_dense(E, rows, keys, grads, keys.numel(), g, device=table.device)
                early[name] = self._start_table_exchange(g, keys, name)
        if m.grad_ready is not None:
            for w in self._works:                        # the current stream waits for each exchange
                w.wait()
            lo, hi = self._ranges['tok']
            otdist.allreduce_dense(m.flat.grad[lo:hi], scale=False)
            m.flat.grad.mul_(1.0 / otdist.world())
            m.grad_ready = None
            self._works = []
        else:
            otdist.allreduce_dense(m.flat.grad)
        if ev_a is not None:
            self.exchange_events.append((ev_a, self._mark()))
        self.steps_done += 1
        K.clip_rmsprop(m.flat.data, m.flat.grad, self.v, self.m, self.segs, self.nseg, m.layout.max_seg_elems,
                       self.current_lr(), self.rho, self.eps, self.momentum, self.clip, device=m.flat.device)
        m.refresh_shadow()
        for (name, keys, grads) in m._pending_sparse:
            table = m.tables[name]
            rows, E = table.shape
            if name in m.sharded:
                # row-sharded: gradient rows go to their owners (all-to-all), global-norm clip, Adagrad
                m.sharded[name].apply_gradient(keys, grads, self.acc[name], self.sparse_lr, self.sparse_eps,
                                               self.sparse_clip)
            elif name in early:
                # one all-reduce of the de-duplicated dense gradient (started above) instead of
                # all-gathering every rank's rows
                g, work, idx, cg = early[name]
                ev_c = self._mark()
                work.wait()
                if ev_c is not None:
                    self.exchange_events.append((ev_c, self._mark()))
                if idx is not None:                      # the union's summed rows back into the dense gradient
                    g.index_copy_(0, idx, cg)
                g.mul_(1.0 / otdist.world())
                K.dense_adagrad(table, self.acc[name], g, rows, E, self.sparse_lr, self.sparse_eps,
                                self.sparse_clip, device=table.device)
            else:
                keys, grads = otdist.allgather_sparse(keys, grads)
                K.sparse_adagrad(table, self.acc[name], E, rows, keys, grads, keys.numel(),
                                 self.sparse_lr, self.sparse_eps, self.sparse_clip, device=table.device)
        m._pending_sparse = []


class OneTransTrainer:
    """train.py:19-338 surface: train_step / val_step / train / save_model / load_model."""

    def __init__(self, config: OneTransConfig, model_dir: str = './models', device=None,
                 model: Optional[OneTransModel] = None, seed: int = 0):
        self.config = config
        self.model_dir = Path(model_dir)
        self.model = model if model is not None else OneTransModel(config, device=device, seed=seed)
        self.device = self.model.flat.device
        self.optimizer = OneTransOptimizer(self.model, config)
        self.history = {'train_loss': [], 'val_loss': [], 'train_metrics': {}, 'val_metrics': {}}

    # --------------------------------------------------------------- steps
    def train_step(self, batch_data, next_batch=None) -> Dict[str, torch.Tensor]:
        """train.py:111-155.  Returns {'total_loss': device scalar} (no host sync).  ``next_batch`` (optional, the
        batch the next call will get, e.g. from a prefetching loader): a row-sharded table routes its ids during
        this step (OneTransModel.route_ahead)."""
        non_seq, seq, labels = batch_data
        dev = self.device
        y = labels if isinstance(labels, torch.Tensor) else stack_labels(labels, self.config.tasks, dev)
        self.model.train()
        probs = self.model.forward_probs(_to_dev(non_seq, dev), _seq_inputs(self.model, seq, dev), training=True)
        if next_batch is not None and self.model.sharded:
            self.model.route_ahead(_seq_inputs(self.model, next_batch[1], dev))
        loss = keras_bce_loss(y, probs, self.config.tasks, label_rank(labels))
        self.optimizer.prepare_table_exchange()
        self.optimizer.begin_backward()
        loss.backward()
        self.optimizer.step()
        return {'total_loss': loss.detach(), 'probs': probs.detach()}

    @torch.no_grad()
    def val_step(self, batch_data) -> Dict[str, torch.Tensor]:
        """train.py:158-190."""
        non_seq, seq, labels = batch_data
        dev = self.device
        y = labels if isinstance(labels, torch.Tensor) else stack_labels(labels, self.config.tasks, dev)
        probs = self.model.forward_probs(_to_dev(non_seq, dev), _seq_inputs(self.model, seq, dev), training=False)
        loss = keras_bce_loss(y, probs, self.config.tasks, label_rank(labels))
        return {'total_loss': loss, 'probs': probs}

    def evaluate(self, batches) -> Dict[str, float]:
        """Per task over a list of batches: 'ctr' / 'cvr' (BCE tasks) the exact rank AUC + the Keras
        200-threshold AUC; any other task (trained with MSE, train.py:88-91) mse and mae, as the
        reference reports for regression tasks (train.py:106, evaluate.py:52-54)."""
        ps, ys = [], []
        for b in batches:
            out = self.val_step(b)
            ps.append(out['probs'].cpu().numpy())
            ys.append(stack_labels(b[2], self.config.tasks, 'cpu').numpy())
        P, Y = np.concatenate(ps, 1), np.concatenate(ys, 1)
        res = {}
        for i, t in enumerate(self.config.tasks):
            if t in BINARY_TASKS:
                res[f'{t}_auc'] = auc(Y[i], P[i])
                res[f'{t}_keras_auc'] = keras_auc(Y[i], P[i])
            else:
                e = P[i].astype(np.float64) - Y[i].astype(np.float64)
                res[f'{t}_mse'] = float(np.mean(e * e))
                res[f'{t}_mae'] = float(np.mean(np.abs(e)))
        return res

    def train(self, train_batches, val_batches=None, epochs: int = 1) -> Dict:
        """Minimal epoch loop (train.py:192-279): loss history and validation AUC."""
        for ep in range(epochs):
            t0 = time.time()
            losses = [self.train_step(b)['total_loss'] for b in train_batches]
            self.history['train_loss'].append(float(torch.stack(losses).mean()))
            if val_batches:
                self.history['val_metrics'][ep] = self.evaluate(val_batches)
            print(f'epoch {ep + 1}/{epochs} loss {self.history["train_loss"][-1]:.5f} ({time.time() - t0:.1f}s)')
        return self.history

    # --------------------------------------------------------------- checkpoint (train.py:281-338)
    def save_model(self, model_name: str) -> None:
        path = self.model_dir / model_name
        path.mkdir(parents=True, exist_ok=True)          # the reference never creates it
        self.model.save_weights(str(path / 'model_weights.npz'))
        with open(path / 'config.json', 'w') as f:
            json.dump(self.config.to_dict(), f, indent=2)
        with open(path / 'training_history.json', 'w') as f:
            # the dense optimizer's step count travels with the history, so a resumed run continues the
            # LR warm-up ramp (apply_warmup) where it stopped
            json.dump(dict(self.history, optimizer_steps=self.optimizer.steps_done), f, indent=2, default=float)

    def load_model(self, model_path: str) -> None:
        path = Path(model_path)
        if (path / 'config.json').exists():
            with open(path / 'config.json') as f:
                self.config = OneTransConfig.from_dict(json.load(f))
            self.model = OneTransModel(self.config, device=self.device)
            self.optimizer = OneTransOptimizer(self.model, self.config)
        if (path / 'model_weights.npz').exists():
            self.model.load_weights(str(path / 'model_weights.npz'))
        if (path / 'training_history.json').exists():
            with open(path / 'training_history.json') as f:
                self.history = json.load(f)
            self.optimizer.steps_done = int(self.history.pop('optimizer_steps', 0))


def train_one_trans_model(config_name: str = 'small', batches=None, epochs: int = 10,
                          model_dir: str = './models') -> OneTransTrainer:
    """train.py:341-374 (synthetic batches when none are given)."""
    from .data import make_batch
    config = get_model_config(config_name)
    trainer = OneTransTrainer(config, model_dir)
    if batches is None:
        batches = [make_batch(32, config, seed=1000 + i, seq_lens=[16, 16, 16]) for i in range(4)]
    trainer.train(batches, batches[:1], epochs=epochs)
    return trainer
