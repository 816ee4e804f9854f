#!/usr/bin/env python3
"""Benchmark: ranked samples/sec (fwd+bwd) of the OneTrans training step at B=4096 seq=128
(BASELINE.json configs[1] = "C2": 4 layers, d=128, H=4, f=512, 12 NS + 128 S tokens, Criteo-shape
inputs with replicated embedding tables), one process per GPU (weak scaling: 4096 samples per GPU).

A step = forward + backward + optimizer (clip + RMSprop dense, Adagrad sparse) + the DP gradient
exchange when N > 1.  Inputs are synthetic Criteo-shape batches generated on the host and made
resident in HBM before the timed region (a ring of distinct batches is cycled).

Launch: python bench.py --gpus 1 --steps 20 --warmup 5
        python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

Prints ONE JSON line (rank 0) with the roofline of the dominant kernel (the mixed-parameterisation
GEMM family, fp32 MFMA) measured with HIP events around its launches inside the timed region, and
the CPU baseline (oracle/ restatement, torch CPU fp32) timed on this node's host cores.
"""

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP32_MFMA_PEAK_TFLOPS = 157.3      # MI355X_MICROARCH.md: Peak FP32 (matrix), dense
BF16_MFMA_PEAK_TFLOPS = 16 * FP32_MFMA_PEAK_TFLOPS   # "1/16 of BF16" (same table): 2516.8 dense
SPLIT_TERMS = 6                    # bf16 MFMA products per f32 product in OT_MATMUL_SPLIT_BF16
HBM_PEAK_GBS = 8000.0
# dense RMSprop settings of the default bench trajectory: config.py's dense_lr 0.005 with momentum 0.99999 drives the
# weights to inf within ~100 steps; at these (an optimizer_config train.py:60-66 accepts) the model trains and every
# timed step runs on finite operands (the kernels' work is the same either way)
TRAINABLE_OPT = {'dense_lr': 1e-4, 'momentum': 0.9}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=50)
    ap.add_argument('--warmup', type=int, default=10)
    ap.add_argument('--config', default='C2')
    ap.add_argument('--batch', type=int, default=0, help='per-GPU batch (default: the config\'s)')
    ap.add_argument('--nbatches', type=int, default=4, help='distinct resident batches cycled')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-batch', type=int, default=0,
                    help="samples per CPU-baseline step (default: the config's per-GPU batch)")
    ap.add_argument('--cpu-steps', type=int, default=2, help='timed CPU-baseline steps (after one warm-up step)')
    ap.add_argument('--optimizer', default='trainable', choices=['trainable', 'reference'],
                    help="dense RMSprop settings.  trainable (default): dense_lr 1e-4, momentum 0.9 (an optimizer_config "
                         "the reference trainer accepts, train.py:60-66), on which the f32 model trains and the loss stays "
                         "finite; reference: config.py's dense_lr 0.005 / momentum 0.99999, under which the weights blow "
                         "up within ~100 steps (identical kernel work, but NaN-state operands change kernel timing)")
    ap.add_argument('--allow-nonfinite', action='store_true',
                    help='report instead of failing when a repeat ends on a non-finite loss (diagnostics only)')
    ap.add_argument('--no-probe', action='store_true', help='skip the per-kernel HIP-event (roofline) pass')
    ap.add_argument('--probe-steps', type=int, default=10, help='steps of the roofline pass (0: no roofline)')
    ap.add_argument('--repeats', type=int, default=3, help='timed regions of --steps steps; value = median')
    ap.add_argument('--no-lookahead', action='store_true',
                    help='row-sharded tables route each step\'s ids when it starts (default: during the step before)')
    ap.add_argument('--no-overlap', action='store_true',
                    help='weight gradients on the main stream for the whole run (rocprofv3 runs: every kernel '
                         'standalone, so its trace durations compare with the roofline pass)')
    ap.add_argument('--precision', default='auto', choices=['auto', 'split', 'f32', 'bf16', 'fp8attn'],
                    help="GEMM / attention arithmetic.  auto: the config's stated precision — C5 (BASELINE "
                         "configs[4]) 'fp8attn' (bf16 GEMMs + block-scaled fp8 attention forward), every other "
                         "config the reference's f32 via the exact split-bf16 GEMMs (ONETRANS_MATMUL overrides)")
    return ap.parse_args()


def init_dist(args):
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        import torch.distributed as dist
        # OT_BENCH_BACKEND=gloo OT_BENCH_SAME_DEVICE=1 rehearses the N>1 path on a one-GPU box (every
        # rank on cuda:0, collectives over gloo); the real multi-GPU run uses RCCL ("nccl"), one GPU/rank
        if os.environ.get('OT_BENCH_SAME_DEVICE') == '1':
            local = 0
        torch.cuda.set_device(local)
        backend = os.environ.get('OT_BENCH_BACKEND', 'nccl')
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    return world, rank, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def device_batches(cfg, B, n, rank, dev):
    from recommend_amd.data import make_batch
    from recommend_amd.trainer import stack_labels
    out = []
    for i in range(n):
        ns, seq, lab = make_batch(B, cfg, seed=100000 * (rank + 1) + i)
        out.append(({k: torch.from_numpy(v).to(dev) for k, v in ns.items()},
                    {k: torch.from_numpy(v).to(dev) for k, v in seq.items()},
                    stack_labels(lab, cfg.tasks, dev)))
    return out


def log(msg):
    """Progress to stderr (rank 0): a long bench keeps writing, and the JSON line stays alone on stdout."""
    if int(os.environ.get('RANK', '0')) == 0:
        print(f'[bench {time.strftime("%H:%M:%S")}] {msg}', file=sys.stderr, flush=True)


def cpu_baseline(cfg_name, batch, steps, optimizer_config):
    """Oracle (torch CPU fp32, the vectorized restatement of model.py / train.py) train steps on the host
    cores at the configured batch: one warm-up step, then ``steps`` timed steps (forward + backward +
    clip + RMSprop + Adagrad, the GPU step's work)."""
    from recommend_amd.config import workload_config
    from recommend_amd.data import make_batch
    from recommend_amd.params import init_params, keras_variables
    from oracle import onetrans_ref as R
    cores = len(os.sched_getaffinity(0))          # the node's host cores this process may run on
    quota = None                                   # cgroup CPU quota (cores' worth), when the container sets one
    try:
        q, per = open('/sys/fs/cgroup/cpu.max').read().split()[:2]
        quota = None if q == 'max' else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    # one thread per core this process can actually run on: the affinity set, or the cgroup's CPU share when
    # that is smaller (the GPU box lists the whole machine's CPUs in the affinity mask but grants a 16-CPU
    # quota; 200+ threads under it throttle each other to a standstill)
    threads = cores if quota is None else max(1, min(cores, int(quota + 0.999)))
    torch.set_num_threads(threads)
    cfg = workload_config(cfg_name)
    cfg.optimizer_config = dict(optimizer_config)
    # the oracle's table gradient is dense (a [rows, E] tensor per table): cap the table cardinalities so it
    # stays small; ids are drawn mod the cap, the transformer work is unchanged
    cfg.sparse_features = {k: min(v, 20000) for k, v in cfg.sparse_features.items()}
    cfg.seq_item_vocab = min(cfg.seq_item_vocab, 50000)
    B = batch
    P = init_params(cfg, cfg.ns_input_width(), seed=0)
    kv = keras_variables(cfg, {k: v.shape for k, v in P.items() if not k.startswith('emb.')})
    tb = [tuple(R.to_torch(x, dtype=torch.float32) for x in make_batch(B, cfg, seed=7000 + i)) for i in range(2)]
    Pt = R.to_torch(P, dtype=torch.float32)
    st = R.init_state(Pt, cfg)
    t0 = time.perf_counter()
    Pt, st, _, _ = R.train_step(Pt, st, cfg, kv, *tb[0], seed=1, variant='vectorized')          # warm-up
    log(f'cpu baseline: warm-up step (B={B}) {time.perf_counter() - t0:.1f}s on {threads} threads')
    t0 = time.perf_counter()
    for n in range(steps):
        Pt, st, loss, _ = R.train_step(Pt, st, cfg, kv, *tb[(n + 1) % 2], seed=2 + n, variant='vectorized')
    el = time.perf_counter() - t0
    log(f'cpu baseline: {steps} steps in {el:.1f}s')
    return {'value': round(B * steps / el, 2), 'unit': 'samples/s', 'cores': torch.get_num_threads(),
            'affinity_cores': cores, 'cgroup_cpu_quota_cores': quota, 'kind': 'port', 'variant': 'vectorized',
            'final_loss': round(float(loss), 5),
            'sample': f'{steps} train steps x B={B} of {cfg_name} after 1 warm-up step (full model shape, fp32, '
                      f'the vectorized oracle restatement of model.py / train.py; embedding tables capped at '
                      f'2e4 / 5e4 rows because the oracle\'s table gradient is dense), {el:.1f}s'}


def hbm_traffic(config):
    """HBM bytes per launch of the GEMM family from the newest committed PMC summary
    (tools/hbm_traffic.py: separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes over this bench,
    calibrated on a known 1 GiB copy).  (None, None) when no summary for this config exists."""
    import glob
    for fn in sorted(glob.glob(os.path.join(ROOT, 'profiles', '*', 'hbm_traffic*.json')), reverse=True):
        try:
            d = json.load(open(fn))
        except (OSError, ValueError):
            continue
        if d.get('config') == config and 'gemm' in d.get('families', {}):
            return round(d['families']['gemm']['hbm_bytes_per_launch']), os.path.relpath(fn, ROOT)
    return None, None


def attention_pmc(config):
    """MFMA-busy and VALU-per-MFMA of the attention kernels from the newest committed PMC summary of this
    config's layer shape (tools/pmc_attn.sh -> profiles/*/pmc_attn_<config>.json), or None."""
    import glob
    for fn in sorted(glob.glob(os.path.join(ROOT, 'profiles', '*', f'pmc_attn_{config}.json')), reverse=True):
        try:
            d = json.load(open(fn))
        except (OSError, ValueError):
            continue
        d['source'] = os.path.relpath(fn, ROOT)
        return d
    return None


def main():
    args = parse()
    world, rank, local = init_dist(args)
    from recommend_amd import kernels as K
    from recommend_amd.config import algorithmic_flops_per_sample, workload_config
    from recommend_amd.model import OneTransModel, keras_bce_loss
    from recommend_amd.trainer import OneTransOptimizer, OneTransTrainer

    dev = torch.device('cuda', local if world > 1 else 0)
    cfg = workload_config(args.config)
    precision = args.precision
    if precision == 'auto':
        precision = 'fp8attn' if args.config == 'C5' else os.environ.get('ONETRANS_MATMUL', 'split')
    K.set_matmul_mode('bf16' if precision in ('bf16', 'fp8attn') else precision)
    cfg.compute_dtype = {'fp8attn': 'fp8attn', 'bf16': 'bf16'}.get(precision, 'fp32')
    if args.optimizer == 'trainable':
        cfg.optimizer_config = dict(cfg.optimizer_config, **TRAINABLE_OPT)
    B = args.batch or cfg._batch
    model = OneTransModel(cfg, device=dev, seed=0)
    if args.no_overlap:
        model.overlap_wgrad = False
    trainer = OneTransTrainer(cfg, model=model)
    log(f'{args.config}: model built ({precision})')
    batches = device_batches(cfg, B, args.nbatches, rank, dev)
    log(f'{args.nbatches} resident batches of {B}')
    torch.cuda.synchronize()
    model.inputs_ready = True           # resident, complete batches: a row-sharded lookup routes them at once

    def step(i):
        ns, seq, y = batches[i % len(batches)]
        # the next batch is known (resident ring): a row-sharded table routes its ids during this step
        nxt = None if args.no_lookahead else batches[(i + 1) % len(batches)]
        return trainer.train_step((ns, seq, y), next_batch=nxt)

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()

    # N > 1 diagnostics: main-stream time spent waiting for the gradient exchange (not hidden by the
    # backward) and the row-sharded tables' all-to-all lookups / updates
    exch = [] if world > 1 else None
    trainer.optimizer.exchange_events = exch
    for st_ in model.sharded.values():
        st_.events = exch

    def timed_region(first):
        barrier(world)
        torch.cuda.synchronize()
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record()
        for i in range(args.steps):
            o = step(first + i)
        ev1.record()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        barrier(world)
        torch.cuda.synchronize()
        return max(wall, ev0.elapsed_time(ev1) / 1e3), o

    times, exposed, route_wait, losses = [], [], [], []
    log(f'{args.warmup} warm-up steps done')
    for r in range(max(1, args.repeats)):
        for st_ in model.sharded.values():
            st_.route_wait_s = 0.0
        t_r, out = timed_region(args.warmup + r * args.steps)
        times.append(t_r)
        losses.append(float(out['total_loss'].item()))        # after the region's closing synchronize
        if not np.isfinite(losses[-1]) and not args.allow_nonfinite:
            raise SystemExit(f'bench: repeat {r} ended on a non-finite loss ({losses[-1]}); the timed steps ran on '
                             f'degenerate operands (--allow-nonfinite to report anyway)')
        log(f'repeat {r}: {1e3 * t_r / args.steps:.3f} ms/step, loss {losses[-1]:.5f}')
        route_wait.append(1e3 * sum(st_.route_wait_s for st_ in model.sharded.values()) / args.steps)
        if exch is not None:
            ms = sum(a.elapsed_time(b) for (a, b) in exch)
            exch.clear()
            exposed.append(ms / args.steps)
    rank_t = sorted(times)[len(times) // 2]          # this rank's median timed region
    t = rank_t
    per_rank = [rank_t]
    if world > 1:
        import torch.distributed as dist
        tt = torch.tensor([rank_t, float(np.median(exposed)) if exposed else 0.0, float(np.median(route_wait))],
                          device='cpu' if dist.get_backend() == 'gloo' else dev)
        gath = [torch.empty_like(tt) for _ in range(world)]
        dist.all_gather(gath, tt)
        allr = torch.stack(gath).cpu()
        per_rank = allr[:, 0].tolist()
        exposed_ranks = allr[:, 1].tolist()
        route_wait_ranks = allr[:, 2].tolist()
        t = max(per_rank)                             # max over ranks
    loss = float(out['total_loss'].item())
    trainer.optimizer.exchange_events = None
    for st_ in model.sharded.values():
        st_.events = None
    done_steps = args.warmup + max(1, args.repeats) * args.steps

    # Roofline pass (after the timed region, every rank): per-launch HIP events on the launch stream,
    # with the weight-gradient side stream off so each kernel is timed standalone (in the timed region
    # the wgrads overlap the dgrad chain and a launch's duration would include its neighbour's share).
    rep = None
    if not args.no_probe and args.probe_steps > 0:
        overlap = model.overlap_wgrad
        model.overlap_wgrad = False
        probe = K.Probe()
        K.set_probe(probe)
        for i in range(args.probe_steps):
            step(done_steps + i)
        torch.cuda.synchronize()
        K.set_probe(None)
        model.overlap_wgrad = overlap
        mm = model.matmul
        gpk = (BF16_MFMA_PEAK_TFLOPS / SPLIT_TERMS if mm == 'split' else
               BF16_MFMA_PEAK_TFLOPS if mm == 'bf16' else FP32_MFMA_PEAK_TFLOPS)
        # each launch is floored against the ceiling of the arithmetic it issues: bf16 dense / 6 for the split-bf16
        # kernels, / 3 for the fp16-pair ones (f16 dense = bf16 dense), bf16 dense for the bf16 mode
        rep = probe.report(args.probe_steps, gpk, HBM_PEAK_GBS,
                           terms_peak=lambda t: BF16_MFMA_PEAK_TFLOPS / t if t in (1, 3, 6) else FP32_MFMA_PEAK_TFLOPS)

    if rank != 0:
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return

    seq_lens = cfg._seq_lens
    fl = algorithmic_flops_per_sample(cfg, seq_lens, cfg.ns_input_width())
    samples = B * args.steps * world
    value = samples / t
    res = {
        'metric': 'ranked samples/sec (fwd+bwd) at B=4096 seq=128; AUC parity vs ref',
        'value': round(value, 1), 'unit': 'samples/s', 'n_gpus': world, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': round(1e3 * t / args.steps, 3), 'higher_is_better': True,
        'scaling': 'weak', 'vs_baseline': None,
        # the f32-accurate mode emulates f32 products on 16-bit MFMA: split-bf16 (three planes, six products) and,
        # for the QKV / FFN1 / FFN2 forward GEMMs and the slice attention, a scaled fp16 pair (22 significant bits
        # relative to a row / column bound); bf16 is C5's stated reduced precision
        'dtype': ('bf16' if model.matmul == 'bf16' else
                  'f32-emulated (fp16-pair / split-bf16)' if model.matmul == 'split' else 'f32'),
        'data': 'synthetic', 'precision': precision,
        'optimizer': {'kind': args.optimizer, 'dense_lr': trainer.optimizer.lr,
                      'momentum': trainer.optimizer.momentum, 'sparse_lr': trainer.optimizer.sparse_lr},
        'config': {'workload': f'{args.config}: OneTrans {cfg.num_layers}L d{cfg.hidden_dim} H{cfg.num_heads} f{cfg.ffn_dim} '
                               f'L_NS{cfg.num_ns_tokens} L_S{sum(seq_lens) + 2} (seq 3x{seq_lens[0]}), '
                               f'Criteo-shape 13 dense + 26 ids, '
                               f'{"row-sharded " + ", ".join(sorted(model.sharded)) if model.sharded else "replicated tables"}, '
                               f'fwd+bwd+optimizer',
                   'global_batch': B * world, 'per_gpu_batch': B, 'seq_len': sum(seq_lens) + 2,
                   'parallelism': f'dp{world}'},
        'model_tflops': round(fl['fwd_bwd'] * value / 1e12, 2),
        'final_loss': round(loss, 5), 'loss_repeats': [round(x, 5) for x in losses],
        'repeats': len(times), 'ms_per_step_repeats': [round(1e3 * x / args.steps, 3) for x in times],
        'peak_hbm_gb': round(torch.cuda.max_memory_allocated(dev) / 2 ** 30, 2),
        'recompute': bool(model.recompute),
    }
    if world > 1:
        import torch.distributed as dist
        res['dist'] = {'backend': dist.get_backend(), 'world_size': dist.get_world_size(),
                       'rank_ms_per_step_min': round(1e3 * min(per_rank) / args.steps, 3),
                       'rank_ms_per_step_max': round(1e3 * max(per_rank) / args.steps, 3),
                       'exposed_exchange_ms_per_step_max': round(max(exposed_ranks), 3),
                       'exposed_exchange_ms_per_step_min': round(min(exposed_ranks), 3),
                       'sharded_tables': sorted(model.sharded),
                       # host time the row-sharded lookups spend routing at the start of a step's forward,
                       # before their first gather launch (look-ahead routing moves it into the step before)
                       'route_host_wait_ms_per_step_max': round(max(route_wait_ranks), 3),
                       'lookahead_routing': not args.no_lookahead,
                       # per row-sharded table: rows this rank sent to their owners in the last lookup
                       # (distinct ids when de-duplicated) and the ids of that lookup
                       'sharded_rows_sent_of_ids': {k: [t.sent_rows, t.last_route[0] if t.last_route else 0]
                                                    for k, t in sorted(model.sharded.items())},
                       'note': 'exposed exchange = HIP-event time the main stream waits for the dense '
                               'gradient all-reduce and the replicated-table exchange after backward, plus the '
                               'row-sharded tables\' all-to-all lookups and updates (median repeat)'}
    if rep is not None and 'mixed_gemm' in rep['families']:
        traffic, tsrc = hbm_traffic(args.config)
        dom = rep['families']['mixed_gemm']
        if model.matmul == 'split':
            # the GEMMs issue either 6 bf16 products per f32 product (the exact three-plane split) or 3 f16 products
            # (the scaled fp16 pair): the family's ceiling is that of the mix it issued (mfma_peak_eff: its flops
            # over sum flops_i / (bf16 dense / terms_i))
            gpeak = round(dom['mfma_peak_eff'], 1)
            gkern = ('plane_gemm_kernel / mixed_gemm_kernel + wgrad_split_kernel: f32 operands as a scaled fp16 pair '
                     '(3 f16 MFMA products per f32 product; ceiling bf16 dense / 3 = 838.9) or split exactly into 3 bf16 '
                     f'parts (6 products; / 6 = 419.5); peak = the issued mix\'s ceiling '
                     f'({dom["pair_launches_per_step"]:.0f} of {dom["launches_per_step"]:.0f} launches per step on the pair)')
        elif model.matmul == 'bf16':
            gpeak = BF16_MFMA_PEAK_TFLOPS
            gkern = ('plane_gemm_kernel (128x128; plane_wide_kernel 128x256 where K >= N) / mixed_gemm_kernel + '
                     'wgrad_bf16_sq_kernel (256x256) / wgrad_split_kernel (operands rounded to bf16, one bf16 MFMA '
                     'product)')
        else:
            gpeak = FP32_MFMA_PEAK_TFLOPS
            gkern = 'mixed_gemm_kernel + wgrad_kernel (native f32 MFMA)'
        res['matmul'] = model.matmul
        # the family's binding roof: each launch is floored by max(flops / MFMA peak, bytes / HBM peak);
        # 'bound' is the roof that holds the larger share of that floor over the family's launches
        # (C2's K = 128 GEMMs sit right of the ridge on HBM; C5's bf16 GEMMs on MFMA)
        hbm_bound = dom['floor_hbm_ms_per_step'] > dom['floor_mfma_ms_per_step']
        mfma = {'achieved': round(dom['tflops'], 2), 'peak': gpeak, 'unit': 'TFLOP/s',
                'frac': round(dom['tflops'] / gpeak, 4)}
        hbm = {'achieved': round(dom['gbs'], 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
               'frac': round(dom['gbs'] / HBM_PEAK_GBS, 4)}
        res['roofline'] = {'bound': 'hbm' if hbm_bound else 'mfma', 'kernel': gkern,
                           **(hbm if hbm_bound else mfma), 'traffic': traffic,
                           'traffic_unit': 'HBM bytes per launch (PMC FETCH_SIZE + WRITE_SIZE, calibrated)',
                           'traffic_source': tsrc,
                           'algorithmic_bytes_per_launch': round(dom['gbyte_per_launch'] * 1e9),
                           'gflop_per_launch': round(dom['gflop_per_launch'], 3),
                           'avg_launch_us': round(dom['avg_us'], 2), 'launches_per_step': dom['launches_per_step'],
                           'mfma': mfma, 'hbm': hbm,
                           'floor_ms_per_step': round(dom['floor_ms_per_step'], 3),
                           'floor_frac': round(dom['floor_ms_per_step'] / dom['ms_per_step'], 4),
                           'floor_split_ms': {'mfma_bound_launches': round(dom['floor_mfma_ms_per_step'], 3),
                                              'hbm_bound_launches': round(dom['floor_hbm_ms_per_step'], 3)},
                           'measured': f'HIP events per launch, {args.probe_steps}-step pass after the timed region, '
                                       'wgrad side stream off (standalone kernel durations); algorithmic bytes = '
                                       'A (+ rstd) read once, C written once, each [M, N] epilogue operand read once, '
                                       'wgrad A + D read once and dW written once (weights of the forward / dgrad '
                                       'launches left out); floor = sum over launches of max(flops / MFMA peak, '
                                       'bytes / HBM peak), floor_frac = floor / measured family time'}
        res['kernel_time_ms_per_step'] = {k: round(v['ms_per_step'], 3) for k, v in rep['families'].items()}
        # north_star "MFMA utilisation on OneTrans attention" (standalone attention at
        # L~140 is memory-heavy, so the block's matrix work is reported beside the core): achieved
        # algorithmic fraction of (i) the attention core kernels, (ii) the transformer block = every
        # MFMA kernel (GEMMs + attention) over all of the block's kernel time (+ row-wise kernels)
        fams = rep['families']
        att = fams.get('attention')
        if att is not None:
            ms = lambda f: fams[f]['ms_per_step'] if f in fams else 0.0
            fl = lambda f: fams[f]['tflops'] * fams[f]['ms_per_step'] * 1e9 if f in fams else 0.0
            blk_fl = fl('mixed_gemm') + fl('attention')
            blk_ms = ms('mixed_gemm') + ms('attention') + ms('rowwise')
            bf16 = model.matmul == 'bf16'
            # the f32-accurate attention is priced against the native f32 MFMA peak (what an exact-f32 attention
            # could reach), and beside it against the ceiling of the arithmetic it actually issues: the slice
            # kernels (I <= 192) run each f32 product as 3 fp16 MFMA products (two scaled fp16 planes; the
            # head_dim-32 forward as 6 bf16 products of three planes), so that ceiling is bf16 dense / 3
            apeak = BF16_MFMA_PEAK_TFLOPS if bf16 else FP32_MFMA_PEAK_TFLOPS
            issued_peak = BF16_MFMA_PEAK_TFLOPS if bf16 else BF16_MFMA_PEAK_TFLOPS / 3
            gpe = fams['mixed_gemm'].get('mfma_peak_eff') or gpk if 'mixed_gemm' in fams else gpk
            busy_ms = fl('mixed_gemm') / (gpe * 1e9) + fl('attention') / (apeak * 1e9)
            res['attention_mfma'] = {
                'core_tflops': round(att['tflops'], 2),
                'core_frac': round(att['tflops'] / apeak, 4),
                'core_peak': apeak,
                'core_frac_of_issued_ceiling': round(att['tflops'] / issued_peak, 4),
                'issued_ceiling': round(issued_peak, 1),
                'block_tflops': round(blk_fl / (blk_ms * 1e-3) / 1e12, 2),
                'block_frac': round(busy_ms / blk_ms, 4), 'unit': 'TFLOP/s',
                'note': 'algorithmic flops (tail-only queries, causal pairs) / HIP-event kernel time; '
                        + ('attention on bf16 MFMA (peak = bf16 dense 2516.8; with fp8attn the forward runs '
                           'block-scaled fp8, whose dense peak is 2x)' if bf16 else
                           'f32-accurate attention: core_frac against the native f32 MFMA peak 157.3; the kernels '
                           'issue split MFMA products (slice kernels: 3 fp16 products per f32 product, the hd-32 '
                           'forward 6 bf16 products; the head_dim-64 backward up to I 544 also on the slice '
                           'kernels; longer forwards: 6 bf16 products, other shapes native f32), so '
                           'core_frac_of_issued_ceiling prices them against bf16 dense / 3')}
            pmc = attention_pmc(args.config)
            if pmc is not None:
                res['attention_mfma']['pmc'] = pmc
    if not args.no_cpu_baseline and world == 1:          # rank 0 at N=1 only
        log('timed region and probe done; CPU baseline')
        res['cpu_baseline'] = cpu_baseline(args.config, args.cpu_batch or B, args.cpu_steps,
                                           cfg.optimizer_config)
    print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
