"""Two-stage cached serving of a trained OneTrans model (paper §3.5.1 "cross-request KV cache").

Reference: the inference engine ``examples/inference_example.py:21-219`` (one full forward per batch
of (user, item, context, sequence) samples) and the model's KV-cache path ``model.py:94-98, 333,
359-381, 395-397``, which is defective (D6: block i's K/V are fed to block i+1 and the causal mask is
not offset by the cache length), so the cache semantics are re-derived from the paper:

* stage I, once per request (user): the S tokens (sequences + [SEP]) run through every layer on their
  own.  Tokens are ordered [S; NS] (model.py:235) and the mask is causal, so no S token ever sees an
  NS token: the S-side hidden states, keys and values do not depend on the candidate.  Each layer's
  S-side K/V rows are cached (``RequestCache``).
* stage II, once per candidate: the NS tokens run through every layer; their queries attend to the
  request's cached S-side K/V plus their own (``ot_attn_fwd_cached``).  Nothing S-side is recomputed.

The result equals ``OneTransModel.forward`` on the expanded batch (each candidate paired with its
request's sequences) up to fp32 summation order — tests/test_serving_gpu.py checks it against the
model and the CPU oracle.  Pyramid keeps (tail, model.py:296/371 with the D2 fix) and the last-layer
dead-code elimination carry over: at layer l the kept tail of K_l tokens splits into S rows (computed
in stage I) and N rows (stage II).  Inference only (no dropout).  Positions restart in every layer,
so every row's weight group is the one of its position in the full layer input
(``layout.layer_maps(p0=, I_full=)``).

Cross-request reuse (``extend_requests``): new behaviours appended to the LAST configured sequence
extend the S side at its end, so with no pruning before the last layer only the new tokens are computed
(their queries over the cached K/V).  Appends anywhere else shift later positions (later sequences,
[SEP] tokens, position-grouped weights) and need a full stage-I re-encode; that case raises.
"""

from __future__ import annotations

from typing import Dict, List, Optional

import torch

from . import kernels as K
from ._lib import (OT_AX_GELU, OT_AX_RMSNORM, OT_EPI_BIAS, OT_EPI_RESIDUAL, OT_GEMM_NT, OneTransHipError)
from .layout import layer_maps

RMS_EPS = 1e-6


class RequestCache:
    """Stage-I output for R requests: per layer the S-side qkv rows [R*Ic, 3d] (k at col d, v at 2d)
    and Ic, the number of S tokens in that layer's input."""

    def __init__(self, R: int, L_S: int, layers: List[Dict], present=()):
        self.R, self.L_S, self.layers = R, L_S, layers
        self.present = tuple(present)          # sequence names present in the requests, config order


class OneTransServer:
    """Cached two-stage inference on a ``OneTransModel`` (weights shared, nothing copied)."""

    def __init__(self, model):
        self.m = model
        cfg = model.config
        if getattr(cfg, 'pyramid_select', 'tail') != 'tail':
            raise ValueError("OneTransServer: pyramid_select must be 'tail' (a score-based keep would depend on "
                             "the NS tokens' positions in every layer)")
        self._maps = {}

    # ------------------------------------------------------------------ schedule

    @property
    def precision_model(self):
        """The model whose arithmetic the cached stages run in (kernels.in_model_precision)."""
        return self.m
    def schedule(self, L_S: int) -> List[Dict]:
        """Per layer: S rows s, N rows n, kept S rows kS, kept N rows kN (kS + kN = the layer's keep)."""
        cfg = self.m.config
        L_NS = cfg.num_ns_tokens
        sched = cfg.pyramid_schedule(L_S + L_NS)
        out, s, n = [], L_S, L_NS
        for l, e in enumerate(sched):
            keep = e['keep'] if l < len(sched) - 1 else 1        # only the last token is read (model.py:390)
            kN = min(keep, n)
            kS = keep - kN
            out.append({'I': s + n, 's': s, 'n': n, 'kS': kS, 'kN': kN})
            s, n = kS, kN
        return out

    def _layer_maps(self, B, I, Kq, p0, I_full):
        key = (B, I, Kq, p0, I_full)
        if key not in self._maps:
            self._maps[key] = layer_maps(self.m.config, B, I, Kq, p0=p0, I_full=I_full)
        return self._maps[key]

    # ------------------------------------------------------------------ one block (forward only)
    def _block(self, l: int, x: torch.Tensor, B: int, I: int, Kq: int, p0: int, I_full: int, attn):
        """OneTransBlock.call (model.py:186-200) on B spans of I rows (positions p0.. of a layer of I_full
        tokens), keeping the last Kq (0: only the K/V rows are produced).  Returns (x_next, qkv)."""
        m = self.m
        cfg = m.config
        d, f = cfg.hidden_dim, cfg.ffn_dim
        dev = x.device
        mp = self._layer_maps(B, I, max(Kq, 1), p0, I_full)
        ma, mt = mp['all'].to(dev), mp['tail'].to(dev)
        na, nt = mp['all'].ntiles, mp['tail'].ntiles
        wqkv, wo = m.pT(f'blk.{l}.wqkv'), m.pT(f'blk.{l}.wo')
        w1, b1, w2, b2 = m.pT(f'blk.{l}.w1'), m.p(f'blk.{l}.b1'), m.pT(f'blk.{l}.w2'), m.p(f'blk.{l}.b2')
        g1, g2 = m.p(f'blk.{l}.norm1'), m.p(f'blk.{l}.norm2')
        rstd1 = torch.empty(B * I, device=dev)
        K.rmsnorm_fwd(x, d, B * I, d, rstd1, eps=RMS_EPS)
        qkv = torch.empty(B * I, 3 * d, device=dev)
        # K/V for every row (weight cols d..3d of each group's [d, 3d] bank), Q for the kept rows
        K.gemm(OT_GEMM_NT, x, d, d, ma['rows'][0], (wqkv, d * d), 3 * d * d, d, 2 * d, ma['tile_group'], na,
               (qkv, d), 3 * d, ma['rows'][0], a_xform=OT_AX_RMSNORM, rstd=rstd1, gamma=g1, m_rows=mp['all'].nrows)
        if Kq == 0:
            return None, qkv
        K.gemm(OT_GEMM_NT, x, d, d, mt['rows'][0], wqkv, 3 * d * d, d, d, mt['tile_group'], nt, qkv, 3 * d,
               mt['rows'][0], a_xform=OT_AX_RMSNORM, rstd=rstd1, gamma=g1, m_rows=mp['tail'].nrows)
        o = attn(qkv)                                                   # [B*Kq, d]
        x1 = torch.empty(B * Kq, d, device=dev)
        K.gemm(OT_GEMM_NT, o, d, d, mt['rows'][1], wo, 0, d, d, mt['tile_group'], nt, x1, d, mt['rows'][1],
               epi=OT_EPI_RESIDUAL, res=x, ldres=d, res_tok=1, tail=(Kq, I), m_rows=mp['tail'].nrows)
        rstd2 = torch.empty(B * Kq, device=dev)
        K.rmsnorm_fwd(x1, d, B * Kq, d, rstd2, eps=RMS_EPS)
        u = torch.empty(B * Kq, f, device=dev)
        K.gemm(OT_GEMM_NT, x1, d, d, mt['rows'][1], w1, d * f, d, f, mt['tile_group'], nt, u, f, mt['rows'][1],
               a_xform=OT_AX_RMSNORM, rstd=rstd2, gamma=g2, bias=b1, bias_gstride=f, epi=OT_EPI_BIAS,
               m_rows=mp['tail'].nrows)
        x2 = torch.empty(B * Kq, d, device=dev)
        K.gemm(OT_GEMM_NT, u, f, f, mt['rows'][1], w2, f * d, f, d, mt['tile_group'], nt, x2, d, mt['rows'][1],
               a_xform=OT_AX_GELU, bias=b2, bias_gstride=d, epi=OT_EPI_BIAS | OT_EPI_RESIDUAL, res=x1, ldres=d,
               res_tok=0, tail=(Kq, I), m_rows=mp['tail'].nrows)
        return x2, qkv

    # ------------------------------------------------------------------ stage I
    @torch.no_grad()
    @K.in_model_precision
    def encode_requests(self, seq_features: Dict[str, torch.Tensor]) -> RequestCache:
        """Tokenize the requests' sequences (model.py:256-277) and run the S side of every layer;
        cache each layer's S-side K/V."""
        from .model import _Tokenize
        m = self.m
        cfg = m.config
        d, H = cfg.hidden_dim, cfg.num_heads
        hd = d // H
        if not seq_features:
            raise ValueError('encode_requests: no sequence features')
        plan = m._plan({}, seq_features)
        R, L0, L_S = plan['B'], plan['L0'], plan['L_S']
        x0 = _Tokenize.apply(m.flat, m, plan)                             # NS rows zero (no NS features)
        x = x0.view(R, L0, d)[:, :L_S].reshape(R * L_S, d)
        layers = []
        for l, e in enumerate(self.schedule(L_S)):
            s, kS = e['s'], e['kS']
            if s == 0:
                layers.append({'Ic': 0, 'kv': None})
                continue

            def attn(qkv, s=s, kS=kS):
                o = torch.empty(R * kS, d, device=qkv.device)
                lse = torch.empty(R * H * kS, device=qkv.device)
                K.attn_fwd(qkv, 3 * d, R, H, s, kS, hd, o, lse)           # S queries see S keys only
                return o

            x, qkv = self._block(l, x, R, s, kS, 0, e['I'], attn)
            layers.append({'Ic': s, 'kv': qkv})
        present = [n for n in cfg.feature_config['sequence_features'] if n in seq_features]
        return RequestCache(R, L_S, layers, present)

    # ------------------------------------------------------------------ cross-request append
    @torch.no_grad()
    @K.in_model_precision
    def extend_requests(self, cache: RequestCache, seq_name: str, new_events: torch.Tensor) -> RequestCache:
        """Cross-request KV cache (paper §3.5.1): the requests' newest behaviours ``new_events``
        ([R, dL, 64] features or [R, dL] ids) are appended to sequence ``seq_name`` and only the new
        S tokens are computed, their queries attending over the cached K/V (ot_attn_fwd_cached).

        Exact (equal to encode_requests on the extended sequences) when the appended tokens land at
        the end of the S side and shift nothing: ``seq_name`` must be the last configured sequence
        (no [SEP] follows it, model.py:270-272) and present in the requests, and no layer before the
        last may prune (a pyramid keep would move with the length).  Weight groups are functions of the
        absolute position, which the old tokens keep."""
        from .model import _Tokenize
        m = self.m
        cfg = m.config
        d, H = cfg.hidden_dim, cfg.num_heads
        hd = d // H
        seqs = cfg.feature_config['sequence_features']
        if seq_name != seqs[-1] or seq_name not in cache.present:
            raise ValueError(f'extend_requests: only the last configured sequence ({seqs[-1]!r}), present in the '
                             'cached requests, can grow without shifting earlier positions')
        old = self.schedule(cache.L_S)
        if any(e['kS'] + e['kN'] < e['I'] for e in old[:-1]):
            raise ValueError('extend_requests: a pyramid keep before the last layer depends on the length; '
                             're-encode instead')
        R = cache.R
        plan = m._plan({}, {seq_name: new_events})
        if plan['B'] != R:
            raise ValueError(f'extend_requests: {plan["B"]} rows of new events for {R} cached requests')
        dL = plan['L_S']
        x0 = _Tokenize.apply(m.flat, m, plan)                             # [R*(dL+L_NS), d], no [SEP]
        x = x0.view(R, dL + cfg.num_ns_tokens, d)[:, :dL].reshape(R * dL, d)
        new = self.schedule(cache.L_S + dL)
        req = torch.arange(R, dtype=torch.int32, device=x.device)
        layers = []
        for l, (e_old, e_new) in enumerate(zip(old, new)):
            Ic = e_old['s']
            lay = cache.layers[l]
            keep = e_new['kS'] - e_old['kS']                              # new S rows kept by this layer

            def attn(qkv, Ic=Ic, lay=lay):
                o = torch.empty(R * dL, d, device=qkv.device)
                kv = (lay['kv'], d) if Ic > 0 else None
                K.attn_fwd_cached(qkv, 3 * d, kv, 3 * d, req, R, H, Ic, dL, dL, hd, o)
                return o

            x, qkv = self._block(l, x, R, dL, dL if keep == dL else 0, Ic, e_new['I'], attn)
            kv = qkv if Ic == 0 else torch.cat([lay['kv'].view(R, Ic, 3 * d), qkv.view(R, dL, 3 * d)], 1)
            layers.append({'Ic': Ic + dL, 'kv': kv.reshape(R * (Ic + dL), 3 * d)})
        return RequestCache(R, cache.L_S + dL, layers, cache.present)

    # ------------------------------------------------------------------ stage II
    @torch.no_grad()
    @K.in_model_precision
    def score(self, cache: RequestCache, req: torch.Tensor, non_seq_features: Dict[str, torch.Tensor]):
        """Candidates' NS tokens (model.py:239-254) through every layer against their request's cache;
        returns {task: probs [C, 1]} like ``OneTransModel.forward`` (model.py:384-391)."""
        from .model import _Head, _Tokenize
        m = self.m
        cfg = m.config
        d, H = cfg.hidden_dim, cfg.num_heads
        hd = d // H
        dev = m.device
        plan = m._plan(non_seq_features, {})
        C = plan['B']
        req = torch.as_tensor(req)
        if req.numel() != C:
            raise ValueError(f'score: {req.numel()} request indices for {C} candidates')
        # the cached-attention kernel indexes the K/V cache with req unchecked: validate before launch
        # (host indices directly; device indices with one min/max read-back)
        lo, hi = (int(v) for v in torch.aminmax(req.reshape(-1).to(torch.int64)))
        if lo < 0 or hi >= cache.R:
            raise ValueError(f'score: request index out of range [0, {cache.R}) (min {lo}, max {hi})')
        req = req.to(dev, torch.int32).contiguous()
        x = _Tokenize.apply(m.flat, m, plan)                              # [C*L_NS, d]: NS tokens only
        for l, e in enumerate(self.schedule(cache.L_S)):
            s, n, kN = e['s'], e['n'], e['kN']
            lay = cache.layers[l]
            if lay['Ic'] != s:
                raise OneTransHipError('score: request cache does not match the schedule')

            def attn(qkv, lay=lay, s=s, n=n, kN=kN):
                o = torch.empty(C * kN, d, device=dev)
                kv = (lay['kv'], d) if s > 0 else None
                K.attn_fwd_cached(qkv, 3 * d, kv, 3 * d, req, C, H, s, n, kN, hd, o)
                return o

            x, _ = self._block(l, x, C, n, kN, s, e['I'], attn)
        probs, _ = _Head.apply(m.flat, x, m)                               # [T, C]
        return {t: probs[i].view(-1, 1) for i, t in enumerate(cfg.tasks)}

    @torch.no_grad()
    @K.in_model_precision
    def predict(self, non_seq_features, seq_features, req: Optional[torch.Tensor] = None):
        """One call: ``seq_features`` hold R requests, ``non_seq_features`` C candidates, ``req`` [C] maps
        candidates to requests (default: candidate i belongs to request i, R == C)."""
        cache = self.encode_requests(seq_features)
        if req is None:
            req = torch.arange(cache.R, dtype=torch.int32)
        return self.score(cache, req, non_seq_features)


class OneTransInferenceEngine:
    """The reference's inference engine surface (examples/inference_example.py:21-219): load a saved
    model directory (config.json + weights, train.py:281-291), preprocess, single / batch inference,
    latency statistics.  ``score_candidates`` adds the two-stage path: one user's sequences once,
    many candidates against the cache."""

    def __init__(self, model_path: str, device=None):
        import json
        import os
        from .config import OneTransConfig
        from .model import OneTransModel
        cfg_path = os.path.join(model_path, 'config.json')
        if not os.path.exists(cfg_path):                                  # inference_example.py:44-45
            raise FileNotFoundError(f'config file not found: {cfg_path}')
        with open(cfg_path) as f:
            self.config = OneTransConfig.from_dict(json.load(f))
        w = os.path.join(model_path, 'model_weights.npz')
        if not os.path.exists(w):                                          # inference_example.py:55-56
            raise FileNotFoundError(f'model weights not found: {w}')
        self.model = OneTransModel(self.config, device=device)
        self.model.load_weights(w)
        self.server = OneTransServer(self.model)
        self.reset_stats()

    # ------------------------------------------------------------------ inference_example.py:63-92
    def preprocess_input(self, user_features: Dict, item_features: Dict, context_features: Dict,
                         sequence_features: Dict):
        from .features import SequenceProcessor
        import numpy as np
        non_seq = {}
        non_seq.update(user_features)
        non_seq.update(item_features)
        non_seq.update(context_features)
        sp = SequenceProcessor(self.config)
        seq = {k: sp.process_sequence(np.asarray(v)) for k, v in sequence_features.items()}
        return non_seq, seq

    def _predict(self, non_seq, seq):
        import numpy as np
        dev = self.model.device
        ns = {k: torch.as_tensor(np.asarray(v)).reshape(-1, 1).to(dev) for k, v in non_seq.items()}
        sq = {k: torch.as_tensor(np.asarray(v)).to(dev) for k, v in seq.items()}
        with torch.no_grad():
            out = self.model((ns, sq), training=False)
        return {t: p.float().cpu().numpy()[:, 0] for t, p in out.items()}

    def single_inference(self, user_features, item_features, context_features, sequence_features) -> Dict[str, float]:
        """inference_example.py:94-129."""
        import time
        t0 = time.time()
        try:
            ns, seq = self.preprocess_input(user_features, item_features, context_features, sequence_features)
            seq = {k: v[None] for k, v in seq.items()}                     # batch dimension
            res = {t: float(v[0]) for t, v in self._predict(ns, seq).items()}
            self._update_stats(True, (time.time() - t0) * 1e3)
            return res
        except Exception:
            self._update_stats(False, 0.0)
            raise

    def batch_inference(self, batch_data) -> List[Dict[str, float]]:
        """inference_example.py:131-179: (user, item, context, sequences) tuples, one full forward."""
        import time
        import numpy as np
        t0 = time.time()
        try:
            pre = [self.preprocess_input(*b) for b in batch_data]
            ns = {k: np.concatenate([np.asarray(p[0][k]).reshape(-1) for p in pre]) for k in pre[0][0]}
            seq = {k: np.stack([p[1][k] for p in pre]) for k in pre[0][1]}
            out = self._predict(ns, seq)
            n = len(batch_data)
            self._update_stats(True, (time.time() - t0) * 1e3 / n, n)
            return [{t: float(v[i]) for t, v in out.items()} for i in range(n)]
        except Exception:
            self._update_stats(False, 0.0, len(batch_data))
            raise

    def score_candidates(self, user_features: Dict, sequence_features: Dict, candidates: List[Dict]):
        """One request (user + sequences), many candidates (item / context features each): stage I once,
        stage II for all candidates (paper §3.5.1).  Same results as ``batch_inference`` on the
        (user, candidate, sequences) samples."""
        import numpy as np
        dev = self.model.device
        _, seq = self.preprocess_input({}, {}, {}, sequence_features)
        cache = self.server.encode_requests({k: torch.as_tensor(v[None]).to(dev) for k, v in seq.items()})
        ns = {}
        for k, v in user_features.items():
            ns[k] = np.repeat(np.asarray(v).reshape(-1)[:1], len(candidates))
        for k in candidates[0]:
            ns[k] = np.concatenate([np.asarray(c[k]).reshape(-1) for c in candidates])
        nsd = {k: torch.as_tensor(v).reshape(-1, 1).to(dev) for k, v in ns.items()}
        out = self.server.score(cache, torch.zeros(len(candidates), dtype=torch.int32), nsd)
        return [{t: float(p[i, 0]) for t, p in out.items()} for i in range(len(candidates))]

    # ------------------------------------------------------------------ inference_example.py:181-219
    def _update_stats(self, success: bool, latency: float, batch_size: int = 1):
        st = self.inference_stats
        st['total_requests'] += batch_size
        if success:
            st['successful_requests'] += batch_size
            st['avg_latency_ms'] = 0.1 * latency + 0.9 * st['avg_latency_ms']      # EMA, alpha 0.1
        else:
            st['failed_requests'] += batch_size

    def get_stats(self) -> Dict:
        st = dict(self.inference_stats)
        st['success_rate'] = (st['successful_requests'] / st['total_requests'] * 100
                              if st['successful_requests'] > 0 else 0.0)
        return st

    def reset_stats(self):
        self.inference_stats = {'total_requests': 0, 'avg_latency_ms': 0.0, 'successful_requests': 0,
                                'failed_requests': 0}
