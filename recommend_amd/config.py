"""OneTrans configuration — mirrors the reference's ``practice/config.py``.

Reference: ``rank/scaling_up/oneTrans/practice/config.py:9-121``.  The attribute
names, defaults, ``to_dict``/``from_dict`` and the small/default/large presets are
kept so a reference ``config.json`` (written by ``train.py:289-291``) loads
unchanged.  Build-only knobs (marked ``# build``) select between the reference's
literal semantics and the fixes recorded in DESIGN.md §Semantics:

* ``dedicated_positions`` — ``'head'`` reproduces ``model.py:69,155`` (positions
  ``< num_ns_tokens`` get the dedicated weights, i.e. the first tokens, which are
  S-tokens because the tokenizer concatenates ``[S; NS]`` at ``model.py:235``);
  ``'tail'`` gives them to the last ``num_ns_tokens`` tokens (paper eq. 12).
* ``pyramid_fix`` — the reference computes pyramid query indices against the
  *original* length (``model.py:293-296,343,349``) which is out of range from
  layer 1 on; the fix indexes against the current length ``I_l`` and caps
  ``keep_l`` at ``I_l``.  With the fix off, an out-of-range schedule raises
  ``IndexError`` (TF's CPU behaviour for the same gather).
* ``pyramid_select`` — which queries a pyramid layer keeps.  ``'tail'`` is the
  reference's static tail slice (``model.py:296, 371``); ``'norm'`` (build
  extension) keeps the NS tokens plus the S tokens of largest RMS (top-K per
  sample, ``ot_pyramid_select``), which needs ``dedicated_positions='tail'`` so
  the dedicated (NS) rows stay at fixed places.  Both run the same wavefront
  top-K kernel; 'tail' passes no score, so the position tie-break picks the tail.
* ``sparse_features`` / ``seq_item_vocab`` — the Criteo-shape embedding-gather
  extension (north_star): NS features named here carry int64 ids looked up in a
  per-field table of width ``ns_embedding_dim``; sequence features carry int64
  item ids looked up in one ``[seq_item_vocab, seq_feature_dim]`` table.
"""

from __future__ import annotations

import copy
import math
from typing import Dict, List, Optional


class OneTransConfig:
    """Same attribute surface as the reference ``OneTransConfig`` (config.py:9-69)."""

    def __init__(self):
        # model architecture (config.py:14-18)
        self.hidden_dim = 384
        self.num_layers = 8
        self.num_heads = 4
        self.ffn_dim = 1536
        # inputs (config.py:20-23)
        self.max_seq_len = 2048
        self.num_ns_tokens = 12
        self.sep_token_id = 0
        # mixed parameterisation (config.py:25-27)
        self.shared_s_params = True
        self.dedicated_ns_params = True
        # pyramid (config.py:29-31)
        self.pyramid_enabled = True
        self.pyramid_ratios = [0.5, 0.3, 0.2, 0.1, 0.05, 0.03, 0.02, 0.01]
        # training (config.py:33-37)
        self.batch_size = 2048
        self.learning_rate = 0.005
        self.num_epochs = 100
        self.warmup_steps = 10000
        # optimiser (config.py:39-48)
        self.optimizer_config = {
            'dense_optimizer': 'rmsprop',
            'sparse_optimizer': 'adagrad',
            'dense_lr': 0.005,
            'sparse_lr': 0.1,
            'beta1': 0.1,
            'beta2': 1.0,
            'momentum': 0.99999,
        }
        # regularisation (config.py:50-53)
        self.dropout_rate = 0.1
        self.weight_decay = 0.0
        self.gradient_clip_norm = 90.0
        # features (config.py:55-61)
        self.feature_config = {
            'user_features': ['user_id', 'age', 'gender', 'location'],
            'item_features': ['item_id', 'category', 'price', 'brand'],
            'context_features': ['time', 'device', 'platform'],
            'sequence_features': ['click_seq', 'cart_seq', 'purchase_seq'],
        }
        # tasks (config.py:63-64)
        self.tasks = ['ctr', 'cvr']
        # system flags (config.py:66-70)
        self.use_mixed_precision = True
        self.use_kv_cache = True
        self.use_flash_attention = True
        self.use_activation_recompute = True

        # ---- build knobs (not in the reference) ----
        self.dedicated_positions = 'head'    # build: 'head' (ref model.py:69) | 'tail' (paper eq.12)
        self.pyramid_fix = True              # build: index pyramid against the current length
        self.pyramid_select = 'tail'         # build: 'tail' (ref model.py:296) | 'norm' (top-K by token RMS)
        self.seq_feature_dim = 64            # build: width of one sequence event (data_loader.py:146,322)
        self.ns_embedding_dim = 16           # build: per-field NS embedding width (Criteo shape)
        self.sparse_features: Dict[str, int] = {}   # build: NS id features -> cardinality
        self.seq_item_vocab = 0              # build: >0 => sequence features are item ids
        self.compute_dtype = 'fp32'          # build: arithmetic of the HIP path (reference is fp32)
        # build: the behaviour behind two reference flags the reference itself never reads
        # (use_activation_recompute config.py:69, warmup_steps config.py:36), opt-in so default numerics and
        # memory match the reference: recompute each block's forward in its backward (keep only the block
        # input), and a linear warm-up of the dense LR over warmup_steps
        self.recompute_blocks = False
        self.apply_warmup = False
        self.sparse_clip_norm = 120.0        # build: paper clip for sparse grads (complete_translation.md:190)
        self.adagrad_initial_accumulator = 0.1   # build: Keras Adagrad default
        self.adagrad_epsilon = 1e-7              # build: Keras Adagrad default
        self.rmsprop_rho = 0.9                   # build: Keras RMSprop default (train.py:66 reads rho default)
        self.rmsprop_epsilon = 1e-7              # build: Keras RMSprop default (train.py:68)

    # ------------------------------------------------------------------ helpers
    def to_dict(self) -> Dict:
        """config.py:71-73."""
        return {k: copy.deepcopy(v) for k, v in self.__dict__.items() if not k.startswith('_')}

    @classmethod
    def from_dict(cls, config_dict: Dict) -> 'OneTransConfig':
        """config.py:75-82: unknown keys are ignored, known keys overwrite."""
        config = cls()
        for key, value in config_dict.items():
            if hasattr(config, key):
                setattr(config, key, copy.deepcopy(value))
        return config

    # derived quantities -------------------------------------------------------
    @property
    def head_dim(self) -> int:
        return self.hidden_dim // self.num_heads

    @property
    def num_groups(self) -> int:
        """Weight groups of the mixed parameterisation: 0 = shared, 1..L_NS = dedicated."""
        return 1 + self.num_ns_tokens

    def ns_feature_names(self) -> List[str]:
        """Concat order of NS features (model.py:243-247)."""
        fc = self.feature_config
        return list(fc['user_features']) + list(fc['item_features']) + list(fc['context_features'])

    def ns_input_width(self, present: Optional[List[str]] = None) -> int:
        """F_ns: 1 per dense feature, ns_embedding_dim per sparse-id feature."""
        names = self.ns_feature_names() if present is None else present
        return sum(self.ns_embedding_dim if n in self.sparse_features else 1 for n in names)

    def seq_token_count(self, seq_lens: List[int]) -> int:
        """L_S = sum(L_i) + one [SEP] after every present sequence i < n-1 (model.py:266-272)."""
        n = len(self.feature_config['sequence_features'])
        return int(sum(seq_lens)) + max(0, n - 1) if len(seq_lens) == n else None

    def pyramid_schedule(self, total_seq_len: int) -> List[Dict]:
        """Per layer (in_len I_l, keep K_l).  Follows PyramidScheduler.get_layer_config
        (model.py:287-302) with the D2 fix: keep_l = max(1, int(L0*ratio_l)) capped at I_l and
        the kept queries are the tail of the *current* sequence.  The last layer keeps
        exactly 1 token downstream (only output_tokens[:, -1] is read at model.py:390),
        which is recorded as ``needed`` (dead-code elimination, exact)."""
        sched = []
        cur = total_seq_len
        for l in range(self.num_layers):
            if self.pyramid_enabled and l < len(self.pyramid_ratios):
                keep = max(1, int(total_seq_len * self.pyramid_ratios[l]))
                if self.pyramid_fix:
                    keep = min(keep, cur)
                elif total_seq_len > cur:
                    # reference gathers range(L0-keep, L0) from a tensor of length cur < L0
                    raise IndexError('pyramid gather out of range (reference defect D2)')
            else:
                keep = cur
            sched.append({'in_len': cur, 'keep': keep})
            cur = keep
        # the model reads only the last token of the final layer
        for l, s in enumerate(sched):
            s['needed'] = s['keep'] if l < len(sched) - 1 else 1
        return sched

    def group_of_position(self, p: int, in_len: int) -> int:
        """Weight group for position p of a layer whose input has in_len tokens.
        'head': model.py:69 (`idx < num_ns_tokens` -> dedicated[idx]); 'tail': paper eq. 12."""
        if self.dedicated_positions == 'head':
            return 1 + p if p < self.num_ns_tokens else 0
        if self.dedicated_positions == 'tail':
            j = p - (in_len - self.num_ns_tokens)
            return 1 + j if j >= 0 else 0
        raise ValueError(f'unknown dedicated_positions {self.dedicated_positions!r}')


class OneTransSmallConfig(OneTransConfig):
    """config.py:85-92."""

    def __init__(self):
        super().__init__()
        self.hidden_dim = 256
        self.num_layers = 6
        self.ffn_dim = 1024


class OneTransLargeConfig(OneTransConfig):
    """config.py:95-103."""

    def __init__(self):
        super().__init__()
        self.hidden_dim = 512
        self.num_layers = 12
        self.num_heads = 8
        self.ffn_dim = 2048


def get_model_config(model_type: str = 'default') -> OneTransConfig:
    """config.py:106-117: ValueError on an unknown preset (same as the reference)."""
    config_map = {
        'small': OneTransSmallConfig,
        'default': OneTransConfig,
        'large': OneTransLargeConfig,
    }
    if model_type not in config_map:
        raise ValueError(f"unknown model type: {model_type}")
    return config_map[model_type]()


DEFAULT_CONFIG = OneTransConfig()

# ---------------------------------------------------------------------------
# BASELINE.json workloads.  B and L_NS values not fixed by
# BASELINE.json are builder choices, reported in DESIGN.md.
# ---------------------------------------------------------------------------

# 26 Criteo-like categorical fields, cardinalities log-spaced 1e3 .. 1e7
CRITEO_CARDINALITIES = [int(round(10 ** (3 + 4 * i / 25))) for i in range(26)]


def _criteo_features(cfg: OneTransConfig, seq_lens: List[int], item_vocab: int) -> None:
    dense = [f'I{i}' for i in range(1, 14)]
    sparse = [f'C{i}' for i in range(1, 27)]
    cfg.feature_config = {
        'user_features': sparse[:13],
        'item_features': sparse[13:],
        'context_features': dense,
        'sequence_features': ['click_seq', 'cart_seq', 'purchase_seq'],
    }
    cfg.sparse_features = {name: card for name, card in zip(sparse, CRITEO_CARDINALITIES)}
    cfg.seq_item_vocab = item_vocab
    cfg._seq_lens = list(seq_lens)


def check_pyramid_select(cfg: OneTransConfig) -> None:
    """``pyramid_select`` is 'tail' (reference) or 'norm' (needs the NS tokens at the dedicated tail)."""
    sel = getattr(cfg, 'pyramid_select', 'tail')
    if sel not in ('tail', 'norm'):
        raise ValueError(f'unknown pyramid_select {sel!r}')
    if sel == 'norm' and cfg.dedicated_positions != 'tail':
        raise ValueError("pyramid_select='norm' needs dedicated_positions='tail' (the kept NS rows keep their "
                         "dedicated weights)")


def workload_config(name: str) -> OneTransConfig:
    """Configs of BASELINE.json as OneTransConfig objects; ``cfg._seq_lens`` and
    ``cfg._batch`` carry the synthetic input shape."""
    cfg = OneTransConfig()
    cfg.pyramid_enabled = False
    name = name.upper()
    if name == 'C1':     # 2L d64, 8 NS + 32 S tokens, B512, reference-literal features
        cfg.hidden_dim, cfg.num_layers, cfg.num_heads, cfg.ffn_dim = 64, 2, 4, 256
        cfg.num_ns_tokens = 8
        cfg._seq_lens = [10, 10, 10]
        cfg._batch = 512
    elif name in ('C2', 'T'):   # 4L d128 (T: d256), L_NS 12, L_S 128 = 42*3+2, B4096
        d = 128 if name == 'C2' else 256
        cfg.hidden_dim, cfg.num_layers, cfg.num_heads, cfg.ffn_dim = d, 4, 4, 4 * d
        cfg.num_ns_tokens = 12
        _criteo_features(cfg, [42, 42, 42], 1_000_000)
        cfg._batch = 4096
    elif name == 'C3':   # 6L d256, L_S 512 = 170*3+2, pyramid 0.5/layer, B2048
        cfg.hidden_dim, cfg.num_layers, cfg.num_heads, cfg.ffn_dim = 256, 6, 4, 1024
        cfg.num_ns_tokens = 12
        cfg.pyramid_enabled = True
        cfg.pyramid_ratios = [0.5 ** (l + 1) for l in range(6)]
        _criteo_features(cfg, [170, 170, 170], 1_000_000)
        cfg._batch = 2048
    elif name == 'C4':   # 8L d256, L0 140, B2048/GPU, 100M-row item table row-sharded
        cfg.hidden_dim, cfg.num_layers, cfg.num_heads, cfg.ffn_dim = 256, 8, 4, 1024
        cfg.num_ns_tokens = 12
        _criteo_features(cfg, [42, 42, 42], 100_000_000)
        cfg._batch = 2048
    elif name == 'C5':   # 12L d512 H8, L_S 1024 = 341+341+340+2, B512/GPU
        cfg.hidden_dim, cfg.num_layers, cfg.num_heads, cfg.ffn_dim = 512, 12, 8, 2048
        cfg.num_ns_tokens = 12
        _criteo_features(cfg, [341, 341, 340], 1_000_000)
        cfg._batch = 512
    else:
        raise ValueError(f'unknown workload {name!r}')
    return cfg


def algorithmic_flops_per_sample(cfg: OneTransConfig, seq_lens: List[int], f_ns: int) -> Dict[str, float]:
    """SURVEY §8d exact minimal work (fwd), counting tail-only queries and the
    single needed query of the final layer.  fwd+bwd = 3 x fwd."""
    d, f = cfg.hidden_dim, cfg.ffn_dim
    L_S = cfg.seq_token_count(seq_lens)
    L0 = L_S + cfg.num_ns_tokens
    sched = cfg.pyramid_schedule(L0)
    attn = layers = 0.0
    for s in sched:
        I, K = s['in_len'], s['needed']
        P = K * I - K * (K - 1) / 2.0
        a = 4.0 * P * d
        attn += a
        layers += 4.0 * I * d * d + 2.0 * K * d * d + a + 2.0 * K * d * d + 4.0 * K * d * f
    tok = 2.0 * sum(seq_lens) * cfg.seq_feature_dim * d + 2.0 * f_ns * cfg.num_ns_tokens * d
    heads = len(cfg.tasks) * (2.0 * d * (d // 2) + 2.0 * (d // 2))
    fwd = layers + tok + heads
    return {'fwd': fwd, 'fwd_bwd': 3.0 * fwd, 'attn_fwd': attn}


__all__ = ['OneTransConfig', 'OneTransSmallConfig', 'OneTransLargeConfig', 'get_model_config',
           'DEFAULT_CONFIG', 'workload_config', 'algorithmic_flops_per_sample',
           'CRITEO_CARDINALITIES']
