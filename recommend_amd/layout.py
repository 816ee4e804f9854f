"""Device data layout: the flat dense-parameter buffer and the row maps of the grouped GEMMs.

HBM layout:

* every dense parameter bank of ``params.dense_param_shapes`` lives in ONE flat fp32 buffer
  (bank offsets 64-float aligned); gradients and the RMSprop state (v, m) are flat buffers
  of the same layout, so the optimizer is one multi-segment launch and the DP all-reduce is
  one contiguous buffer.
* activations are token-major ``[B * I, width]`` (row = b * I + p); a layer that keeps only
  its last K tokens writes compact ``[B * K, width]`` rows (row = b * K + j).
* a *row map* lists, tile by tile (128 rows per tile), which rows a grouped GEMM reads and
  writes; every tile belongs to one weight group (mixed parameterisation, model.py:67-74).
  Padding entries are -1.
"""

from __future__ import annotations

import os
from typing import Callable, Dict, List, Sequence, Tuple

import numpy as np

from .config import OneTransConfig
from .params import dense_param_shapes, keras_variables

TILE = 128
ALIGN = 64
IMAGE_UNIT_ELEMS = 3 * TILE * 16      # one (group, column tile, 16-k stage) block of a B image (bf16)
# wgrad workgroups per launch (chunk sizing), by output tiles per chunk.  Small weights (< 8 tiles:
# all of C2's) are capped at one round of the split kernel's 512 resident workgroups -- a count just
# past a multiple of 512 (e.g. 513) leaves a nearly empty extra round; capped, the C2 GEMM family
# measured 332 -> 316 us/launch standalone.  Weights of >= 8 tiles (d >= 256) take ~3 rounds plus one
# chunk per weight group (C5 +5-7%, T +2% over 768; a hard cap measured worse there).  Weights of >= 32
# tiles (d = 512: C5's) take 4096 since the kernels place whole chunks per XCD (round 4, gemm.hip
# wgrad_tile): shorter chunks keep a chunk's tiles closer together in the rows they stream, so more of the
# shared rows hit the XCD's L2 (C5 1,425 / 1,438 / 1,463 / 1,466 samples/s at 1536 / 3072 / 4096 / 6144 on one
# box; T, C3, C4 flat or -1% at 3072, so they keep 1536).  Tuning override ONETRANS_WGRAD_SLOTS (every case);
# tools/wgrad_probe.py sweeps it.
_SLOTS_ENV = os.environ.get('ONETRANS_WGRAD_SLOTS')
WGRAD_SLOTS = int(_SLOTS_ENV) if _SLOTS_ENV else 1536
WGRAD_SLOTS_SMALL = int(_SLOTS_ENV) if _SLOTS_ENV else 512
WGRAD_SLOTS_LARGE = int(_SLOTS_ENV) if _SLOTS_ENV else 4096


def wgrad_slots(tiles_per_chunk: int) -> int:
    if tiles_per_chunk >= 32:
        return WGRAD_SLOTS_LARGE
    return WGRAD_SLOTS if tiles_per_chunk >= 8 else WGRAD_SLOTS_SMALL


def round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


class FlatLayout:
    """Offsets of every dense bank inside the flat parameter buffer."""

    def __init__(self, cfg: OneTransConfig, f_ns: int, pair_dgrad: bool = False):
        self.f_ns = f_ns
        self.f_pad = max(4, round_up(f_ns, 4))
        self.shapes = dense_param_shapes(cfg, self.f_pad)
        self.offsets: Dict[str, int] = {}
        off = 0
        for name, shp in self.shapes.items():
            self.offsets[name] = off
            off += round_up(int(np.prod(shp)), ALIGN)
        self.total = off
        segs = []
        for (bank, eoff, rows, cols, stride) in keras_variables(cfg, self.shapes, f_ns=f_ns):
            segs.append((self.offsets[bank] + eoff, rows, cols, stride))
        self.segments = np.array(segs, dtype=np.int64)
        self.max_seg_elems = int((self.segments[:, 1] * self.segments[:, 2]).max())
        # GEMM weight banks (Keras [G][K][N]) kept transposed ([G][N][K]) in a shadow buffer for the
        # forward GEMMs: name -> (G, K, N)
        d, f, T = cfg.hidden_dim, cfg.ffn_dim, len(cfg.tasks)
        nseq = len(cfg.feature_config['sequence_features'])
        self.gemm_banks = {'tok.ns.kernel': (1, self.f_pad, cfg.num_ns_tokens * d),
                           'tok.seq.kernel': (nseq, cfg.seq_feature_dim, d),
                           'head.w1': (T, d, d // 2)}
        for l in range(cfg.num_layers):
            G = cfg.num_groups
            self.gemm_banks.update({f'blk.{l}.wqkv': (G, d, 3 * d), f'blk.{l}.wo': (1, d, d),
                                    f'blk.{l}.w1': (G, d, f), f'blk.{l}.w2': (G, f, d)})
        recs, tiles = [], 0
        for name, (G, K, N) in self.gemm_banks.items():
            o = self.offsets[name]
            recs.append((o, o, G, K, N, tiles))
            tiles += G * ((K + 31) // 32) * ((N + 31) // 32)
        self.transpose_desc = np.array(recs, dtype=np.int64)
        self.transpose_tiles = tiles
        # pre-split B images of the plane GEMM (ot_split_images), per bank and orientation:
        # 'fwd' (B = W^T, k = the Keras input dim; the RMSNorm gamma in front of wqkv / w1 folded in)
        # and 'dgrad' (B = W); only where the GEMM has whole 128-column tiles and 16-k stages
        self.images: Dict[Tuple[str, str], Tuple[int, int, int, int]] = {}   # -> (offset, G, N, K)
        irecs, units, ioff = [], 0, 0
        # images written in the scaled-fp16-pair form in split mode (gamma-folded, kscale >= 0, and the FFN2 W2
        # forward image, kscale -2): the plane GEMM reads them with three f16 products only
        self.pair_images = set()
        for name, (G, K, N) in self.gemm_banks.items():
            o = self.offsets[name]
            gamma = None
            if name.endswith('.wqkv'):
                gamma = self.offsets[name[:-len('wqkv')] + 'norm1']
            elif name.endswith('.w1') and name.startswith('blk.'):
                gamma = self.offsets[name[:-len('w1')] + 'norm2']
            for orient, (Nb, Kb, sn, sk) in (('fwd', (N, K, 1, N)), ('dgrad', (K, N, N, 1))):
                if Nb % TILE or Kb % 16:
                    continue
                nu = G * (Nb // TILE) * (Kb // 16)
                # -2: the FFN2 forward's W2 image in the scaled-fp16-pair form (split mode: the GEMM reads U's row
                # maxima from the FFN1 epilogue, ot_rms_epilogue.a_rowmax); gamma-folded images are pairs too
                # (only when W1's forward image exists too, f % 128 == 0 and d % 16 == 0: the FFN1 forward then runs on
                # the plane GEMM, whose epilogue writes those maxima — OneTransModel allocates them under pair_form())
                pair_w2 = (orient == 'fwd' and name.endswith('.w2') and name.startswith('blk.')
                           and K % TILE == 0 and N % 16 == 0)
                # pair_dgrad: the FFN2 / FFN1 / Wo dgrad images too (their A operands' row maxima come from the
                # producers: ot_dropout_apply_ex / rowabs_out, or ot_rows_absmax)
                # (and the Wo forward image: its A, the attention output, gets row maxima from the attention forward)
                pair_dg = pair_dgrad and name.startswith('blk.') and (
                    (orient == 'dgrad' and name.endswith(('.w1', '.w2', '.wo', '.wqkv')))
                    or (orient == 'fwd' and name.endswith('.wo')))
                kscale = gamma if (orient == 'fwd' and gamma is not None) else (-2 if (pair_w2 or pair_dg) else -1)
                irecs.append((o, sn, sk, K * N, kscale, ioff, units, G, Nb, Kb))
                self.images[(name, orient)] = (ioff, G, Nb, Kb)
                if kscale != -1:
                    self.pair_images.add((name, orient))
                units += nu
                ioff += nu * IMAGE_UNIT_ELEMS
        self.image_desc = np.array(irecs, dtype=np.int64).reshape(-1, 10)
        self.image_units = units
        self.image_elems = ioff

    def tview(self, flatT, name):
        """Transposed bank [G][N][K] inside the shadow buffer (1-D view)."""
        off = self.offsets[name]
        G, K, N = self.gemm_banks[name]
        return flatT[off:off + G * K * N]

    def view(self, flat, name):
        off = self.offsets[name]
        n = int(np.prod(self.shapes[name]))
        return flat[off:off + n].view(self.shapes[name])


class RowMap:
    """Tiles of a grouped GEMM: ``rows[k]`` (one int32 array per index space, length
    ntiles*TILE, -1 padded), ``tile_group`` [ntiles], and wgrad chunks {group, begin, count}
    with ``gchunk`` [G, 2] {first chunk, n chunks}."""

    def __init__(self, rows: List[np.ndarray], tile_group: np.ndarray, chunks: np.ndarray,
                 gchunk: np.ndarray, nrows: int, group_rows=None):
        self.group_rows = list(group_rows) if group_rows is not None else []
        self._chunk_cache = {}
        self.rows = rows
        self.tile_group = tile_group
        self.chunks = chunks
        self.gchunk = gchunk
        self.ntiles = len(tile_group)
        self.nrows = nrows              # real (unpadded) rows
        self.dev = None

    def to(self, device):
        import torch
        if self.dev is None:
            self.dev = {
                'rows': [torch.from_numpy(r).to(device) for r in self.rows],
                'tile_group': torch.from_numpy(self.tile_group).to(device),
                'chunks': torch.from_numpy(self.chunks).to(device),
                'gchunk': torch.from_numpy(self.gchunk).to(device),
            }
        return self.dev

    def chunks_for(self, tiles_per_chunk: int, device):
        """wgrad chunk table whose workgroup count (chunks x output tiles) stays within
        wgrad_slots(tiles_per_chunk): the smallest chunk size (multiple of 32 rows) that does.  Returns (chunks_dev, gchunk_dev, nchunks)."""
        import torch
        key = (tiles_per_chunk, str(device))
        if key not in self._chunk_cache:
            padded = [round_up(n, TILE) for n in self.group_rows]
            # every nonempty group needs a chunk of its own: on top of them, the budget of one round
            # (with as many groups as budget slots -- C5's 13 groups x 64 output tiles -- a budget of
            # one round would leave the shared group a single chunk, 64 workgroups on 256 CUs)
            ng = sum(1 for p in padded if p > 0)
            if tiles_per_chunk < 8:       # hard cap: chunks x tiles within the slots (groups floor aside)
                budget = max(ng, wgrad_slots(tiles_per_chunk) // max(1, tiles_per_chunk))
            else:
                budget = max(1, wgrad_slots(tiles_per_chunk) // max(1, tiles_per_chunk)) + ng
            lo, hi = 32, max(32, round_up(max(padded) if padded else 32, 32))
            while lo < hi:
                mid = round_up((lo + hi) // 2, 32)
                if mid >= hi:
                    mid = hi - 32 if hi - 32 >= lo else lo
                n = sum((p + mid - 1) // mid for p in padded if p > 0)
                if n <= budget:
                    hi = mid
                else:
                    lo = mid + 32
            cr = lo
            chunks, gchunk, base = [], [], 0
            for g, p in enumerate(padded):
                first = len(chunks)
                for c0 in range(0, p, cr):
                    chunks.append((g, base + c0, min(cr, p - c0)))
                gchunk.append((first, len(chunks) - first))
                base += p
            ch = np.array(chunks, dtype=np.int32).reshape(-1, 3)
            gc = np.array(gchunk, dtype=np.int32).reshape(-1, 2)
            self._chunk_cache[key] = (torch.from_numpy(ch).to(device), torch.from_numpy(gc).to(device), len(ch))
        return self._chunk_cache[key]


def build_map(per_group: Sequence[Sequence[np.ndarray]], chunk_rows: int = 0) -> RowMap:
    """``per_group[g]`` = list (one per index space) of equal-length int arrays of rows of group g.
    Each group is padded to a multiple of TILE; wgrad chunks split each group into runs of
    ``chunk_rows`` (a multiple of TILE; 0 = auto, ~256 chunks overall)."""
    G = len(per_group)
    nspace = len(per_group[0]) if G else 0
    total = sum(len(pg[0]) for pg in per_group)
    if chunk_rows <= 0:
        chunk_rows = max(4 * TILE, round_up(max(1, total // 256), TILE))
    rows = [[] for _ in range(nspace)]
    tile_group, chunks, gchunk = [], [], []
    base = 0
    for g, pg in enumerate(per_group):
        n = len(pg[0])
        npad = round_up(n, TILE)
        for s in range(nspace):
            r = np.full(npad, -1, dtype=np.int32)
            r[:n] = pg[s]
            rows[s].append(r)
        tile_group.extend([g] * (npad // TILE))
        first = len(chunks)
        for c0 in range(0, npad, chunk_rows):
            chunks.append((g, base + c0, min(chunk_rows, npad - c0)))
        gchunk.append((first, len(chunks) - first))
        base += npad
    cat = [np.concatenate(r) if r else np.zeros(0, np.int32) for r in rows]
    return RowMap(cat, np.array(tile_group, dtype=np.int32),
                  np.array(chunks, dtype=np.int32).reshape(-1, 3),
                  np.array(gchunk, dtype=np.int32).reshape(-1, 2), total,
                  group_rows=[len(pg[0]) for pg in per_group])


def layer_maps(cfg: OneTransConfig, B: int, I: int, K: int, p0: int = 0,
               I_full: int = 0) -> Dict[str, RowMap]:
    """Row maps of one block whose input has I tokens and which keeps the last K.

    * ``all``:  every token (b*I + p), grouped by group_of_position(p, I): K/V projections,
      and the Q projection too when K == I.
    * ``tail``: the kept tokens; space 0 = token rows b*I + p in the input, space 1 = compact
      rows b*K + j (p = I - K + j): Q projection (K < I), Wo, FFN.

    ``p0`` / ``I_full`` (serving, recommend_amd/serving.py): the I rows are the span of positions
    p0 .. p0+I-1 of a layer with I_full tokens, so a row's weight group is
    group_of_position(p0 + p, I_full).
    """
    G = cfg.num_groups
    I_full = I_full or I
    grp = np.array([cfg.group_of_position(p0 + p, I_full) for p in range(I)])
    b = np.arange(B)[:, None]

    def rows_for(positions, fn):
        if len(positions) == 0:
            return np.zeros(0, np.int64)
        return fn(b, np.asarray(positions)[None, :]).reshape(-1)

    all_pg, tail_pg = [], []
    for g in range(G):
        pos = np.nonzero(grp == g)[0]
        all_pg.append([rows_for(pos, lambda bb, pp: bb * I + pp)])
        tpos = pos[pos >= I - K]
        tail_pg.append([rows_for(tpos, lambda bb, pp: bb * I + pp),
                        rows_for(tpos, lambda bb, pp: bb * K + (pp - (I - K)))])
    return {'all': build_map(all_pg), 'tail': build_map(tail_pg)}


def head_map(B: int, T: int) -> RowMap:
    """Task heads: group t reads sample row b (space 0) and writes row t*B + b (space 1)."""
    b = np.arange(B)
    return build_map([[b, t * B + b] for t in range(T)])


def identity_map(n: int) -> RowMap:
    r = np.arange(n)
    return build_map([[r, r]])
