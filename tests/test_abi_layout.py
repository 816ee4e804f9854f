"""CPU: the C-ABI library loads and exports every entry point include/onetrans_hip.h declares, the
ctypes signatures match the header prototypes, and the row maps / flat layout are consistent."""

import os
import re

import numpy as np
import pytest

from recommend_amd import _lib
from recommend_amd.config import workload_config
from recommend_amd.layout import TILE, FlatLayout, build_map, head_map, layer_maps


def _prototypes():
    txt = open(_lib.HEADER).read()
    txt = re.sub(r'/\*.*?\*/', '', txt, flags=re.S)
    protos = {}
    for m in re.finditer(r'\b(?:int|size_t|const char\*)\s+(ot_[a-z0-9_]+)\s*\(([^)]*)\)\s*;', txt):
        args = [a.strip() for a in m.group(2).split(',') if a.strip() and a.strip() != 'void']
        protos[m.group(1)] = args
    return protos


def test_header_and_ctypes_agree():
    protos = _prototypes()
    assert set(protos) == set(_lib.SIGNATURES), set(protos) ^ set(_lib.SIGNATURES)
    for name, args in protos.items():
        assert len(args) == len(_lib.SIGNATURES[name][1]), name


@pytest.mark.skipif(not os.path.exists(_lib.LIB_PATH), reason='library not built')
def test_library_exports_every_symbol():
    lib = _lib.load()
    for s in _lib.header_symbols():
        assert hasattr(lib, s), s
    assert lib.ot_version() == 20000
    assert lib.ot_gemm_tile_rows() == TILE
    # workspace-size queries are host-only (no GPU needed)
    assert lib.ot_wgrad_workspace_size(3, 128, 64) == (3 * 128 * 64 + 3 * 64) * 4
    assert lib.ot_sparse_adagrad_workspace_size(1000, 64) > 1000 * 64 * 4


@pytest.mark.skipif(not os.path.exists(_lib.LIB_PATH), reason='library not built')
def test_errors_are_reported_not_crashing():
    """Invalid arguments return OT_ERR_INVALID_ARG with a message (no device work)."""
    with pytest.raises(_lib.OneTransHipError, match='null operand'):
        _lib.call('ot_attn_fwd', None, 96, 1, 1, 4, 4, None, 32, None, None, 1, None)
    with pytest.raises(_lib.OneTransHipError, match='multiples of 4'):
        _lib.call('ot_mixed_gemm', 0, 8, 3, 3, None, 0, None, None, 8, 0, 4, 4, None, 1, None, 0, 8, 4, None, 0,
                  None, 0, 0, None, 0, 0, 0, 0.0, 1, 1, None, 1, None)
    with pytest.raises(_lib.OneTransHipError, match='unknown precision'):
        _lib.call('ot_attn_fwd', None, 96, 1, 1, 4, 4, None, 32, None, None, 7, None)
    # an ot_rms_epilogue from another header version (struct_size differs) is refused, not read past its end
    import ctypes
    e = _lib.RmsEpilogue()
    e.struct_size = ctypes.sizeof(_lib.RmsEpilogue) - 24
    with pytest.raises(_lib.OneTransHipError, match='struct_size'):
        _lib.call('ot_mixed_gemm_rms', 0, None, 128, 128, None, 0, None, None, None, 0, 128, 128, None, 1, None, 0,
                  None, 128, None, 0, None, 0, 0, None, 0, 0, 0, 0.0, 1, 1, None, ctypes.byref(e), 1, None)
    with pytest.raises(_lib.OneTransHipError, match='bad sizes'):
        _lib.call('ot_pyramid_select', None, 1.0, 2, 8, 9, 0, 8, None, None, 0, None)    # K > I
    with pytest.raises(_lib.OneTransHipError, match='bad sizes'):
        _lib.call('ot_pyramid_select', None, 1.0, 2, 5000, 9, 0, 8, None, None, 0, None)  # I > 4096
    with pytest.raises(_lib.OneTransHipError, match='nforce'):
        _lib.call('ot_pyramid_select', None, 1.0, 2, 40, 6, 8, 8, None, None, 0, None)    # nforce > K


@pytest.mark.parametrize('mode', ['head', 'tail'])
@pytest.mark.parametrize('I,K', [(140, 140), (140, 1), (40, 17)])
def test_layer_maps_cover_rows(mode, I, K):
    cfg = workload_config('C2')
    cfg.dedicated_positions = mode
    B = 37
    m = layer_maps(cfg, B, I, K)
    a = m['all']
    rows = a.rows[0]
    assert len(rows) == a.ntiles * TILE
    valid = rows[rows >= 0]
    assert sorted(valid) == list(range(B * I))                   # every token exactly once
    for t in range(a.ntiles):                                    # every tile one group, right group
        r = rows[t * TILE:(t + 1) * TILE]
        r = r[r >= 0]
        g = {cfg.group_of_position(int(x % I), I) for x in r}
        assert g <= {int(a.tile_group[t])}
    tl = m['tail']
    tin, tc = tl.rows[0], tl.rows[1]
    ok = tin >= 0
    assert np.all((tc >= 0) == ok)
    b = tc[ok] // K
    j = tc[ok] % K
    assert np.array_equal(tin[ok], b * I + (I - K) + j)           # tail token <-> compact row
    assert sorted(tc[ok]) == list(range(B * K))
    # wgrad chunks partition each group's padded rows
    for mp in (a, tl):
        cov = np.zeros(len(mp.rows[0]), int)
        for (g, s, n) in mp.chunks:
            cov[s:s + n] += 1
            assert np.all(mp.tile_group[s // TILE:(s + n - 1) // TILE + 1] == g)
        assert np.all(cov == 1)
        for g, (c0, cn) in enumerate(mp.gchunk):
            assert np.all(mp.chunks[c0:c0 + cn, 0] == g)


def test_flat_layout():
    cfg = workload_config('C2')
    L = FlatLayout(cfg, cfg.ns_input_width())
    assert L.f_pad % 4 == 0 and L.f_pad >= L.f_ns == 429
    offs = sorted((o, n) for n, o in L.offsets.items())
    for (o, n), (o2, _) in zip(offs, offs[1:] + [(L.total, None)]):
        assert o % 64 == 0
        assert o + int(np.prod(L.shapes[n])) <= o2
    # every clip segment lies inside one bank
    ends = {n: L.offsets[n] + int(np.prod(L.shapes[n])) for n in L.shapes}
    for (o, r, c, s) in L.segments:
        last = o + (r - 1) * s + c
        assert any(L.offsets[n] <= o and last <= ends[n] for n in L.shapes)


def test_head_map():
    m = head_map(300, 2)
    assert m.ntiles == 2 * 3
    assert np.array_equal(m.rows[1][m.rows[1] >= 0], np.arange(600))


@pytest.mark.parametrize('name,tiles', [('C2', 3), ('C2', 4), ('T', 12), ('C5', 64)])
def test_wgrad_chunks_partition_and_budget(name, tiles):
    """layout.RowMap.chunks_for: the chunks of each weight group tile its padded rows exactly once, in
    32-row multiples, and the launch stays within the workgroup budget of layout.wgrad_slots (the
    per-group floor aside: every nonempty group has a chunk of its own)."""
    from recommend_amd import layout as L
    cfg = workload_config(name)
    I = cfg.num_ns_tokens + cfg.seq_token_count(cfg._seq_lens)       # L0: 140 / 140 / 1036
    B = 64
    mp = layer_maps(cfg, B, I, I)['all']
    ch, gc, n = mp.chunks_for(tiles, 'cpu')
    ch, gc = ch.numpy(), gc.numpy()
    padded = [(r + TILE - 1) // TILE * TILE for r in mp.group_rows]
    groups = sum(1 for p in padded if p > 0)
    assert n == len(ch) and n * tiles <= L.wgrad_slots(tiles) + groups * tiles
    base = 0
    for g, p in enumerate(padded):
        c0, cn = gc[g]
        rows = ch[c0:c0 + cn]
        assert np.all(rows[:, 0] == g)
        assert np.all(rows[:-1, 2] % 32 == 0) if cn > 1 else True
        assert sum(rows[:, 2]) == p and (cn == 0 or rows[0, 1] == base)
        assert np.all(rows[1:, 1] == rows[:-1, 1] + rows[:-1, 2])
        base += p
    assert L.wgrad_slots(8) >= L.wgrad_slots(4)
