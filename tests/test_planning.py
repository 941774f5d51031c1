"""Host-side planning logic of the HIP path (runs on CPU: no device needed).

Checks the invariants the kernels rely on: the forward tile list covers every (row, column)
tile pair exactly once counting the mirrored lower triangle of the own-rank block, the dZ
tiles cover the output, and the persistent stream-K schedule covers every K-step of every
tile exactly once with the per-block work balanced.
"""
import pytest

from ntxent_amd.ops import _ext


@pytest.fixture(scope="module")
def C():
    return _ext.load()


@pytest.mark.parametrize("rows,dim", [(64, 128), (34, 100), (8192, 2048), (600, 200), (2048, 8192)])
def test_geometry(C, rows, dim):
    g = C.geometry(rows, dim)
    assert g["rows_pad"] % C.TILE == 0 and g["rows_pad"] >= rows > g["rows_pad"] - C.TILE
    assert g["dim_k"] % 64 == 0 and g["dim_k"] >= dim
    assert g["dim_n"] % C.TILE == 0 and g["dim_n"] >= g["dim_k"]
    assert g["ld_k"] >= g["dim_k"] and g["ld_t"] >= g["rows_pad"]
    # de-aliased strides: never a multiple of 1024 elements
    assert g["ld_k"] % 1024 != 0 and g["ld_t"] % 1024 != 0
    assert g["col_tiles"] == g["row_tiles"] and g["global_rows"] == rows


def test_geometry_rejects_bad_input(C):
    with pytest.raises(Exception):
        C.geometry(7, 16)
    with pytest.raises(Exception):
        C.geometry(8, 16, 2, 2)
    with pytest.raises(Exception):
        C.geometry(8, 0)


@pytest.mark.parametrize("rows,world,rank", [(512, 1, 0), (8192, 1, 0), (1024, 4, 2), (300, 2, 1), (8192, 8, 7)])
def test_fwd_tiles_cover_once(C, rows, world, rank):
    g = C.geometry(rows, 64, world, rank)
    tiles = C.fwd_tile_list(rows, 64, world, rank)
    own = rank * g["row_tiles"]
    covered = {}
    for ti, tj, kind in tiles:
        local = tj - own
        if 0 <= local < g["row_tiles"]:
            assert local >= ti
            assert kind == (1 if local == ti else 2)
            covered[(ti, tj)] = covered.get((ti, tj), 0) + 1
            if local != ti:
                covered[(local, own + ti)] = covered.get((local, own + ti), 0) + 1
        else:
            assert kind == 0
            covered[(ti, tj)] = covered.get((ti, tj), 0) + 1
    assert len(covered) == g["row_tiles"] * g["col_tiles"]
    assert set(covered.values()) == {1}
    rt = g["row_tiles"]
    assert len(tiles) == rt * (g["col_tiles"] - rt) + rt * (rt + 1) // 2
    # the own block ends with its diagonal tiles (the strip kernel's remainder, launch_fwd_stats)
    n_own = rt * (rt + 1) // 2
    assert [t[2] for t in tiles[n_own - rt:n_own]] == [1] * rt
    assert [t[0] for t in tiles[n_own - rt:n_own]] == list(range(rt))


def test_dz_tiles_cover_output(C):
    g = C.geometry(1024, 600)
    tiles = C.dz_tile_list(1024, 600)
    assert sorted((t[0], t[1]) for t in tiles) == [(i, j) for i in range(g["row_tiles"]) for j in range(g["dim_n"] // C.TILE)]


@pytest.mark.parametrize("ntiles,nk,cus", [(528, 32, 256), (256, 128, 256), (10, 4, 256), (1, 3, 256),
                                           (300, 7, 256), (136, 16, 80), (1000, 2, 256), (36, 128, 256),
                                           (528, 8, 256), (2080, 16, 256)])
def test_stream_k_schedule(C, ntiles, nk, cus):
    s = C.schedule(ntiles, nk, cus)
    G = s["grid"]
    assert 1 <= G <= cus
    assert s["dp_tiles"] + s["sk_tiles"] == ntiles
    assert s["dp_tiles"] % G == 0  # whole data-parallel rounds
    # only the remainder of the DP rounds is split
    assert s["sk_tiles"] == ntiles % cus
    # every stream-K iteration is owned by exactly one block, contiguous ranges
    total = s["sk_tiles"] * nk
    if total:
        ipb = s["ipb"]
        assert G * ipb >= total
        owned = 0
        pieces = {}
        for b in range(G):
            lo, hi = b * ipb, min((b + 1) * ipb, total)
            owned += max(0, hi - lo)
            for t in range(lo // nk, (hi - 1) // nk + 1) if hi > lo else []:
                pieces[t] = pieces.get(t, 0) + 1
        assert owned == total
        # few contributors per split tile: the split p minimises nk/p + (p > 1: 10 + 4 (p - 1))
        # (make_schedule's cost model); the last arriver sums at most p + 1 slabs
        cands = range(1, max(1, min(cus // s["sk_tiles"], nk)) + 1)
        p_opt = min(cands, key=lambda c: (nk / c + (10 + 4 * (c - 1) if c > 1 else 0), c))
        assert max(pieces.values()) <= p_opt + 1
        assert s["ipb"] == -(-nk // p_opt)
    # balance: the busiest block does at most one DP round + ipb steps more than the mean
    mean = ntiles * nk / G
    worst = (s["dp_tiles"] // G) * nk + s["ipb"]
    assert worst <= mean + nk + 1


def test_workspace_bytes(C):
    # fixed layout: 2*num_cus arrival counters (stream-K splits < 2G tiles) + 2 fp32 tiles per block,
    # independent of the launch's tile count so launches can share one zero-initialised workspace
    b = C.gemm_workspace_bytes(528, 256)
    assert b >= 2 * 256 * 4 + 2 * 256 * 256 * 256 * 4
    assert b == C.gemm_workspace_bytes(7696, 256) == C.gemm_workspace_bytes(1, 256)
    for nt, nk in [(528, 32), (7696, 32), (300, 7), (255, 3)]:
        assert C.schedule(nt, nk, 256)["sk_tiles"] <= 2 * 256


def _panels_per_group(tiles, n_own, group=32):
    """Mean distinct Zq row panels (A and B) over consecutive `group`-tile runs of the own block:
    the L2 footprint of one XCD's share of a GEMM round (XCD-contiguous block mapping)."""
    own = [t for t in tiles[:n_own]]
    counts = []
    for s in range(0, len(own) - group + 1, group):
        counts.append(len({t[0] for t in own[s:s + group]} | {t[1] for t in own[s:s + group]}))
    return sum(counts) / len(counts)


def _zorder_list(rt):
    """The Z-order (Morton) own-block list the superblock order replaced (kept here as the
    reference: the off-diagonal upper tiles by Morton key, then the diagonal tail)."""
    def key(i, j):
        r = 0
        for b in range(16):
            r |= ((i >> b) & 1) << (2 * b + 1) | ((j >> b) & 1) << (2 * b)
        return r
    off = sorted([(i, j, 2) for i in range(rt) for j in range(i + 1, rt)], key=lambda t: key(t[0], t[1]))
    return off + [(i, i, 1) for i in range(rt)]


@pytest.mark.parametrize("rows", [8192, 16384, 2048, 6144])
def test_superblock_order_covers_same_tiles_with_fewer_panels(C, rows):
    """own_block_tiles: 8-panel superblocks (row-tile counts that are multiples of 8, >= 16; else
    the Z-order fallback) list the same tiles as Z-order with the diagonal tail last, and touch
    fewer distinct panels per 32-tile group (13.2 vs 15.4 at 32 row tiles)."""
    g = C.geometry(rows, 64, 1, 0)
    rt = g["row_tiles"]
    n_own = rt * (rt + 1) // 2
    a = [tuple(t) for t in C.fwd_tile_list(rows, 64, 1, 0)]
    b = _zorder_list(rt)
    assert sorted(a) == sorted(b) and len(set(a)) == len(a)
    assert a[n_own - rt:n_own] == b[n_own - rt:n_own] == [(i, i, 1) for i in range(rt)]
    if rt % 8 == 0 and rt >= 16:
        assert a != b
        pa, pb = _panels_per_group(a, n_own - rt), _panels_per_group(b, n_own - rt)
        assert pa < pb - (1.5 if rt == 32 else 0.0), (pa, pb)
    else:
        assert a == b
