"""The kernels run every sub-block through the 2-D filter with the phase-0 tap row standing in
for a zero fraction.  This checks, against a direct restatement of xPredInterBlkMM's four-way
dispatch (InterPrediction.cpp:785-826) and InterpolationFilter::filterCopy/filter, that the
substitution is exact for luma (8-tap) and chroma (4-tap), uni and bi, bit depths 8..12."""
import json
import os

import numpy as np
import pytest

from helpers import GOLDEN

TAPS = json.load(open(os.path.join(GOLDEN, "filter_taps.json")))


def frac_bits(bd):
    return max(2, 14 - bd)


def param(first, last, bd):
    hr, s = frac_bits(bd), 6
    if last:
        s += 0 if first else hr
        o = (1 << (s - 1)) + (0 if first else 8192 << 6)
    else:
        s -= hr if first else 0
        o = -8192 * (1 << s) if first else 0
    return s, o


def i16(x):
    return ((x + 32768) % 65536) - 32768


@pytest.mark.parametrize("nt,table", [(8, "luma"), (4, "chroma")])
@pytest.mark.parametrize("bd", [8, 10, 12])
def test_two_d_form_equals_dispatch(nt, table, bd):
    rng = np.random.default_rng(bd * 10 + nt)
    taps = np.array(TAPS[table], dtype=np.int64)
    nph = len(taps)
    n = 200000
    mx = (1 << bd) - 1
    win = rng.integers(0, mx + 1, size=(n, nt, nt))
    kind = rng.integers(0, 4, size=(n, nt, nt))
    win = np.where(kind == 0, 0, np.where(kind == 1, mx, win)).astype(np.int64)
    xf = rng.integers(0, nph, size=n)
    yf = rng.integers(0, nph, size=n)
    xf[rng.random(n) < 0.3] = 0
    yf[rng.random(n) < 0.3] = 0
    c = nt // 2 - 1
    for bi in (False, True):
        rnd = not bi
        # unified 2-D form (kernels)
        s0, o0 = param(True, False, bd)
        h = np.stack([i16((np.einsum("nt,nt->n", win[:, r, :], taps[xf]) + o0) >> s0) for r in range(nt)], axis=1)
        s2, o2 = param(False, rnd, bd)
        u = i16((np.einsum("nt,nt->n", h, taps[yf]) + o2) >> s2)
        if rnd:
            u = np.clip(u, 0, mx)
        # reference dispatch
        ref = np.empty(n, dtype=np.int64)
        s1, o1 = param(True, rnd, bd)
        copy = (xf == 0) & (yf == 0)
        ref[copy] = win[copy, c, c] if rnd else i16(i16(win[copy, c, c] << frac_bits(bd)) - 8192)
        hor = (yf == 0) & (xf != 0)
        v = i16((np.einsum("nt,nt->n", win[hor, c, :], taps[xf[hor]]) + o1) >> s1)
        ref[hor] = np.clip(v, 0, mx) if rnd else v
        ver = (xf == 0) & (yf != 0)
        v = i16((np.einsum("nt,nt->n", win[ver, :, c], taps[yf[ver]]) + o1) >> s1)
        ref[ver] = np.clip(v, 0, mx) if rnd else v
        two = (xf != 0) & (yf != 0)
        ref[two] = u[two]
        assert np.array_equal(u, ref), f"bi={bi}: {(u != ref).sum()} mismatches"


def test_packed_tap_pair_regrouping_matches_scalar_filter():
    """The device interior filter regroups the 8-/4-tap sums into v_dot2 tap pairs chosen by
    output and window parity (mm_filter.h PackedTaps).  A host emulation of exactly that
    arithmetic equals the scalar 2-D filter for random windows, every phase, bit depths 8-12,
    bi and uni."""
    import ctypes
    import twin
    lib = twin.load()
    lib.twin_packed_taps_selftest.restype = ctypes.c_long
    lib.twin_packed_taps_selftest.argtypes = [ctypes.c_int]
    assert lib.twin_packed_taps_selftest(20000) == 0


@pytest.mark.parametrize("bd", [8, 9, 10, 11, 12])
def test_bcw_default_weighted_avg_equals_add_avg(bd):
    """The kernels use AreaBuf<Pel>::addWeightedAvg (Buffer.cpp:398-424) for every bi sub-block;
    with BCW_DEFAULT (w0 = w1 = 4) it must equal AreaBuf<Pel>::addAvg (Buffer.cpp:551-582)
    exactly, over the whole range of 14-bit intermediates (int16)."""
    rng = np.random.default_rng(bd)
    p0 = np.concatenate([rng.integers(-32768, 32768, 400000), np.arange(-32768, 32768)]).astype(np.int64)
    p1 = np.concatenate([rng.integers(-32768, 32768, 400000), np.arange(32767, -32769, -1)]).astype(np.int64)
    s = frac_bits(bd)
    maxv = (1 << bd) - 1
    avg = np.clip((p0 + p1 + (1 << s) + 2 * 8192) >> (s + 1), 0, maxv)
    sw = s + 3
    wavg = np.clip((p0 * 4 + p1 * 4 + (1 << (sw - 1)) + (8192 << 3)) >> sw, 0, maxv)
    assert np.array_equal(avg, wavg)


def test_bcw_weight_nibbles():
    """bcw_w1 (mm_pipeline.h) packs g_BcwWeights (Rom.cpp:203) as nibbles of w1 + 2."""
    want = [-2, 3, 4, 5, 10]
    got = [((0xC7650 >> (4 * i)) & 15) - 2 for i in range(5)]
    assert got == want
