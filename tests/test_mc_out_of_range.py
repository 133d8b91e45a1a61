"""Out-of-range sub-blocks in the interpolation body (CPU twin of mm_pipeline.h mc_rec_impl).

xPredInterBlkMM (InterPrediction.cpp:780-783) memsets a sub-block whose window lies out of range
(xPos < -maxCU, xPos >= W + maxCU - sb, likewise y) at the precision the list is predicted at:
the final samples for a uni PU (rndRes), the 14-bit intermediate for bi (and for the 14-bit
mm_pred_list output).  ERP reprojection never produces such positions, so the twin's explicit-
position entry (twin_mc_subblock) drives the body directly; the oracle restates the same rule
(oracle/mm_oracle.c pred_blk_mm_x).
"""
import numpy as np
import pytest

import mm360
import twin
from mm360 import workload as W

W_, H_ = 256, 128
BD = 10
OFFS = 1 << 13  # IF_INTERNAL_OFFS
SHIFT = 14 - BD


def planes(seed=5):
    rng = np.random.default_rng(seed)
    y = rng.integers(0, 1 << BD, size=(H_, W_), dtype=np.int16)
    cb = rng.integers(0, 1 << BD, size=(H_ // 2, W_ // 2), dtype=np.int16)
    cr = rng.integers(0, 1 << BD, size=(H_ // 2, W_ // 2), dtype=np.int16)
    return y, cb, cr


def pos_in(x, y):  # a luma position (samples) and its co-sited chroma one, both with a fraction
    return [16 * x + 5, 16 * y + 3, 16 * x + 7, 16 * y + 9]


FAR = [-16 * 200, 16 * 10, -32 * 100, 32 * 5]  # xPos < -maxCU for luma and chroma


BCW_W1 = {0: -2, 1: 3, 2: 4, 3: 5, 4: 10}  # BCW index -> w1 (w0 = 8 - w1), Rom.cpp:203 g_BcwWeights


def addavg(p0, p1, bcw):
    """addWeightedAvg (Buffer.cpp:398-424): shiftNum = IF_INTERNAL_FRAC_BITS + 3."""
    w1 = BCW_W1[bcw]
    shift = SHIFT + 3
    off = (1 << (shift - 1)) + (OFFS << 3)
    v = (p0.astype(np.int64) * (8 - w1) + p1.astype(np.int64) * w1 + off) >> shift
    return np.clip(v, 0, (1 << BD) - 1)


@pytest.mark.parametrize("lst", [0, 1])
def test_uni_out_of_range_is_zero(lst):
    params = mm360.seq_params(W_, H_, W.MPA3)
    pos = np.zeros((2, 4), np.int32)
    pos[lst] = FAR
    y, cb, cr = twin.mc_subblock(params, 1 << lst, 0, 0, pos, planes())
    assert not y.any() and not cb.any() and not cr.any(), (y, cb, cr)


def test_hp_out_of_range_is_zero_intermediate():
    params = mm360.seq_params(W_, H_, W.MPA3)
    pos = np.array([FAR, FAR], np.int32)
    y, cb, cr = twin.mc_subblock(params, 1, 0, 1, pos, planes())
    assert not y.any() and not cb.any() and not cr.any()


@pytest.mark.parametrize("bcw", [2, 0, 4])
def test_bi_with_one_list_out_of_range_averages_a_zero_intermediate(bcw):
    params = mm360.seq_params(W_, H_, W.MPA3)
    ref = planes()
    pos = np.array([FAR, pos_in(40, 30)], np.int32)
    hy, hcb, hcr = twin.mc_subblock(params, 2, 0, 1, pos, ref)  # list 1 alone at 14 bits
    y, cb, cr = twin.mc_subblock(params, 3, bcw, 0, pos, ref)
    for got, h in ((y, hy), (cb, hcb), (cr, hcr)):
        assert np.array_equal(got, addavg(np.zeros_like(h), h, bcw))


def test_uni_in_range_matches_its_rounded_intermediate():
    """The in-range uni path the fill shares its weighting with: final = (p + 2^(h-1) + 2^13) >> h."""
    params = mm360.seq_params(W_, H_, W.MPA3)
    ref = planes()
    pos = np.array([pos_in(50, 20), FAR], np.int32)
    hy, _, _ = twin.mc_subblock(params, 1, 0, 1, pos, ref)
    y, _, _ = twin.mc_subblock(params, 1, 0, 0, pos, ref)
    want = np.clip((hy.astype(np.int64) + (1 << (SHIFT - 1)) + OFFS) >> SHIFT, 0, (1 << BD) - 1)
    assert np.array_equal(y, want)
