"""Encoder MM motion-search candidate evaluation (mm_sad_window):
InterSearch::xMVReprojectionInterpolation + RdCost::xGetSAD over candidate windows.

CPU suite: the product's planner and per-thread bodies (CPU twin) against the oracle's direct
restatement, bit-exact, for every model, integer / half / quarter-pel windows, both subShift
values and blocks at the picture edges (out-of-range margin 0)."""
import numpy as np
import pytest

import mm360
import twin
from helpers import EPI
from mm360 import workload as W
from oracle.oracle import Oracle

ALL = W.MPA3 + (mm360.TANGENTIAL, mm360.THREE_D_TRANSLATIONAL, mm360.ROTATIONAL, mm360.GEODESIC_CAMPOSE)


def _case(w, h, models, n_blocks, seed, sub_shift=0):
    blocks = W.me_blocks(w, h, models, grid=16, seed=seed, sub_shift=sub_shift, max_blocks=n_blocks)
    rng = np.random.default_rng(seed)
    # mixed sizes and edge positions
    for i in range(0, len(blocks), 5):
        bw, bh = [int(v) for v in rng.choice([4, 8, 16, 32], size=2)]
        blocks[i]["w"], blocks[i]["h"] = bw, bh
        blocks[i]["x"] = min(int(blocks[i]["x"]), w - bw)
        blocks[i]["y"] = min(int(blocks[i]["y"]), h - bh)
    blocks[0]["x"], blocks[0]["y"] = w - int(blocks[0]["w"]), h - int(blocks[0]["h"])
    blocks[1]["x"], blocks[1]["y"] = 0, 0
    blocks["mv_hor"] += rng.integers(0, 16, size=len(blocks))  # fractional centres too
    blocks["mv_ver"] += rng.integers(0, 16, size=len(blocks))
    refs = {poc: W.ref_planes(w, h, poc)[0] for poc in W.REF_POCS}
    org = W.org_plane(w, h)
    return blocks, refs, org


@pytest.mark.parametrize("w,h,models,step,sub_shift", [
    (256, 128, W.MPA3, 16, 0),
    (256, 128, ALL, 16, 1),
    (256, 128, ALL, 4, 0),
    (512, 256, ALL, 8, 0),
])
def test_twin_sad_window_matches_oracle(w, h, models, step, sub_shift):
    params = mm360.seq_params(w, h, models)
    blocks, refs, org = _case(w, h, models, 60, seed=w + step + sub_shift, sub_shift=sub_shift)
    want = Oracle(params, EPI).sad_window(W.CUR_POC, blocks, 3, step, refs, org)
    got = twin.sad_window(params, W.CUR_POC, blocks, 3, step, refs, org, EPI)
    assert want.shape == got.shape and want.max() > 0
    assert np.array_equal(got, want), np.argwhere(got != want)[:5]


@pytest.mark.parametrize("pattern", ["square2", "diamond8", "refine_quarter", "scattered"])
def test_twin_sad_pattern_matches_oracle(pattern):
    """mm_sad_pattern's host logic (planner with one thread row per block, pattern offsets, the head
    shared by the block's candidates) == the oracle's range-0 SAD of every (block, offset)."""
    w, h = 256, 128
    params = mm360.seq_params(w, h, ALL)
    sq = [(-1, -1), (0, -1), (1, -1), (-1, 0), (1, 0), (-1, 1), (0, 1), (1, 1)]
    if pattern == "square2":
        off = [(32 * x, 32 * y) for x, y in sq]
    elif pattern == "diamond8":
        off = [(0, -128), (-64, -64), (64, -64), (-128, 0), (128, 0), (-64, 64), (64, 64), (0, 128)]
    elif pattern == "refine_quarter":
        off = [(4 * x, 4 * y) for y in (-1, 0, 1) for x in (-1, 0, 1)]
    else:
        off = [(3, 0), (0, 0), (-40, 17), (100, -90), (7, 7)]
    blocks, refs, org = _case(w, h, ALL, 50, seed=31 + len(off), sub_shift=int(pattern == "scattered"))
    k = len(off)
    rep = np.repeat(blocks, k)
    o = np.tile(np.asarray(off, np.int32), (len(blocks), 1))
    rep["mv_hor"] += o[:, 0]
    rep["mv_ver"] += o[:, 1]
    want = Oracle(params, EPI).sad_window(W.CUR_POC, rep, 0, 16, refs, org).reshape(len(blocks), k)
    got = twin.sad_pattern(params, W.CUR_POC, blocks, off, refs, org, EPI)
    assert want.max() > 0
    assert np.array_equal(got, want), np.argwhere(got != want)[:5]


def test_sad_window_centre_equals_uni_prediction_sad():
    """Window centre of an interior block == SAD of the decoder-path uni prediction (the two
    differ only in the out-of-range margin, which interior blocks with small motion never hit)."""
    w, h = 256, 128
    params = mm360.seq_params(w, h, ALL)
    blocks, refs, org = _case(w, h, ALL, 40, seed=9)
    keep = (blocks["x"] >= 48) & (blocks["x"] <= w - 80) & (blocks["y"] >= 48) & (blocks["y"] <= h - 80)
    blocks = blocks[keep]
    blocks["mv_hor"] //= 8
    blocks["mv_ver"] //= 8
    blocks["sub_shift"] = 0
    sads = Oracle(params, EPI).sad_window(W.CUR_POC, blocks, 0, 16, refs, org)[:, 0]
    full = {poc: W.ref_planes(w, h, poc) for poc in W.REF_POCS}
    pus = mm360.new_pus(len(blocks))
    for i, b in enumerate(blocks):
        pus[i]["x"], pus[i]["y"], pus[i]["w"], pus[i]["h"] = b["x"], b["y"], b["w"], b["h"]
        pus[i]["mv"] = [[b["mv_hor"], b["mv_ver"]], [0, 0]]
        pus[i]["ref_poc"] = [b["ref_poc"], -1]
        pus[i]["model"] = [b["model"], b["model"]]
    orc = Oracle(params, EPI)
    for i in range(len(blocks)):
        y, _, _ = orc.predict(W.CUR_POC, pus[i:i + 1], full, w, h)
        b = blocks[i]
        pred = y[b["y"]:b["y"] + b["h"], b["x"]:b["x"] + b["w"]].astype(np.int64)
        ref = org[b["y"]:b["y"] + b["h"], b["x"]:b["x"] + b["w"]].astype(np.int64)
        assert int(np.abs(ref - pred).sum()) == int(sads[i]), i


def test_sad_window_errors():
    params = mm360.seq_params(256, 128, W.MPA3)
    blocks, refs, org = _case(256, 128, W.MPA3, 4, seed=1)
    bad = blocks.copy()
    bad[2]["model"] = mm360.TANGENTIAL
    with pytest.raises(RuntimeError, match="5"):  # MM_ERR_MODEL
        twin.sad_window(params, W.CUR_POC, bad, 1, 16, refs, org)
    bad = blocks.copy()
    bad[1]["x"] = 250
    with pytest.raises(RuntimeError, match="1"):  # MM_ERR_ARG
        twin.sad_window(params, W.CUR_POC, bad, 1, 16, refs, org)
    bad = blocks.copy()
    bad[3]["ref_poc"] = 99
    with pytest.raises(RuntimeError, match="3"):  # MM_ERR_NOREF
        twin.sad_window(params, W.CUR_POC, bad, 1, 16, refs, org)
