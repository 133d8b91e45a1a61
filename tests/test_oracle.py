"""The CPU oracle against the committed golden vectors and against the CPU twin of the device
pipeline (the product's per-thread bodies compiled for the host)."""
import numpy as np
import pytest

import mm360
import twin
from helpers import EPI, GOLDEN, describe_mismatch, load_blocks, load_pus
from mm360 import workload as W
from oracle.oracle import Oracle
import os


@pytest.mark.parametrize("name", ["reproject_c1_all_models.npz", "reproject_c2_all_models.npz",
                                  "reproject_c1_offset15_original.npz"])
def test_oracle_reproduces_golden(name):
    z = np.load(os.path.join(GOLDEN, name))
    blocks = load_blocks(z)
    off, flav = [int(v) for v in z["params"]]
    params = mm360.seq_params(int(z["width"]), int(z["height"]), [int(m) for m in z["models"]], mm_offset4x4=off,
                              ged_flavor=flav)
    got = Oracle(params, EPI).reproject(blocks)
    assert np.array_equal(got, z["result"]), describe_mismatch(blocks, got, z["result"])


def test_oracle_pred_reproduces_golden():
    z = np.load(os.path.join(GOLDEN, "pred_c1.npz"))
    cfg = W.CONFIGS["C1"]
    pus = load_pus(z)
    params = mm360.seq_params(cfg.width, cfg.height, cfg.models)
    refs = {poc: W.ref_planes(cfg.width, cfg.height, poc) for poc in W.REF_POCS}
    y, cb, cr = Oracle(params, EPI).predict(W.CUR_POC, pus, refs, cfg.width, cfg.height)
    assert np.array_equal(y, z["y"]) and np.array_equal(cb, z["cb"]) and np.array_equal(cr, z["cr"])


@pytest.mark.parametrize("w,h,models,seed,off,flav", [
    (256, 128, W.ALL_MODELS, 1, 1, 1),
    (256, 128, W.ALL_MODELS + (7, 8, 9), 2, 0, 1),
    (512, 256, W.ALL_MODELS, 3, 4, 0),
    (2048, 1024, W.ALL_MODELS, 4, 2, 1),
    (6144, 3072, W.ALL_MODELS, 5, 1, 1),
])
def test_twin_reproject_matches_oracle(w, h, models, seed, off, flav):
    params = mm360.seq_params(w, h, models, mm_offset4x4=off, ged_flavor=flav)
    blocks = W.random_blocks(w, h, models, 1500, seed, sizes=(4, 8, 16, 32, 64, 128))
    o = Oracle(params, EPI).reproject(blocks)
    t = twin.reproject(params, blocks, EPI)
    assert np.array_equal(o, t), describe_mismatch(blocks, o, t)


def test_twin_reproject_edge_cases():
    """Poles, seam, frame corners, N in {1, 2}, zero and extreme MVs (NaN / out-of-range)."""
    w, h = 512, 256
    models = W.ALL_MODELS + (7, 8, 9)
    params = mm360.seq_params(w, h, models)
    rows = []
    for m in models:
        for comp in (0, 1, 2):
            cs = 1 if comp else 0
            for (x, y, bw, bh) in [(0, 0, 4, 4), (w - 4, 0, 4, 8), (0, h - 4, 8, 4), (w - 8, h - 8, 8, 8),
                                   (w // 2 - 8, h // 2 - 8, 16, 16), (0, 0, 128, 128), (w - 128, h - 64, 128, 64)]:
                for mv in [(0, 0), (1, 0), (0, -1), (16 * 200, 0), (0, 16 * 120), (-(1 << 15), (1 << 15) - 1),
                           (8191 * 16, -8191 * 16)]:
                    bx, by, bwc, bhc = x >> cs, y >> cs, bw >> cs, bh >> cs
                    sb = 2 if comp else 4
                    if bwc < sb or bhc < sb:
                        continue
                    rows.append((bx, by, bwc, bhc, mv[0], mv[1], m, comp, W.CUR_POC, 0))
    blocks = np.array(rows, dtype=mm360.BLOCK_DTYPE)
    o = Oracle(params, EPI).reproject(blocks)
    t = twin.reproject(params, blocks, EPI)
    assert np.array_equal(o, t), describe_mismatch(blocks, o, t)


@pytest.mark.parametrize("cfg_name", ["C1", "C2", "C3"])
def test_twin_pred_matches_oracle(cfg_name):
    cfg = W.CONFIGS[cfg_name]
    params = mm360.seq_params(cfg.width, cfg.height, cfg.models)
    pus = W.pu_list(cfg, frame=1)
    refs = {poc: W.ref_planes(cfg.width, cfg.height, poc) for poc in W.REF_POCS}
    o = Oracle(params, EPI).predict(W.CUR_POC, pus, refs, cfg.width, cfg.height)
    t = twin.predict(params, W.CUR_POC, pus, refs, cfg.width, cfg.height, EPI)
    for name, a, b in zip("Y Cb Cr".split(), o, t):
        assert np.array_equal(a, b), f"{name}: {(a != b).sum()} samples differ"


def test_twin_pred_extreme_motion_zeroing():
    """MVs far outside the picture hit the out-of-range rule (InterPrediction.cpp:780)."""
    cfg = W.CONFIGS["C1"]
    params = mm360.seq_params(cfg.width, cfg.height, W.ALL_MODELS)
    pus = W.pu_list(cfg, frame=2)
    rng = np.random.default_rng(9)
    pus["model"] = rng.choice(np.array(W.ALL_MODELS), size=pus["model"].shape)
    pus["mv"] = rng.integers(-(1 << 14), 1 << 14, size=pus["mv"].shape)
    refs = {poc: W.ref_planes(cfg.width, cfg.height, poc) for poc in W.REF_POCS}
    o = Oracle(params, EPI).predict(W.CUR_POC, pus, refs, cfg.width, cfg.height)
    t = twin.predict(params, W.CUR_POC, pus, refs, cfg.width, cfg.height, EPI)
    for a, b in zip(o, t):
        assert np.array_equal(a, b)


def test_epipole_lookup_order():
    """EpipoleList::findEpipoleFixed: exact (cur, ref), then (cur, -1), then (-1, -1)."""
    w, h = 256, 128
    params = mm360.seq_params(w, h, [10])
    blocks = np.array([(16, 16, 16, 16, 100, -50, 10, 0, 8, 0), (16, 16, 16, 16, 100, -50, 10, 0, 8, 16),
                       (16, 16, 16, 16, 100, -50, 10, 0, 3, 16)], dtype=mm360.BLOCK_DTYPE)
    epi = [(8, 0, (0, 0, 1 << 24)), (8, -1, (1 << 24, 0, 0)), (-1, -1, (0, 1 << 24, 0))]
    o = Oracle(params, epi).reproject(blocks)
    t = twin.reproject(params, blocks, epi)
    assert np.array_equal(o, t)
    n = 16
    assert not np.array_equal(o[:n], o[n:2 * n]) and not np.array_equal(o[n:2 * n], o[2 * n:])


@pytest.mark.parametrize("w,h", [(256, 128), (2048, 1024), (6144, 3072)])
def test_mpa_chroma_equals_luma_for_packet_blocks(w, h):
    """The planner's MPA chroma->luma aliasing (mm_devplan.h mpa_chroma_aliases) restated on the
    oracle: for N >= 4 the 1/32-pel chroma result equals the 1/16-pel luma result."""
    params = mm360.seq_params(w, h, W.MPA3)
    rng = np.random.default_rng(w)
    rows = []
    for i in range(400):
        bw, bh = [int(v) for v in rng.choice([4, 8, 16, 32, 64], size=2)]
        if (bw // 4) * (bh // 4) < 4:
            bw, bh = 8, 8
        x = int(rng.integers(0, (w - bw) // 8 + 1)) * 8
        y = int(rng.integers(0, (h - bh) // 8 + 1)) * 8
        mvh, mvv = [int(v) for v in rng.integers(-4000, 4000, size=2)]
        m = int(rng.choice(W.MPA3))
        rows.append((x, y, bw, bh, mvh, mvv, m, 0, 8, 0))
        rows.append((x // 2, y // 2, bw // 2, bh // 2, mvh, mvv, m, 1, 8, 0))
    blocks = np.array(rows, dtype=mm360.BLOCK_DTYPE)
    r = Oracle(params, EPI).reproject(blocks)
    off = helpers_offsets(blocks)
    for i in range(0, len(blocks), 2):
        assert np.array_equal(r[off[i]:off[i + 1]], r[off[i + 1]:off[i + 2]]), blocks[i]


def helpers_offsets(blocks):
    from helpers import block_offsets
    return block_offsets(blocks)


@pytest.mark.parametrize("cfg_name", ["C1", "C2"])
def test_twin_pred_bcw_matches_oracle(cfg_name):
    """Every BCW index on bi PUs (addWeightedAvg, Buffer.cpp:398-424): the product's single
    weighted form (CPU twin) == the oracle's addAvg / addWeightedAvg dispatch."""
    cfg = W.CONFIGS[cfg_name]
    params = mm360.seq_params(cfg.width, cfg.height, cfg.models)
    pus = W.pu_list(cfg, frame=4)
    pus["bcw_idx"] = np.random.default_rng(4).integers(0, 5, len(pus))
    refs = {poc: W.ref_planes(cfg.width, cfg.height, poc) for poc in W.REF_POCS}
    o = Oracle(params, EPI).predict(W.CUR_POC, pus, refs, cfg.width, cfg.height)
    t = twin.predict(params, W.CUR_POC, pus, refs, cfg.width, cfg.height, EPI)
    for name, a, b in zip("Y Cb Cr".split(), o, t):
        assert np.array_equal(a, b), f"{name}: {(a != b).sum()} samples differ"
    # the weights matter: the same list with BCW_DEFAULT predicts a different picture
    plain = Oracle(params, EPI).predict(W.CUR_POC, W.pu_list(cfg, frame=4), refs, cfg.width, cfg.height)
    assert not np.array_equal(plain[0], o[0])


@pytest.mark.parametrize("list_,hp", [(0, 1), (1, 1), (0, 0), (1, 0)])
def test_twin_pred_list_matches_oracle(list_, hp):
    """mm_pred_list (xPredInterBlkMM 1:1 per list): the 14-bit bi=true intermediate (hp) or the
    clipped uni prediction of one list of every PU."""
    cfg = W.CONFIGS["C2"]
    params = mm360.seq_params(cfg.width, cfg.height, cfg.models)
    pus = W.pu_list(cfg, frame=5)
    pus = pus[pus["ref_poc"][:, list_] >= 0]
    refs = {poc: W.ref_planes(cfg.width, cfg.height, poc) for poc in W.REF_POCS}
    o = Oracle(params, EPI).predict_list(W.CUR_POC, pus, list_, hp, refs, cfg.width, cfg.height)
    t = twin.predict_list(params, W.CUR_POC, pus, list_, hp, refs, cfg.width, cfg.height, EPI)
    for name, a, b in zip("Y Cb Cr".split(), o, t):
        assert np.array_equal(a, b), f"{name}: {(a != b).sum()} samples differ"
    if hp:  # 14-bit intermediates leave the 10-bit range
        assert o[0].min() < 0 or o[0].max() > 1023
