"""Synthetic workload generator and host-side sub-PU split rules."""
import mm360
import numpy as np
import pytest

from mm360 import workload as W


@pytest.mark.parametrize("cfg_name", ["C1", "C2", "C3"])
def test_pu_list_tiles_picture(cfg_name):
    cfg = W.CONFIGS[cfg_name]
    pus = W.pu_list(cfg)
    cover = np.zeros((cfg.height // 4, cfg.width // 4), dtype=np.int32)
    for p in pus:
        cover[p["y"] // 4:(p["y"] + p["h"]) // 4, p["x"] // 4:(p["x"] + p["w"]) // 4] += 1
    assert (cover == 1).all()
    assert W.luma_area(pus) == cfg.width * cfg.height


def test_pu_rules():
    pus = W.pu_list(W.CONFIGS["C2"])
    bi = (pus["ref_poc"][:, 0] >= 0) & (pus["ref_poc"][:, 1] >= 0)
    small = pus["w"] * pus["h"] < 64
    assert not (bi & small).any(), "8x4 / 4x8 PUs are uni-only"
    assert (pus["w"][bi] <= 16).all() and (pus["h"][bi] <= 16).all(), "bi PUs split to <=16x16 (xSubPuBio)"
    assert set(np.unique(pus["model"])) <= set(W.CONFIGS["C2"].models)
    frac_bi_area = (pus["w"] * pus["h"] * bi).sum() / (pus["w"] * pus["h"]).sum()
    assert 0.45 < frac_bi_area < 0.75


def test_ref_planes_deterministic_10bit():
    a = W.ref_planes(256, 128, 0)
    b = W.ref_planes(256, 128, 0)
    for x, y in zip(a, b):
        assert np.array_equal(x, y) and x.dtype == np.int16 and x.min() >= 0 and x.max() <= 1023
    assert a[0].shape == (128, 256) and a[1].shape == (64, 128)


def test_pu_lists_come_from_the_effective_block_derivation():
    """The bench / test PU lists are the product's mm_derive_effective_blocks output on the decoded
    PUs (InterPrediction::motionCompensation's BDOF split), equal to the oracle's own derivation;
    with a DMVR share the merge/mvRefine PUs come out unsplit and flagged MM_PUF_DMVR."""
    from oracle.oracle import effective_blocks
    cfg = W.CONFIGS["C2"]
    for share in (0.0, 0.4):
        dec, tools = W.decoded_pus(cfg, frame=3, dmvr_share=share)
        mc, dm = effective_blocks(tools, dec, mm360.new_pus(0), mm360.PU_DTYPE)
        got = W.pu_list(cfg, frame=3, dmvr_share=share)
        flag = W.dmvr_flagged(got)
        assert got[~flag].tobytes() == mc.tobytes()
        g = got[flag].copy()
        g["flags"] = 0
        assert g.tobytes() == dm.tobytes()
        assert (len(dm) > 0) == (share > 0)
        # every bi PU of the plain list is at most 16x16 (xSubPuBio), DMVR PUs keep their size
        bi = (got["ref_poc"][:, 0] >= 0) & (got["ref_poc"][:, 1] >= 0)
        assert (got["w"][bi & ~flag] <= 16).all() and (got["h"][bi & ~flag] <= 16).all()
        if share:
            assert (got["w"][flag] * got["h"][flag] > 256).any()
