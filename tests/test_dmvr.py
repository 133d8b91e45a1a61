"""MM-DMVR (mm_pred_dmvr): InterPrediction::xProcessDMVRProjected.

CPU suite: the product's planner and per-thread bodies (CPU twin) equal the oracle's direct
restatement -- predicted planes and the refined per-sub-PU MV deltas -- for every model."""
import numpy as np
import pytest

import mm360
import twin
from helpers import EPI, describe_mismatch
from mm360 import workload as W
from oracle.oracle import Oracle

ALL = W.MPA3 + (mm360.TANGENTIAL, mm360.THREE_D_TRANSLATIONAL, mm360.ROTATIONAL, mm360.GEODESIC_CAMPOSE)


def _cfg(w, h, models):
    return W.Config("T", w, h, tuple(models), 1, "test")


@pytest.mark.parametrize("w,h,models", [(256, 128, W.MPA3), (512, 256, ALL)])
def test_twin_dmvr_matches_oracle(w, h, models):
    cfg = _cfg(w, h, models)
    params = mm360.seq_params(w, h, models)
    pus = W.dmvr_pu_list(cfg)
    refs = {poc: W.ref_planes(w, h, poc) for poc in W.REF_POCS}
    want, want_mvd = Oracle(params, EPI).predict_dmvr(W.CUR_POC, pus, refs, w, h)
    got, got_mvd = twin.predict_dmvr(params, W.CUR_POC, pus, refs, w, h, EPI)
    assert np.array_equal(got_mvd, want_mvd), np.argwhere(got_mvd != want_mvd)[:5]
    # the search moves a good share of the sub-PUs, with sub-pel deltas among them
    assert (want_mvd != 0).any(axis=1).mean() > 0.3 and ((want_mvd % 16) != 0).any()
    for name, a, b in zip(("y", "cb", "cr"), got, want):
        assert np.array_equal(a, b), describe_mismatch(name, a, b)


def test_dmvr_rejects_ineligible_pus():
    cfg = _cfg(256, 128, W.MPA3)
    params = mm360.seq_params(256, 128, W.MPA3)
    pus = W.dmvr_pu_list(cfg)[:8]
    refs = {poc: W.ref_planes(256, 128, poc) for poc in W.REF_POCS}
    bad = pus.copy()
    bad[3]["model"][1] = (int(bad[3]["model"][0]) % 3) + 1  # unequal models
    with pytest.raises(RuntimeError, match="1"):
        twin.predict_dmvr(params, W.CUR_POC, bad, refs, 256, 128)
    bad = pus.copy()
    bad[2]["ref_poc"][1] = -1  # uni
    with pytest.raises(RuntimeError, match="1"):
        twin.predict_dmvr(params, W.CUR_POC, bad, refs, 256, 128)


@pytest.mark.parametrize("w,h,models,share", [(256, 128, W.MPA3, 0.5), (1024, 512, ALL, 0.3)])
def test_twin_mixed_picture_matches_oracle(w, h, models, share):
    """A picture list mixing MM_PUF_DMVR PUs with ordinary PUs (mm_set_dmvr): the DMVR search runs
    inside the planned picture (placement -> search -> decision patches the sub-PUs' jobs ->
    setup / reprojection / interpolation) == the oracle's predict + predict_dmvr."""
    cfg = _cfg(w, h, models)
    params = mm360.seq_params(w, h, models)
    pus = W.pu_list(cfg, frame=1, dmvr_share=share)
    dm = W.dmvr_flagged(pus)
    assert dm.sum() > 5 and (~dm).sum() > 5
    refs = {poc: W.ref_planes(w, h, poc) for poc in W.REF_POCS}
    want = Oracle(params, EPI).predict_mixed(W.CUR_POC, pus, refs, w, h)
    got = twin.predict(params, W.CUR_POC, pus, refs, w, h, EPI, dmvr=True)
    for name, a, b in zip(("y", "cb", "cr"), got, want):
        assert np.array_equal(a, b), describe_mismatch(name, a, b)
    # without the picture's DMVR enable the flagged PUs are rejected
    with pytest.raises(RuntimeError, match="1"):
        twin.predict(params, W.CUR_POC, pus, refs, w, h, EPI)
