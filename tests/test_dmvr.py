"""MM-DMVR (mm_pred_dmvr): InterPrediction::xProcessDMVRProjected.

CPU suite: the product's planner and per-thread bodies (CPU twin) equal the oracle's direct
restatement -- predicted planes and the refined per-sub-PU MV deltas -- for every model."""
import numpy as np
import pytest

import mm360
import twin
from helpers import EPI, describe_mismatch, dmvr_zero_mv_pus
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


def test_twin_dmvr_zero_mv_offsets_matches_oracle():
    """Offsets on the zero MV and zero merge MVs (identity setups; the device search derives the
    offsets' setups from centre terms, test_gpu.py test_pred_dmvr_zero_mv_offsets_vs_oracle)."""
    cfg = _cfg(512, 256, ALL)
    params = mm360.seq_params(512, 256, ALL)
    pus = dmvr_zero_mv_pus(cfg, ALL)
    assert len(pus) >= 4 * len(ALL)  # every (aim, model) pair
    refs = {poc: W.ref_planes(512, 256, poc) for poc in W.REF_POCS}
    want, want_mvd = Oracle(params, EPI).predict_dmvr(W.CUR_POC, pus, refs, 512, 256)
    got, got_mvd = twin.predict_dmvr(params, W.CUR_POC, pus, refs, 512, 256, EPI)
    assert np.array_equal(got_mvd, want_mvd), np.argwhere(got_mvd != want_mvd)[:5]
    for g, x in zip(got, want):
        assert np.array_equal(g, x)


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


# ---- every branch of the decision (tests/golden/dmvr_branches.npz, tools/gen_dmvr_branch_fixture.py) ----
def branch_fixture():
    """(params, width, height, [(family, refs, pus, mvd, trace)]) of the DMVR branch fixture."""
    import os
    from helpers import GOLDEN
    z = np.load(os.path.join(GOLDEN, "dmvr_branches.npz"))
    w, h = int(z["width"]), int(z["height"])
    models = [int(m) for m in z["models"]]
    params = mm360.seq_params(w, h, models)
    fams = []
    for fam in [str(f) for f in z["families"]]:
        refs = {poc: W.dmvr_branch_planes(fam, w, h, poc) for poc in W.REF_POCS}
        fams.append((fam, refs, z[f"{fam}_pus"], z[f"{fam}_mvd"], z[f"{fam}_trace"]))
    return params, w, h, fams


def test_dmvr_branch_fixture_reaches_every_branch():
    """The fixture pins the oracle's decision (deltas and branch words) and covers every branch of
    InterPrediction.cpp:2516-2531 (early exit), the border rule of xDMVRSubPixelErrorSurface
    (:2162-2163) and xSubPelErrorSrfc (:1996-2048: division, half-pel tie on each side of each axis,
    zero denominator).  The `!minCost` exit (:2528-2531) cannot be reached after the dx*dy test."""
    from oracle.oracle import dmvr_branches
    params, w, h, fams = branch_fixture()
    orc = Oracle(params, EPI)
    tot = {}
    for fam, refs, pus, mvd, tr in fams:
        _, got_mvd, got_tr = orc.predict_dmvr(W.CUR_POC, pus, refs, w, h, trace=True)
        assert np.array_equal(got_mvd, mvd), (fam, np.argwhere(got_mvd != mvd)[:5])
        assert np.array_equal(got_tr, tr), fam
        for k, v in dmvr_branches(tr).items():
            tot[k] = tot.get(k, 0) + v
    for k in ("early_exit", "border_best", "centre_best", "h_div", "v_div", "h_tie_minus", "h_tie_plus",
              "v_tie_minus", "v_tie_plus", "v_den0"):
        assert tot[k] > 0, (k, tot)


def test_twin_dmvr_branch_fixture_matches_oracle():
    """The product's DMVR bodies (CPU twin: planner, search kernels' bodies, decision) on every
    branch: the deltas and the refined predictions == the oracle, per family; and the same PUs
    mixed into a picture with unflagged PUs (mm_pred_device path)."""
    params, w, h, fams = branch_fixture()
    orc = Oracle(params, EPI)
    for fam, refs, pus, mvd, _ in fams:
        got, got_mvd = twin.predict_dmvr(params, W.CUR_POC, pus, refs, w, h, EPI)
        assert np.array_equal(got_mvd, mvd), (fam, np.argwhere(got_mvd != mvd)[:5])
        want, _ = orc.predict_dmvr(W.CUR_POC, pus, refs, w, h)
        for name, a, b in zip(("y", "cb", "cr"), got, want):
            assert np.array_equal(a, b), describe_mismatch(f"{fam} {name}", a, b)
        mixed = pus.copy()
        mixed["flags"][::2] |= mm360.PUF_DMVR
        want = orc.predict_mixed(W.CUR_POC, mixed, refs, w, h)
        got = twin.predict(params, W.CUR_POC, mixed, refs, w, h, EPI, dmvr=True)
        for name, a, b in zip(("y", "cb", "cr"), got, want):
            assert np.array_equal(a, b), describe_mismatch(f"{fam} mixed {name}", a, b)
