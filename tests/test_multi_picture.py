"""mm_pred_device_multi (several independent pictures in one launch chain): the product's planner
with per-picture segments, camera-pose epipole tables per current POC and per-picture destination
planes (CPU twin), against the oracle's one-picture-at-a-time predictions."""
import numpy as np
import pytest

import mm360
import twin
from mm360 import workload as W
from oracle.oracle import Oracle


def _pictures(cfg, n, dmvr_share=0.0):
    """n pictures of cfg: picture q predicts POC 8 + 16 q from (16 q, 16 q + 16), its own PU list,
    its own camera-pose epipole for (cur, -1); dmvr_share: that share of the DMVR-eligible bi leaves
    flagged MM_PUF_DMVR (the references are equally far on both sides)."""
    pics, epis = [], []
    for q in range(n):
        pus = W.pu_list(cfg, frame=q, dmvr_share=dmvr_share)
        pus["ref_poc"] = np.where(pus["ref_poc"] >= 0, pus["ref_poc"] + 16 * q, -1)
        cur = W.CUR_POC + 16 * q
        pics.append((cur, pus))
        a = 1 << 24
        epis.append((cur, -1, [(a, 0, 0), (0, a, 0), (0, 11863283, 11863283), (11863283, 0, 11863283)][q % 4]))
    refs = {16 * k: W.ref_planes(cfg.width, cfg.height, 16 * k) for k in range(n + 1)}
    return pics, refs, epis


@pytest.mark.parametrize("cfg_name,n", [("C1", 2), ("C1", 4), ("C2", 3)])
def test_twin_multi_picture_matches_oracle(cfg_name, n):
    cfg = W.CONFIGS[cfg_name]
    models = tuple(cfg.models) + (mm360.GEODESIC_CAMPOSE,)
    params = mm360.seq_params(cfg.width, cfg.height, models)
    pics, refs, epis = _pictures(cfg, n)
    # every picture uses the camera-pose model somewhere, so each needs its own epipole
    for _, pus in pics:
        pus["model"][::7] = mm360.GEODESIC_CAMPOSE
    got = twin.predict_multi(params, pics, refs, cfg.width, cfg.height, epis)
    orc = Oracle(params, epis)
    for q, (cur, pus) in enumerate(pics):
        want = orc.predict(cur, pus, refs, cfg.width, cfg.height)
        for name, g, w in zip(("y", "cb", "cr"), got[q], want):
            assert np.array_equal(g, w), (q, name, int((g != w).sum()))
    # the pictures differ (own lists, own epipoles), so a mix-up of planes or epipoles would show
    assert not np.array_equal(got[0][0], got[1][0])


def test_twin_multi_picture_with_dmvr_matches_oracle():
    """mm_pred_device_multi with mm_set_dmvr on (twin): three C2 pictures, each with its own current
    POC, references and camera-pose epipole, mixing MM_PUF_DMVR PUs with ordinary ones, planned as ONE
    list == the oracle's predict_mixed picture by picture."""
    cfg = W.CONFIGS["C2"]
    models = tuple(cfg.models) + (mm360.GEODESIC_CAMPOSE,)
    params = mm360.seq_params(cfg.width, cfg.height, models)
    pics, refs, epis = _pictures(cfg, 3, dmvr_share=0.3)
    for _, pus in pics:
        pus["model"][::7] = mm360.GEODESIC_CAMPOSE
        assert W.dmvr_flagged(pus).sum() > 100
    orc = Oracle(params, epis)
    got = twin.predict_multi(params, pics, refs, cfg.width, cfg.height, epis, dmvr=True)
    for q, ((cur, pus), g) in enumerate(zip(pics, got)):
        want = orc.predict_mixed(cur, pus, refs, cfg.width, cfg.height)
        for name, a, b in zip(("y", "cb", "cr"), g, want):
            assert np.array_equal(a, b), (q, name, int((a != b).sum()))
