"""MM-MVP (mm_mvp_convert): MVReprojection::motionVectorInDesiredMotionModel.

CPU suite: the product's planner and mm_mvp.h bodies (CPU twin) equal the oracle's restatement
for every ordered model pair including CLASSIC, both GED flavours, camera-pose epipoles that
differ between the candidate's and the current reference, poles and the ERP seam."""
import numpy as np
import pytest

import mm360
import twin
from mm360 import workload as W
from oracle.oracle import Oracle

ALL = W.MPA3 + (mm360.TANGENTIAL, mm360.THREE_D_TRANSLATIONAL, mm360.ROTATIONAL, mm360.GEODESIC_X,
                mm360.GEODESIC_Z, mm360.GEODESIC_CAMPOSE)
# two different camera-pose epipoles: (8 -> 0) and the (8, -1) wildcard for (8 -> 16)
EPI2 = [(W.CUR_POC, 0, (1 << 24, 0, 0)), (W.CUR_POC, -1, (0, 11863283, 11863283))]


@pytest.mark.parametrize("w,h,flavor", [(256, 128, 1), (2048, 1024, 1), (2048, 1024, 0)])
def test_twin_mvp_matches_oracle(w, h, flavor):
    params = mm360.seq_params(w, h, ALL, ged_flavor=flavor)
    q = W.mvp_queries(w, h, ALL, 4000, seed=w + flavor)
    orc = Oracle(params, EPI2)
    want = orc.mvp(q)
    got = twin.mvp(params, q, EPI2)
    bad = np.argwhere((got != want).any(axis=1))[:, 0]
    assert len(bad) == 0, [(int(i), q[i], got[i], want[i]) for i in bad[:3]]
    # the conversions are not trivial: most change the MV, some hit the early returns
    changed = (got != np.stack([q["mv_hor"], q["mv_ver"]], axis=1)).any(axis=1)
    assert changed.mean() > 0.5 and (~changed).sum() > 50


def test_mvp_early_returns_and_errors():
    params = mm360.seq_params(256, 128, ALL)
    q = W.mvp_queries(256, 128, ALL, 64, seed=3)
    q["mv_hor"][:4] = 0
    q["mv_ver"][:4] = 0
    q["model_orig"][4:8] = mm360.ROTATIONAL
    q["model_desired"][4:8] = mm360.ROTATIONAL
    out = twin.mvp(params, q, EPI2)
    assert (out[:4] == 0).all()
    assert (out[4:8, 0] == q["mv_hor"][4:8]).all() and (out[4:8, 1] == q["mv_ver"][4:8]).all()
    bad = q.copy()
    bad["model_orig"][10] = mm360.GEODESIC_CAMPOSE
    bad["mv_hor"][10] = 37
    with pytest.raises(RuntimeError, match="4"):  # no epipoles at all -> MM_ERR_NOEPIPOLE
        twin.mvp(params, bad, [])
    params2 = mm360.seq_params(256, 128, W.MPA3)
    with pytest.raises(RuntimeError, match="5"):  # model not active
        twin.mvp(params2, q, EPI2)


@pytest.mark.parametrize("w,h,flavor", [(256, 128, 1), (2048, 1024, 1), (6144, 3072, 1), (2048, 1024, 0)])
def test_host_mvp_matches_oracle(w, h, flavor):
    """mm_mvp_convert_host (the product library's host form, for the spatial candidates VTM converts
    in decoding order) equals the oracle query by query, without a GPU."""
    params = mm360.seq_params(w, h, ALL, ged_flavor=flavor)
    q = W.mvp_queries(w, h, ALL, 3000, seed=7 * w + flavor)
    want = Oracle(params, EPI2).mvp(q)
    epi = mm360.EpipoleList()
    for cur, ref, q24 in EPI2:
        epi.add(cur, ref, q24, make_available=True)
    got = mm360.mvp_convert_host(params, q, epi)
    bad = np.argwhere((got != want).any(axis=1))[:, 0]
    assert len(bad) == 0, [(int(i), q[i], got[i], want[i]) for i in bad[:3]]
    # one query per call (the decoder's per-candidate use) gives the same MVs
    one = np.concatenate([mm360.mvp_convert_host(params, q[i:i + 1], epi) for i in range(0, 200)])
    assert (one == want[:200]).all()


def test_host_mvp_errors_and_epipole_refresh():
    params = mm360.seq_params(256, 128, ALL)
    q = W.mvp_queries(256, 128, ALL, 64, seed=3)
    q["model_orig"][10] = mm360.GEODESIC_CAMPOSE
    q["model_desired"][10] = mm360.ROTATIONAL
    q["mv_hor"][10] = 37
    epi = mm360.EpipoleList()
    with pytest.raises(mm360.MMError) as e:  # no epipoles at all
        mm360.mvp_convert_host(params, q, epi)
    assert e.value.code == mm360.MM_ERR_NOEPIPOLE
    # adding the epipoles afterwards refreshes the host table (list version)
    for cur, ref, q24 in EPI2:
        epi.add(cur, ref, q24, make_available=True)
    want = Oracle(params, EPI2).mvp(q)
    assert (mm360.mvp_convert_host(params, q, epi) == want).all()
    with pytest.raises(mm360.MMError) as e:  # model not active
        mm360.mvp_convert_host(mm360.seq_params(256, 128, W.MPA3), q, epi)
    assert e.value.code == mm360.MM_ERR_MODEL
