"""Effective blocks and the EpipoleList (a14): the product's host code in the HIP
library (called on the CPU, no GPU needed) against the oracle's independent restatements.

a2  InterPrediction::motionCompensation (InterPrediction.cpp:1681-1810): BDOF pre-check 16x16
    split (xSubPuBio :361-453), SbTMVP strip merging of identical MotionInfo (xSubPuMC :283-359),
    xCheckIdenticalMotion (:248-281), DMVR decision (UnitTools.cpp:1698-1726).
a14 EpipoleList (EpipoleList.cpp:8-99): availability, wildcard lookup, derivePredictor with its
    `predictors[0] + predictors[1] / 2` tie rule as written.
"""
import numpy as np
import pytest

import mm360
from oracle.oracle import OracleEpipoleList, effective_blocks

MODELS = (1, 2, 3, 4, 5, 6, 10)


def _random_motion(rng, n_pu, cur_poc=8):
    """Decoded PUs with every flag combination, SbTMVP PUs with partly repeated 8x8 motion."""
    pus = np.zeros(n_pu, dtype=mm360.PU_MOTION_DTYPE)
    subs = []
    n_sub = 0
    sizes = [4, 8, 16, 32, 64, 128]
    for i in range(n_pu):
        w = int(rng.choice(sizes))
        h = int(rng.choice(sizes))
        if w * h < 32:
            w = h = 8
        p = pus[i]
        p["pu"]["x"], p["pu"]["y"], p["pu"]["w"], p["pu"]["h"] = 8 * int(rng.integers(0, 64)), 8 * int(rng.integers(0, 32)), w, h
        kind = rng.random()
        refs = [int(rng.choice([0, 4, 16, 12])), int(rng.choice([16, 0, 4, 12]))]
        if w + h == 12 or kind < 0.25:  # uni
            lst = int(rng.integers(0, 2))
            refs[1 - lst] = -1
        p["pu"]["ref_poc"] = refs
        mv = rng.integers(-300, 300, size=(2, 2))
        if rng.random() < 0.15:
            mv[1] = mv[0]
            refs[1] = refs[0] if refs[0] >= 0 and refs[1] >= 0 else refs[1]
            p["pu"]["ref_poc"] = refs
        p["pu"]["mv"] = mv
        m0 = int(rng.choice(MODELS))
        p["pu"]["model"] = [m0, m0 if rng.random() < 0.7 else int(rng.choice(MODELS))]
        p["pu"]["bcw_idx"] = 2 if rng.random() < 0.7 else int(rng.integers(0, 5))
        flags = 0
        for f, prob in ((mm360.PU_MERGE, 0.6), (mm360.PU_CIIP, 0.08), (mm360.PU_SMVD, 0.08), (mm360.PU_MMVD, 0.1),
                        (mm360.PU_MVREFINE, 0.5), (mm360.PU_WEIGHTED, 0.08), (mm360.PU_LONGTERM, 0.05),
                        (mm360.PU_REF_SCALED, 0.05), (mm360.PU_MMVD_ENC2, 0.05)):
            if rng.random() < prob:
                flags |= f
        if w >= 8 and h >= 8 and rng.random() < 0.25:  # SbTMVP: a motion field on the 8x8 grid
            flags |= mm360.PU_SUBPU
            cols, rows = max(w // 8, 1), max(h // 8, 1)
            field = mm360.new_pus(cols * rows)
            base = mm360.new_pus(3)
            for b in base:
                b["ref_poc"] = [int(rng.choice([0, 16])), int(rng.choice([16, -1]))]
                b["mv"] = rng.integers(-100, 100, size=(2, 2))
                b["model"] = [int(rng.choice(MODELS)), int(rng.choice(MODELS))]
            for k in range(cols * rows):  # runs of equal motion
                field[k] = base[min(int(rng.integers(0, 5)), 2)] if rng.random() < 0.5 or k == 0 else field[k - 1]
            field["mv"][field["ref_poc"] < 0] = 0
            p["sub_motion"] = n_sub
            subs.append(field)
            n_sub += len(field)
        p["flags"] = flags
        p["cur_poc"] = cur_poc
    sub = np.concatenate(subs) if subs else mm360.new_pus(0)
    return pus, sub


@pytest.mark.parametrize("seed", range(6))
def test_effective_blocks_match_oracle(seed):
    rng = np.random.default_rng(seed)
    pus, sub = _random_motion(rng, 400)
    for tools in (mm360.ToolFlags(1, 1, 1, 0), mm360.ToolFlags(0, 1, 1, 0), mm360.ToolFlags(1, 0, 0, 1),
                  mm360.ToolFlags(1, 1, 0, 0)):
        mc, dm = mm360.derive_effective_blocks(tools, pus, sub)
        omc, odm = effective_blocks(tools, pus, sub, mm360.PU_DTYPE)
        assert np.array_equal(mc, omc), (tools.bdof, tools.dmvr, len(mc), len(omc))
        assert np.array_equal(dm, odm)
        # every luma sample of every PU is covered exactly once by the effective blocks
        cov = {}
        for b in np.concatenate([mc, dm]):
            cov[(int(b["x"]), int(b["y"]))] = cov.get((int(b["x"]), int(b["y"])), 0) + int(b["w"]) * int(b["h"])
        assert sum(cov.values()) == int((pus["pu"]["w"] * pus["pu"]["h"]).sum())


def test_effective_blocks_rules():
    """Spot checks of each rule on hand-made PUs."""
    tools = mm360.ToolFlags(1, 1, 1, 0)
    p = np.zeros(1, dtype=mm360.PU_MOTION_DTYPE)
    p["pu"]["x"], p["pu"]["y"], p["pu"]["w"], p["pu"]["h"] = 0, 0, 64, 32
    p["pu"]["ref_poc"] = [0, 16]
    p["pu"]["mv"] = [[5, 7], [-3, 2]]
    p["pu"]["model"] = [1, 1]
    p["pu"]["bcw_idx"] = 2
    p["cur_poc"] = 8
    mc, dm = mm360.derive_effective_blocks(tools, p)  # BDOF pre-check passes -> 4 x 2 sub-PUs of 16x16
    assert len(mc) == 8 and (mc["w"] == 16).all() and (mc["h"] == 16).all() and len(dm) == 0
    q = p.copy()
    q["flags"] = mm360.PU_MERGE | mm360.PU_MVREFINE  # DMVR wins over the split
    mc, dm = mm360.derive_effective_blocks(tools, q)
    assert len(mc) == 0 and len(dm) == 1 and dm[0]["w"] == 64
    r = p.copy()
    r["pu"]["bcw_idx"] = 0  # BCW disables BDOF -> no split
    mc, dm = mm360.derive_effective_blocks(tools, r)
    assert len(mc) == 1 and mc[0]["bcw_idx"] == 0
    s = p.copy()
    s["pu"]["ref_poc"] = [16, 16]
    s["pu"]["mv"] = [[5, 7], [5, 7]]
    s["pu"]["model"] = [1, 3]  # the model is not compared by xCheckIdenticalMotion
    mc, dm = mm360.derive_effective_blocks(tools, s)
    assert len(mc) == 1 and mc[0]["ref_poc"][1] == -1 and mc[0]["model"][0] == 1
    t = p.copy()  # uneven POC distances: no BDOF, no split
    t["pu"]["ref_poc"] = [0, 12]
    mc, _ = mm360.derive_effective_blocks(tools, t)
    assert len(mc) == 1 and mc[0]["w"] == 64
    # SbTMVP 32x16 (horizontal strips): 4x2 motion field, first row all equal -> one 32x8 strip
    u = p.copy()
    u["pu"]["w"], u["pu"]["h"] = 32, 16
    u["flags"] = mm360.PU_SUBPU
    field = mm360.new_pus(8)
    field["ref_poc"] = [0, 16]
    field["model"] = [1, 1]
    field["mv"][4:] = [[1, 1], [2, 2]]
    field["mv"][6] = [[9, 9], [2, 2]]
    mc, _ = mm360.derive_effective_blocks(tools, u, field)
    assert [(int(b["x"]), int(b["y"]), int(b["w"]), int(b["h"])) for b in mc] == \
        [(0, 0, 32, 8), (0, 8, 16, 8), (16, 8, 8, 8), (24, 8, 8, 8)]
    bad = p.copy()
    bad["pu"]["w"], bad["pu"]["h"] = 4, 8  # bi 4x8
    with pytest.raises(mm360.MMError):
        mm360.derive_effective_blocks(tools, bad)


def _epi_ops(rng, n):
    ops = []
    for _ in range(n):
        k = rng.random()
        cur = int(rng.choice([-1, 0, 4, 8, 12, 16, 24, 32]))
        ref = int(rng.choice([-1, 0, 16, 32]))
        q = [int(v) for v in rng.integers(-(1 << 24), (1 << 24) + 1, size=3)]
        if k < 0.1:
            q = [int(v) for v in rng.integers(-(1 << 25), (1 << 25), size=3)]  # |component| > 1
        if k < 0.45:
            ops.append(("add", cur, ref, q, bool(rng.random() < 0.6)))
        elif k < 0.55:
            ops.append(("avail", cur))
        else:
            ops.append(("query", cur, ref))
    return ops


@pytest.mark.parametrize("seed", range(8))
def test_epipole_list_matches_oracle(seed):
    rng = np.random.default_rng(100 + seed)
    a, b = mm360.EpipoleList(), OracleEpipoleList()
    assert a.count() == b.count() == 0
    for op in _epi_ops(rng, 300):
        if op[0] == "add":
            a.add(op[1], op[2], op[3], op[4])
            b.add(op[1], op[2], op[3], op[4])
        elif op[0] == "avail":
            a.make_available(op[1])
            b.make_available(op[1])
        else:
            cur, ref = op[1], op[2]
            assert a.has(cur, ref) == b.has(cur, ref)
            want = b.find(cur, ref)
            if want is None:
                with pytest.raises(mm360.MMError):
                    a.find(cur, ref)
            else:
                assert a.find(cur, ref) == want
            rc, pred = b.derive_predictor(cur)
            if rc:
                with pytest.raises(mm360.MMError):
                    a.derive_predictor(cur)
            else:
                assert a.derive_predictor(cur) == pred
        assert a.count() == b.count()


def test_epipole_predictor_tie_rule_as_written():
    """Two available epipoles at equal POC distance: predictor = p0 + p1 / 2 (not (p0 + p1) / 2),
    EpipoleList.cpp:71; the global entry must be available (CHECK :42)."""
    e = mm360.EpipoleList()
    with pytest.raises(mm360.MMError):
        e.derive_predictor(8)  # global (-1, -1) exists but is not available
    e.add(-1, -1, (1 << 20, 0, 0), True)
    e.add(4, -1, (1 << 24, 1 << 22, -(1 << 22)), True)
    e.add(12, -1, (-(1 << 23), 1 << 21, 3), True)
    # walk in key order: (-1,-1) d=9 -> p0; (4,-1) d=4 -> p0; (12,-1) d=4 -> p1 (4 < INT_MAX)
    p = e.derive_predictor(8)
    p0, p1 = (1 << 24, 1 << 22, -(1 << 22)), (-(1 << 23), 1 << 21, 3)
    assert p == tuple(a + int(b / 2) for a, b in zip(p0, p1))
    assert p != tuple((a + b) // 2 for a, b in zip(p0, p1))
    e.add(8, -1, (5, 6, 7), False)  # not available: ignored
    assert e.derive_predictor(8) == p
    e.make_available(8)
    assert e.derive_predictor(8) == (5, 6, 7)
