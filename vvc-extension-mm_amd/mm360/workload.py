"""Seeded synthetic ERP workloads.

No MM bitstreams exist and none can be produced offline, so every "decode" configuration is a
synthetic per-picture PU list over synthetic 10-bit 4:2:0 ERP reference planes:

* planes: clip(512 + 300 sin(3 phi) sin(2 theta) + 120 sin(17 phi + 5 theta) + U(-16, 16)),
  seed 0x4D4D0000 + poc;
* PU lists: every 128x128 CTU split by a seeded random QT/BT into PUs of 8x8 .. 64x64 plus
  8x4 / 4x8 (uni only); per PU a model uniform over the active non-CLASSIC ids, 60 % bi /
  40 % uni, MV integer part U[-32, 32] px and fraction U{0..15}/16, curPOC 8, refPOCs {0, 16};
* the host applies the reference's sub-PU split for bi PUs (motionCompensation ->
  xSubPuBio, InterPrediction.cpp:1786-1789 + :361-453): with refs 0 and 16 around POC 8 every
  bi PU >= 8x8 with area >= 128 is BDOF-eligible by the pre-check, so a bi PU wider or taller
  than 16 becomes min(16, w) x min(16, h) sub-PUs (the reprojection block centre moves).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Sequence, Tuple

import numpy as np

from . import (GEODESIC_CAMPOSE, MPA_FRONT_BACK, MPA_LEFT_RIGHT, MPA_TOP_BOTTOM, ROTATIONAL,
               TANGENTIAL, THREE_D_TRANSLATIONAL, new_pus)

MPA3 = (MPA_FRONT_BACK, MPA_LEFT_RIGHT, MPA_TOP_BOTTOM)
ALL_MODELS = MPA3 + (TANGENTIAL, THREE_D_TRANSLATIONAL, ROTATIONAL, GEODESIC_CAMPOSE)

CUR_POC = 8
REF_POCS = (0, 16)
GED_EPIPOLE_Q24 = (1 << 24, 0, 0)  # epipole (1, 0, 0) in Q24 (README.md:59)


@dataclass(frozen=True)
class Config:
    name: str
    width: int
    height: int
    models: Tuple[int, ...]
    frames: int
    description: str


CONFIGS = {
    "C1": Config("C1", 256, 128, MPA3, 4, "256x128 ERP, MPA=1 only (CPU plumbing case)"),
    "C2": Config("C2", 2048, 1024, MPA3 + (GEODESIC_CAMPOSE, ROTATIONAL), 32,
                 "2048x1024 ERP decode, MPA+GED+ROT"),
    "C3": Config("C3", 6144, 3072, ALL_MODELS, 1, "6144x3072 ERP decode, all 5 motion models"),
    "C5": Config("C5", 2048, 1024, ALL_MODELS, 1,
                 "2048x1024 ERP encoder ME candidate eval: 16x16 PU grid x every model x 33x33 integer window"),
}
ME_RANGE = 16  # C5: 33x33 integer candidate window


def ref_planes(width: int, height: int, poc: int, bit_depth: int = 10):
    """Synthetic 10-bit ERP content (int16 Y, Cb, Cr; 4:2:0)."""
    rng = np.random.default_rng(0x4D4D0000 + poc)

    def plane(w, h, phase):
        x = (np.arange(w, dtype=np.float64) + 0.5) / w * 2.0 * math.pi
        y = (np.arange(h, dtype=np.float64) + 0.5) / h * math.pi
        phi, theta = np.meshgrid(x + phase, y)
        v = 512 + 300 * np.sin(3 * phi) * np.sin(2 * theta) + 120 * np.sin(17 * phi + 5 * theta)
        v = v + rng.integers(-16, 17, size=v.shape)
        return np.clip(np.rint(v), 0, (1 << bit_depth) - 1).astype(np.int16)

    return plane(width, height, 0.0), plane(width // 2, height // 2, 0.7), plane(width // 2, height // 2, 1.9)


def _split_ctu(rng, x0, y0, w, h, out):
    """Seeded random QT/BT split down to 8x8 .. 64x64 leaves (plus occasional 8x4 / 4x8)."""
    options = []
    if w <= 64 and h <= 64 and w >= 8 and h >= 8:
        options += ["leaf"] * 3
    if w >= 16 and h >= 16:
        options += ["qt"] * (4 if (w > 64 or h > 64) else 2)
    if w >= 16 and h <= 64:
        options.append("btv")
    if h >= 16 and w <= 64:
        options.append("bth")
    if w == 8 and h == 8:
        options.append("small")
    choice = options[int(rng.integers(0, len(options)))] if options else "leaf"
    if choice == "leaf":
        out.append((x0, y0, w, h))
    elif choice == "qt":
        for dy in (0, h // 2):
            for dx in (0, w // 2):
                _split_ctu(rng, x0 + dx, y0 + dy, w // 2, h // 2, out)
    elif choice == "btv":
        _split_ctu(rng, x0, y0, w // 2, h, out)
        _split_ctu(rng, x0 + w // 2, y0, w // 2, h, out)
    elif choice == "bth":
        _split_ctu(rng, x0, y0, w, h // 2, out)
        _split_ctu(rng, x0, y0 + h // 2, w, h // 2, out)
    else:  # 8x8 -> two 4x8 or two 8x4 (uni-only PUs)
        if rng.random() < 0.5:
            out += [(x0, y0, 4, 8), (x0 + 4, y0, 4, 8)]
        else:
            out += [(x0, y0, 8, 4), (x0, y0 + 4, 8, 4)]


def decoded_pus(cfg: Config, frame: int = 0, uniform: bool = False, uniform_model: int = None, ctu: int = 128,
                dmvr_share: float = 0.0):
    """The decoded PUs of a synthetic picture (PU_MOTION_DTYPE) and the picture's tool switches:
    one record per leaf of the seeded CTU split, with its motion and the flags the decoder would
    carry.  BDOF is on (RA cfg, cfg/encoder_randomaccess_vtm.cfg:139); DMVR is on only when
    `dmvr_share` > 0, and then that share of the DMVR-eligible bi leaves (w, h >= 8, w * h >= 128)
    is a merge PU with mvRefine and one model for both lists (PU::checkDMVRCondition requires
    equal models, UnitTools.cpp:1715).  The DMVR decisions draw from their own seeded stream, so
    the workload without DMVR does not change."""
    from . import PU_MERGE, PU_MOTION_DTYPE, PU_MVREFINE, ToolFlags
    rng = np.random.default_rng(0x4D4D1000 + 977 * frame + cfg.width)
    rng_d = np.random.default_rng(0x4D4D5000 + 977 * frame + cfg.width)
    models = cfg.models
    leaves: List[Tuple[int, int, int, int]] = []
    if uniform:
        for y in range(0, cfg.height, 16):
            for x in range(0, cfg.width, 16):
                leaves.append((x, y, 16, 16))
    else:
        for y0 in range(0, cfg.height, ctu):
            for x0 in range(0, cfg.width, ctu):
                _split_ctu(rng, x0, y0, min(ctu, cfg.width - x0), min(ctu, cfg.height - y0), leaves)
    out = np.zeros(len(leaves), dtype=PU_MOTION_DTYPE)
    out["pu"]["bcw_idx"] = 2  # BCW_DEFAULT
    out["cur_poc"] = CUR_POC
    out["sub_motion"] = -1
    for i, (x, y, w, h) in enumerate(leaves):
        small = (w * h) < 64  # 8x4 / 4x8: uni only
        bi = (not small) and rng.random() < 0.6
        if uniform:
            m0 = m1 = uniform_model if uniform_model is not None else models[0]
        else:
            m0 = int(models[rng.integers(0, len(models))])
            m1 = int(models[rng.integers(0, len(models))])
        mvs = []
        for _ in range(2):
            mvs.append([int(rng.integers(-32, 33)) * 16 + int(rng.integers(0, 16)),
                        int(rng.integers(-32, 33)) * 16 + int(rng.integers(0, 16))])
        if bi:
            refs = (REF_POCS[0], REF_POCS[1])
        else:
            lst = int(rng.integers(0, 2))
            refs = (REF_POCS[0], -1) if lst == 0 else (-1, REF_POCS[1])
        if dmvr_share > 0 and bi and w >= 8 and h >= 8 and w * h >= 128 and rng_d.random() < dmvr_share:
            m1 = m0
            out[i]["flags"] = PU_MERGE | PU_MVREFINE
        u = out[i]["pu"]
        u["x"], u["y"], u["w"], u["h"] = x, y, w, h
        u["mv"] = np.array(mvs, dtype=np.int32)
        u["ref_poc"] = refs
        u["model"] = (m0, m1)
    tools = ToolFlags(bdof=1, dmvr=1 if dmvr_share > 0 else 0, bcw=1, wp_bi=0)
    return out, tools


def pu_list(cfg: Config, frame: int = 0, uniform: bool = False, uniform_model: int = None,
            ctu: int = 128, dmvr_share: float = 0.0) -> np.ndarray:
    """Per-picture PU list, PU_DTYPE: the decoded PUs (decoded_pus) through the product's
    effective-block derivation (mm_derive_effective_blocks = InterPrediction::motionCompensation's
    control flow, InterPrediction.cpp:1681-1810): bi PUs wider or taller than 16 become 16x16
    sub-PUs by the BDOF pre-check (xSubPuBio).  With a DMVR share, the DMVR PUs follow the rest,
    flagged MM_PUF_DMVR (mm_pred_device runs their search; mm_set_dmvr must be on)."""
    from . import PUF_DMVR, derive_effective_blocks
    dec, tools = decoded_pus(cfg, frame, uniform, uniform_model, ctu, dmvr_share)
    mc, dmvr = derive_effective_blocks(tools, dec)
    if len(dmvr):
        dmvr = dmvr.copy()
        dmvr["flags"] |= PUF_DMVR
        return np.concatenate([mc, dmvr])
    return mc


def dmvr_flagged(pus: np.ndarray) -> np.ndarray:
    """Mask of the MM_PUF_DMVR PUs of a list."""
    from . import PUF_DMVR
    return (pus["flags"] & PUF_DMVR) != 0


def luma_area(pus: np.ndarray) -> int:
    return int((pus["w"].astype(np.int64) * pus["h"]).sum())


def algorithmic_bytes(pus: np.ndarray) -> int:
    """uni 6 B / bi 9 B per output luma pixel (int16 samples, 4:2:0)."""
    area = pus["w"].astype(np.int64) * pus["h"]
    bi = (pus["ref_poc"][:, 0] >= 0) & (pus["ref_poc"][:, 1] >= 0)
    return int((area * np.where(bi, 9, 6)).sum())


def random_blocks(width: int, height: int, models: Sequence[int], n: int, seed: int,
                  comps=(0, 1), sizes=(4, 8, 16, 32, 64), mv_range: int = 32, cur_poc: int = CUR_POC,
                  ref_pocs=REF_POCS) -> np.ndarray:
    """Random reprojection requests covering every model / component / N in {1,2,4,...}."""
    from . import BLOCK_DTYPE
    rng = np.random.default_rng(seed)
    out = np.zeros(n, dtype=BLOCK_DTYPE)
    for i in range(n):
        comp = int(comps[rng.integers(0, len(comps))])
        cs = 1 if comp else 0
        w = int(sizes[rng.integers(0, len(sizes))])
        h = int(sizes[rng.integers(0, len(sizes))])
        if comp == 0 and (w < 4 or h < 4):
            w, h = max(w, 4), max(h, 4)
        wc, hc = w >> cs, h >> cs
        if comp and (wc < 2 or hc < 2):
            wc, hc = max(wc, 2), max(hc, 2)
        sb = 2 if comp else 4
        Wc, Hc = width >> cs, height >> cs
        x = int(rng.integers(0, (Wc - wc) // sb + 1)) * sb
        y = int(rng.integers(0, (Hc - hc) // sb + 1)) * sb
        kind = rng.random()
        if kind < 0.1:
            mvh = mvv = 0
        elif kind < 0.2:
            mvh = int(rng.integers(-2000, 2001))
            mvv = int(rng.integers(-2000, 2001))
        else:
            mvh = int(rng.integers(-mv_range * 16, mv_range * 16 + 1))
            mvv = int(rng.integers(-mv_range * 16, mv_range * 16 + 1))
        model = int(models[rng.integers(0, len(models))])
        out[i] = (x, y, wc, hc, mvh, mvv, model, comp if comp == 0 else int(rng.integers(1, 3)),
                  cur_poc, int(ref_pocs[rng.integers(0, len(ref_pocs))]))
    return out


def org_plane(width: int, height: int, poc: int = CUR_POC, bit_depth: int = 10) -> np.ndarray:
    """Seeded 'original' luma picture for the encoder SAD (the reference content of POC `poc`
    plus noise, so that good candidates exist)."""
    y, _, _ = ref_planes(width, height, poc, bit_depth)
    return y


def me_blocks(width: int, height: int, models: Sequence[int], grid: int = 16, seed: int = 5,
              ref_poc: int = REF_POCS[0], sub_shift: int = 0, max_blocks: int = None) -> np.ndarray:
    """a grid x grid PU grid, every block once per active model, seeded window
    centres (integer MVs within +-32 px, 1/16 units)."""
    from . import ME_BLOCK_DTYPE
    rng = np.random.default_rng(0x4D4D2000 + seed)
    rows = []
    for y in range(0, height, grid):
        for x in range(0, width, grid):
            for m in models:
                mvx, mvy = (int(v) * 16 for v in rng.integers(-32, 33, size=2))
                rows.append((x, y, grid, grid, mvx, mvy, int(m), ref_poc, sub_shift))
    out = np.array(rows, dtype=ME_BLOCK_DTYPE)
    if max_blocks is not None and len(out) > max_blocks:
        out = out[rng.choice(len(out), size=max_blocks, replace=False)]
    return out


def dmvr_pu_list(cfg: Config, frame: int = 0, ctu: int = 128) -> np.ndarray:
    """MM-DMVR PUs: the seeded CTU split's leaves that satisfy the
    descriptor part of PU::checkDMVRCondition (w, h >= 8, w*h >= 128), bi-predicted from POCs 0
    and 16 (equal distances around POC 8) with one model for both lists; not pre-split -- DMVR
    splits into <= 16x16 sub-PUs itself."""
    rng = np.random.default_rng(0x4D4D3000 + 977 * frame + cfg.width)
    leaves: List[Tuple[int, int, int, int]] = []
    for y0 in range(0, cfg.height, ctu):
        for x0 in range(0, cfg.width, ctu):
            _split_ctu(rng, x0, y0, min(ctu, cfg.width - x0), min(ctu, cfg.height - y0), leaves)
    rows = []
    for (x, y, w, h) in leaves:
        if w < 8 or h < 8 or w * h < 128:
            continue
        m = int(cfg.models[rng.integers(0, len(cfg.models))])
        mv0 = [int(rng.integers(-24, 25)) * 16 + int(rng.integers(0, 16)),
               int(rng.integers(-24, 25)) * 16 + int(rng.integers(0, 16))]
        mv1 = [-mv0[0] + int(rng.integers(-8, 9)), -mv0[1] + int(rng.integers(-8, 9))]
        rows.append((x, y, w, h, [mv0, mv1], (REF_POCS[0], REF_POCS[1]), (m, m)))
    from . import PU_DTYPE
    out = new_pus(len(rows))
    for i, (x, y, w, h, mvs, refs, ms) in enumerate(rows):
        out[i]["x"], out[i]["y"], out[i]["w"], out[i]["h"] = x, y, w, h
        out[i]["mv"] = np.array(mvs, dtype=np.int32)
        out[i]["ref_poc"] = refs
        out[i]["model"] = ms
    return out


def mvp_queries(width: int, height: int, models: Sequence[int], n: int, seed: int = 7) -> np.ndarray:
    """Seeded MM-MVP conversions: every ordered pair of {CLASSIC} + models,
    neighbour positions around random current blocks (incl. the poles and the ERP seam), MVs in
    1/16 pel, some zero MVs and identical model pairs (the early returns)."""
    from . import MVP_QUERY_DTYPE
    rng = np.random.default_rng(0x4D4D4000 + seed)
    allm = [0] + [int(m) for m in models]
    q = np.zeros(n, dtype=MVP_QUERY_DTYPE)
    for i in range(n):
        w, h = [int(v) for v in rng.choice([8, 16, 32, 64], size=2)]
        x = int(rng.integers(0, width // 4)) * 4
        y = int(rng.integers(0, height // 4)) * 4
        if i % 11 == 0:
            y = 0 if i % 2 else height - 4  # poles
        if i % 13 == 0:
            x = width - 4  # seam
        cw, ch = [int(v) for v in rng.choice([8, 16, 32], size=2)]
        cx, cy = x - cw, y - ch  # candidate: above-left neighbour
        mv = [int(v) for v in rng.integers(-64 * 16, 64 * 16, size=2)]
        if i % 17 == 0:
            mv = [0, 0]
        mo, md = int(rng.choice(allm)), int(rng.choice(allm))
        shift = 4 if i % 5 else 2
        q[i] = (x, y, mv[0], mv[1], mo, md, shift, shift, CUR_POC, REF_POCS[i % 2], CUR_POC, REF_POCS[(i // 2) % 2],
                cx, cy, cw, ch, x, y, w, h)
    return q


# MM-DMVR decision branches (InterPrediction.cpp:2516-2531 early exit, :2576-2580 border best,
# xSubPelErrorSrfc :1996-2048 division / half-pel tie / zero denominator).  The ERP-like planes
# above carry independent noise per POC, so the centre cost never falls below dx * dy and the
# 25 costs almost never tie.  These content families make every branch reachable: identical
# reference pictures (early exits when both lists' positions coincide), and piecewise-flat
# content (costs on a coarse lattice: ties and zero denominators).
DMVR_FAMILIES = ("steps", "sparse", "flatdots", "erp_same")


def dmvr_branch_planes(family: str, width: int, height: int, poc: int, bit_depth: int = 10):
    """Reference planes (Y, Cb, Cr) of one DMVR branch family.  Every family gives POCs 0 and 16
    the same content, except `sparse`, whose POC-16 dots are drawn independently."""
    def plane(w, h, salt):
        rng = np.random.default_rng(0x4D4D6000 + salt + (17 * poc if family == "sparse" else 0))
        y, x = np.mgrid[0:h, 0:w].astype(np.float64)
        if family == "steps":
            v = 400 + 8 * np.floor(x / 5) + 4 * np.floor(y / 7)
        elif family == "sparse":
            v = 500 + 64 * (rng.random((h, w)) < 0.02)
        elif family == "flatdots":
            v = np.full((h, w), 500.0)
            v[::9, ::11] += 40
        elif family == "erp_same":
            v = ref_planes(width, height, 0, bit_depth)[0 if salt == 0 else salt].astype(np.float64)
        else:
            raise ValueError(family)
        return np.clip(np.rint(v), 0, (1 << bit_depth) - 1).astype(np.int16)

    return plane(width, height, 0), plane(width // 2, height // 2, 1), plane(width // 2, height // 2, 2)


def dmvr_branch_candidates(family: str, width: int, height: int, models: Sequence[int], seed: int) -> np.ndarray:
    """One DMVR candidate PU per 16x16 cell of the picture (16x16, 16x8 or 8x16 at the cell origin,
    bi from POCs 0 / 16, one model for both lists), with the motion pattern that reaches the
    family's branches: equal MVs on identical content (early exits), mirrored integer MVs, or
    small independent MVs (costs near the threshold)."""
    rng = np.random.default_rng(0x4D4D7000 + 131 * seed + DMVR_FAMILIES.index(family))
    cells = [(x, y) for y in range(0, height, 16) for x in range(0, width, 16)]
    out = new_pus(len(cells))
    for i, (x, y) in enumerate(cells):
        r = rng.random()
        w, h = (16, 16) if r < 0.7 else ((16, 8) if r < 0.85 else (8, 16))
        m = int(models[rng.integers(0, len(models))])
        kind = rng.random()
        if family == "erp_same" and kind < 0.6:
            mv0 = [int(rng.integers(-64, 65)), int(rng.integers(-64, 65))]
            mv1 = list(mv0)
            if kind < 0.2:  # one list a quarter sample off: costs just around dx * dy
                mv1[int(rng.integers(0, 2))] += int(rng.choice([-4, 4]))
        elif family in ("sparse", "flatdots") or kind < 0.5:
            mv0 = [int(rng.integers(-3, 4)) * 16, int(rng.integers(-3, 4)) * 16]
            mv1 = [-mv0[0], -mv0[1]]
        else:
            mv0 = [int(rng.integers(-20, 21)), int(rng.integers(-20, 21))]
            mv1 = [int(rng.integers(-20, 21)), int(rng.integers(-20, 21))]
        out[i]["x"], out[i]["y"], out[i]["w"], out[i]["h"] = x, y, w, h
        out[i]["mv"] = np.array([mv0, mv1], dtype=np.int32)
        out[i]["ref_poc"] = REF_POCS
        out[i]["model"] = (m, m)
    return out
