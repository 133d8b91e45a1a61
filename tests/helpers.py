"""Shared helpers for the test suites."""
import os

import numpy as np

import mm360
from mm360 import workload as W

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
EPI = [(W.CUR_POC, -1, W.GED_EPIPOLE_Q24), (-1, -1, (0, 1 << 24, 1 << 23))]


def load_blocks(npz):
    return np.ascontiguousarray(npz["blocks"]).view(mm360.BLOCK_DTYPE).reshape(-1)


def load_pus(npz):
    """Fixture PUs: the first 12 int32 words of mm_pu_desc (x, y, w, h, mv, ref_poc, model) per row;
    bcw_idx = BCW_DEFAULT."""
    words = np.ascontiguousarray(npz["pus"], dtype=np.int32)
    out = mm360.new_pus(len(words))
    out.view(np.int32).reshape(len(words), -1)[:, :12] = words[:, :12]
    return out


def block_offsets(blocks):
    sb = np.where(blocks["comp"] != 0, 2, 4)
    n = (blocks["w"] // sb) * (blocks["h"] // sb)
    return np.concatenate([[0], np.cumsum(n)])


def describe_mismatch(blocks, a, b, limit=3):
    off = block_offsets(blocks)
    diff = np.any(a != b, axis=1)
    bad = [i for i in range(len(blocks)) if diff[off[i]:off[i + 1]].any()]
    lines = [f"{len(bad)} blocks differ"]
    for i in bad[:limit]:
        lines.append(f"block {blocks[i]} first: {a[off[i]:off[i+1]][:2].tolist()} vs {b[off[i]:off[i+1]][:2].tolist()}")
    return "\n".join(lines)


def dmvr_zero_mv_pus(cfg, models, frame=3):
    """DMVR PUs (workload.dmvr_pu_list) re-aimed so that search offsets land on a zero MV -- merge
    (16, 0): offset (-1, 0) of L0 / (+1, 0) of L1; merge (-32, 16): offset (+2, -1) -- or the merge
    MVs are zero themselves (an identity centre setup), every model in turn; every fourth PU keeps
    its random MVs."""
    pus = W.dmvr_pu_list(cfg, frame=frame)
    aims = ([16, 0], [-32, 16], [0, 0])
    for i in range(len(pus)):
        if i % 4 == 3:
            continue
        mv0 = aims[i % 4]
        pus[i]["mv"] = np.array([mv0, [-mv0[0], -mv0[1]]], dtype=np.int32)
        pus[i]["model"] = (int(models[i % len(models)]),) * 2
    return pus
