"""Generate tests/golden/dmvr_branches.npz: MM-DMVR PU lists that reach every branch of the
decision (InterPrediction.cpp:2516-2531 early exit, :2567-2580 border best, xSubPelErrorSrfc
:1996-2048 division / half-pel tie on either side / zero denominator), with the oracle's refined
deltas and branch words as the expected outputs.

For each content family (mm360.workload.DMVR_FAMILIES, 512x256, all models) the script draws
ROUNDS candidate lists (one PU per 16x16 cell), traces the oracle's decision of every candidate,
and fills the cells class by class, rarest first, up to a quota per class -- a picture of non-overlapping PUs
whose branch counts the tests assert.  Inputs are regenerated from the family name and the
seeded candidates; the fixture holds the chosen PU records and the expected outputs.

    python tools/gen_dmvr_branch_fixture.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vvc-extension-mm_amd"), ROOT]

import mm360  # noqa: E402
from mm360 import workload as W  # noqa: E402
from oracle.oracle import Oracle, dmvr_branches  # noqa: E402

WIDTH, HEIGHT, ROUNDS, QUOTA = 512, 256, 40, 80
EPI = [(W.CUR_POC, -1, W.GED_EPIPOLE_Q24)]


def rank(tr):
    """Lower = rarer branch class of one traced sub-PU."""
    if tr & 1:
        return 4  # early exit
    if tr & 64:
        return 6  # border best
    cases = ((tr >> 8) & 3, (tr >> 10) & 3)
    if 0 in cases:
        return 0  # zero denominator
    if 2 in cases:
        return 1  # tie on the -1 side
    if 3 in cases:
        return 2  # tie on the +1 side
    return 3 if ((tr >> 1) & 31) == 12 else 5


def main():
    models = W.ALL_MODELS
    params = mm360.seq_params(WIDTH, HEIGHT, models)
    orc = Oracle(params, EPI)
    out = {"width": WIDTH, "height": HEIGHT, "models": np.array(models, dtype=np.int32),
           "families": np.array(W.DMVR_FAMILIES)}
    for fam in W.DMVR_FAMILIES:
        refs = {poc: W.dmvr_branch_planes(fam, WIDTH, HEIGHT, poc) for poc in W.REF_POCS}
        cands, ranks = [], []
        for r in range(ROUNDS):
            cand = W.dmvr_branch_candidates(fam, WIDTH, HEIGHT, models, seed=r)
            _, _, tr = orc.predict_dmvr(W.CUR_POC, cand, refs, WIDTH, HEIGHT, trace=True)
            # 16x16 / 16x8 / 8x16 PUs are one sub-PU each: one trace word per cell
            cands.append(cand)
            ranks.append(np.array([rank(int(t)) for t in tr]))
        ranks = np.stack(ranks)  # [round, cell]
        # greedy quota per class, rarest first: up to QUOTA cells take a candidate of the class
        best = cands[0].copy()
        free = np.ones(ranks.shape[1], dtype=bool)
        for cls in range(7):
            hit = np.argwhere((ranks == cls) & free[None, :])
            taken = 0
            for r, c in hit:
                if taken >= QUOTA or not free[c]:
                    continue
                best[c] = cands[r][c]
                free[c] = False
                taken += 1
        _, mvd, tr = orc.predict_dmvr(W.CUR_POC, best, refs, WIDTH, HEIGHT, trace=True)
        out[f"{fam}_pus"] = best
        out[f"{fam}_mvd"] = mvd
        out[f"{fam}_trace"] = tr
        print(fam, dmvr_branches(tr))
    path = os.path.join(ROOT, "tests", "golden", "dmvr_branches.npz")
    np.savez_compressed(path, **out)
    print("wrote", path)


if __name__ == "__main__":
    main()
