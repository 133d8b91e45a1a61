"""How much each unverifiable Eigen 3.3.7 belief matters at C3: the CPU twin
(product headers) built in each alternative numerics mode, against the default build, on the C3
picture (frame 0): sub-block reprojection results that change, PUs with any changed sample, and
changed predicted samples.  Writes a markdown table (DESIGN 2 quotes it).

    python tools/numerics_sensitivity.py [out.txt]
"""
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(ROOT, "vvc-extension-mm_amd"), ROOT, os.path.join(ROOT, "tests", "native")]
import mm360  # noqa: E402
import twin  # noqa: E402
from mm360 import workload as W  # noqa: E402

MODES = [("round", "ROUND: packet lanes round ties-to-even (pround) instead of std::round"),
         ("prod3", "PROD3: 3x3 product coefficient (p0 + p1) + p2 instead of p0 + (p1 + p2)"),
         ("tanc", "TAN_CENTRE: float sinf/cosf instead of double sin/cos for the TAN centre"),
         ("psqrt", "PSQRT: IEEE sqrt instead of rsqrtps + 1 Newton step")]


def blocks_of(pus):
    rows = []
    for u in pus:
        for l in range(2):
            if u["ref_poc"][l] < 0:
                continue
            for comp in (0, 1):
                cs = comp
                rows.append((u["x"] >> cs, u["y"] >> cs, u["w"] >> cs, u["h"] >> cs, u["mv"][l][0], u["mv"][l][1],
                             u["model"][l], comp, W.CUR_POC, u["ref_poc"][l]))
    return np.array(rows, dtype=mm360.BLOCK_DTYPE)


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else None
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tests", "native"), "variants"])
    cfg = W.CONFIGS["C3"]
    params = mm360.seq_params(cfg.width, cfg.height, cfg.models)
    pus = W.pu_list(cfg, frame=0)
    refs = {poc: W.ref_planes(cfg.width, cfg.height, poc) for poc in W.REF_POCS}
    epi = [(W.CUR_POC, -1, W.GED_EPIPOLE_Q24)]
    blocks = blocks_of(pus)
    sb = np.where(blocks["comp"] != 0, 2, 4)
    n_elem = (blocks["w"] // sb) * (blocks["h"] // sb)
    owner = np.repeat(np.arange(len(blocks)), n_elem)
    twin.use_variant(None)
    base_r = twin.reproject(params, blocks, epi)
    base_p = twin.predict(params, W.CUR_POC, pus, refs, cfg.width, cfg.height, epi)
    lines = [f"C3 picture (frame 0): {len(pus)} PUs, {len(blocks)} reprojection blocks, {len(base_r)} sub-block "
             f"results, {cfg.width * cfg.height * 3 // 2} predicted samples (Y+Cb+Cr)", "",
             "| Mode (alternative to the default belief) | sub-block results changed | blocks changed | "
             "predicted samples changed (Y / Cb / Cr) |", "|---|---|---|---|"]
    for mode, desc in MODES:
        t0 = time.time()
        twin.use_variant(mode)
        r = twin.reproject(params, blocks, epi)
        p = twin.predict(params, W.CUR_POC, pus, refs, cfg.width, cfg.height, epi)
        diff = np.any(r != base_r, axis=1)
        nb = len(np.unique(owner[diff]))
        ps = [int((a != b).sum()) for a, b in zip(p, base_p)]
        lines.append(f"| {desc} | {int(diff.sum())} ({diff.mean() * 100:.4f} %) | {nb} | {ps[0]} / {ps[1]} / {ps[2]} |")
        print(lines[-1], f"({time.time() - t0:.0f} s)", flush=True)
    twin.use_variant(None)
    text = "\n".join(lines) + "\n"
    print(text)
    if out:
        open(out, "w").write(text)


if __name__ == "__main__":
    main()
