"""One mm_pred_dmvr call on the test suite's DMVR workload (tests/test_gpu.py
test_pred_dmvr_vs_oracle) with a chosen library build: debugging aid for A/B builds.
  python tools/dmvr_probe.py --lib ab_variants/X/libmm360.so --size 1024x512 [--check]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vvc-extension-mm_amd"), ROOT, os.path.join(ROOT, "tests")]

import mm360  # noqa: E402
from mm360 import workload as W  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=None)
ap.add_argument("--size", default="1024x512", help="one or more WxH, comma-separated, run in order in one process")
ap.add_argument("--repeat", type=int, default=1)
ap.add_argument("--check", action="store_true", help="compare the deltas with the oracle")
a = ap.parse_args()
if a.lib:
    mm360.LIB_PATH = os.path.abspath(a.lib)
import torch  # noqa: E402
from helpers import EPI  # noqa: E402

def run(size):
    w, h = (int(v) for v in size.split("x"))
    models = W.MPA3 + (mm360.TANGENTIAL, mm360.THREE_D_TRANSLATIONAL, mm360.ROTATIONAL, mm360.GEODESIC_CAMPOSE)
    cfg = W.Config("T", w, h, models, 1, "probe")
    params = mm360.seq_params(w, h, models)
    pus = W.dmvr_pu_list(cfg, frame=2)
    refs = {poc: W.ref_planes(w, h, poc) for poc in W.REF_POCS}
    with mm360.MMContext(params, device=0) as ctx:
        for cur, ref, q in EPI:
            ctx.set_epipole(cur, ref, q)
        for poc, (y, cb, cr) in refs.items():
            ctx.upload_ref(poc, y, cb, cr)
        dst = (torch.zeros((h, w), dtype=torch.int16, device="cuda"),
               torch.zeros((h // 2, w // 2), dtype=torch.int16, device="cuda"),
               torch.zeros((h // 2, w // 2), dtype=torch.int16, device="cuda"))
        for r in range(a.repeat):
            mvd = ctx.predict_dmvr(W.CUR_POC, pus, *dst)
            torch.cuda.synchronize()
            print(f"{size} call {r} ok: {len(pus)} PUs, {len(mvd)} sub-PUs", flush=True)
    if a.check:
        from oracle.oracle import Oracle
        _, want = Oracle(params, EPI).predict_dmvr(W.CUR_POC, pus, refs, w, h)
        print("mvd mismatches:", int((mvd != want).any(axis=1).sum()), flush=True)


for size in a.size.split(","):
    run(size)
