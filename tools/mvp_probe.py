"""Debug aid: k_mvp_dev device time for the seeded C3 query mix vs the same queries sorted by
(candidate model, desired model), vs one model pair only -- does the kernel pay for running many
models' code in one launch?  python tools/mvp_probe.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vvc-extension-mm_amd"), ROOT]
import mm360  # noqa: E402
import torch  # noqa: E402
from mm360 import workload as W  # noqa: E402

cfg = W.CONFIGS["C3"]
params = mm360.seq_params(cfg.width, cfg.height, cfg.models)
ctx = mm360.MMContext(params, device=0)
ctx.set_epipole(W.CUR_POC, -1, W.GED_EPIPOLE_Q24)
q = np.resize(W.mvp_queries(cfg.width, cfg.height, cfg.models, 20000, seed=5), 155894)


def timeit(qq, name):
    d_q = mm360.queries_to_device(qq)
    d_o = torch.zeros((len(qq), 2), dtype=torch.int32, device="cuda")
    ctx.mvp_convert_device(d_q, d_o)
    ctx.mvp_status()
    t = []
    for _ in range(10):
        ctx.mvp_convert_device(d_q, d_o)
        t.append(ctx.last_timing_ms())
    ctx.mvp_status()
    print(f"{name:40s} {len(qq):7d} queries  {np.median(t) * 1e3:8.1f} us", flush=True)


timeit(q, "mixed (bench order)")
o = np.lexsort((q["model_desired"], q["model_orig"]))
timeit(q[o], "sorted by (orig, desired) model")
for mo, md in ((4, 4), (10, 10), (1, 4), (4, 10)):
    sel = q[(q["model_orig"] == mo) & (q["model_desired"] == md)]
    timeit(np.resize(sel, len(q)), f"only ({mo}, {md}) tiled to the same count")
