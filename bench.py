"""Benchmark: MC+reprojection Mpixels/s on 6144x3072 ERP (BASELINE.json metric, config C3).

One step = one pass of the MM motion-compensation path over one picture's PU list: device-side
planning (PU classification + validation, job bucketing), the per-block setup, the per-sub-block
reprojection of every (PU, list, component) and the 8-tap / 4-tap interpolation + bi-averaging
of every predicted sample, for a synthetic 6144x3072 10-bit 4:2:0 ERP picture whose PU list uses
all five motion models (MPA x3, TAN, 3DT, ROT, GED_CAMPOSE).  Inputs (reference planes, the PU
descriptor list) are resident in HBM before the timed region; nothing is planned on the host.

roofline: the dominant kernel is k_mc (interpolation + averaging); its algorithmic bytes (SURVEY
8(d): 6 B uni / 9 B bi per luma pixel) over its per-launch device time, measured with HIP events
on the context stream (mm_last_stage_timing).

    python bench.py [--gpus N] [--steps K] [--warmup W]

Multi-GPU (torch.distributed.run, one rank per GPU): every rank predicts its own picture (PU
list of frame = rank) from its own resident references -- independent pictures, no data-path
collective ("scaling": "weak"); value = pictures' luma area of all ranks / max-over-ranks time.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "vvc-extension-mm_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import mm360  # noqa: E402
from mm360 import workload as W  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--kernel-steps", type=int, default=10, help="extra steps timed per launch with HIP events")
    ap.add_argument("--lib", default=None, help="alternative build of libmm360.so (A/B experiments)")
    args = ap.parse_args()

    if args.lib:
        mm360.LIB_PATH = os.path.abspath(args.lib)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl")
    torch.cuda.set_device(local)

    cfg = W.CONFIGS[args.config]
    params = mm360.seq_params(cfg.width, cfg.height, cfg.models)
    pus = W.pu_list(cfg, frame=rank)
    area = W.luma_area(pus)
    alg_bytes = W.algorithmic_bytes(pus)

    ctx = mm360.MMContext(params, device=local)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    ctx.set_epipole(W.CUR_POC, -1, W.GED_EPIPOLE_Q24)
    for poc in W.REF_POCS:
        y, cb, cr = W.ref_planes(cfg.width, cfg.height, poc)
        ctx.upload_ref(poc, torch.from_numpy(y).cuda(), torch.from_numpy(cb).cuda(), torch.from_numpy(cr).cuda())
    dy = torch.zeros((cfg.height, cfg.width), dtype=torch.int16, device="cuda")
    dcb = torch.zeros((cfg.height // 2, cfg.width // 2), dtype=torch.int16, device="cuda")
    dcr = torch.zeros_like(dcb)
    ctx.prepare(W.CUR_POC, pus)  # PU descriptors -> HBM (outside the timed region)

    for _ in range(args.warmup):
        ctx.run(dy, dcb, dcr)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.run(dy, dcb, dcr)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        at = torch.tensor([area], dtype=torch.float64, device="cuda")
        dist.all_reduce(at, op=dist.ReduceOp.SUM)
        total_area = float(at.item())
    else:
        total_area = float(area)

    ctx.synchronize()  # raises if the device planner rejected a PU
    # per-launch device time of each stage (HIP events between the launches on the context stream)
    ctx.set_stage_timing(True)
    stages = []
    for _ in range(args.kernel_steps):
        ctx.run(dy, dcb, dcr)
        stages.append(ctx.last_stage_timing_ms())
    ctx.set_stage_timing(False)
    st = np.mean(np.array(stages), axis=0)
    kernel_ms = float(st[3])
    pipeline_ms = float(st.sum())

    ms_per_step = elapsed / args.steps * 1e3
    value = total_area * args.steps / elapsed / 1e6
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle.oracle import Oracle
        refs = {poc: W.ref_planes(cfg.width, cfg.height, poc) for poc in W.REF_POCS}
        orc = Oracle(params, [(W.CUR_POC, -1, W.GED_EPIPOLE_Q24)])
        t = time.perf_counter()
        orc.predict(W.CUR_POC, pus, refs, cfg.width, cfg.height)
        cpu_s = time.perf_counter() - t
        cpu = {"value": round(area / cpu_s / 1e6, 3), "unit": "Mpixels/s", "cores": 1, "kind": "port",
               "sample": f"one full {cfg.width}x{cfg.height} picture ({len(pus)} PUs) through the oracle "
                         f"(oracle/mm_oracle.c, array-at-a-time restatement, glibc libm + SSE packets), "
                         f"single thread, {cpu_s:.2f} s incl. reference padding"}

    if rank == 0:
        line = {
            "metric": "MC+reprojection Mpixels/s on 6144x3072 ERP; bit-exact vs VTM CPU",
            "value": round(value, 2),
            "unit": "Mpixels/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32+int16",
            "data": "synthetic (seeded ERP planes + PU lists, SURVEY 8(d))",
            "config": {"workload": f"{args.config}: {cfg.description}", "width": cfg.width, "height": cfg.height,
                       "pus": int(len(pus)), "luma_area": int(area), "models": [mm360.MODEL_NAMES[m] for m in cfg.models],
                       "parallelism": f"replicas x{world} (one picture per GPU)"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                         "kernel": "k_mc_dev", "kernel_ms": round(kernel_ms, 4),
                         "algorithmic_bytes": int(alg_bytes)},
            "stages_ms": {"plan": round(float(st[0]), 4), "setup": round(float(st[1]), 4),
                          "reproj": round(float(st[2]), 4), "mc": round(float(st[3]), 4),
                          "pipeline": round(pipeline_ms, 4)},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    ctx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
