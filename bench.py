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


def measured_traffic(args):
    """HBM bytes per k_mc_dev launch from the committed rocprofv3 FETCH_SIZE / WRITE_SIZE passes
    (profiles/r01_traffic.json, tools/traffic_json.py), only when that profile was taken with
    this very library (sha256) and the C3 workload; else None."""
    import hashlib
    path = os.path.join(ROOT, "profiles", "r01_traffic.json")
    if args.config != "C3" or args.uniform_model is not None or args.coherent_mv or not os.path.exists(path):
        return None
    d = json.load(open(path))
    sha = hashlib.sha256(open(mm360.LIB_PATH, "rb").read()).hexdigest()
    return d["traffic_bytes_per_launch"] if d.get("lib_sha256") == sha else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="length of the CPU baseline sample")
    ap.add_argument("--kernel-steps", type=int, default=10, help="extra steps timed per launch with HIP events")
    ap.add_argument("--lib", default=None, help="alternative build of libmm360.so (A/B experiments)")
    ap.add_argument("--stripes", type=int, default=None, help="mm_set_stripes (default: the library's)")
    ap.add_argument("--coherent-mv", action="store_true",
                    help="experiment: one MV for every PU and list (spatially coherent motion)")
    ap.add_argument("--uniform-model", type=int, default=None,
                    help="per-model workload: all PUs 16x16 with this MotionModelID (SURVEY 8(d))")
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
    if args.config == "C5":
        return bench_me(args, cfg, params, rank, world, local, dist)
    if args.uniform_model is not None:
        pus = W.pu_list(cfg, frame=rank, uniform=True, uniform_model=args.uniform_model)
    else:
        pus = W.pu_list(cfg, frame=rank)
    if args.coherent_mv:
        pus["mv"][:, 0, :] = (85, -43)
        pus["mv"][:, 1, :] = (-37, 91)
    area = W.luma_area(pus)
    alg_bytes = W.algorithmic_bytes(pus)

    ctx = mm360.MMContext(params, device=local)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    if args.stripes:
        ctx.set_stripes(args.stripes)
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
        # bounded sample of the same workload, ~10 s on one host thread: the PU lists of
        # consecutive synthetic pictures (frames 0, 1, ...) of this configuration
        from oracle.oracle import Oracle
        refs = {poc: W.ref_planes(cfg.width, cfg.height, poc) for poc in W.REF_POCS}
        orc = Oracle(params, [(W.CUR_POC, -1, W.GED_EPIPOLE_Q24)])
        done_area, cpu_s, frames = 0, 0.0, 0
        while cpu_s < args.cpu_seconds:
            fp = pus if frames == 0 else W.pu_list(cfg, frame=frames)
            t = time.perf_counter()
            orc.predict(W.CUR_POC, fp, refs, cfg.width, cfg.height)
            cpu_s += time.perf_counter() - t
            done_area += W.luma_area(fp)
            frames += 1
        cpu = {"value": round(done_area / cpu_s / 1e6, 3), "unit": "Mpixels/s", "cores": 1, "kind": "port",
               "sample": f"{frames} full {cfg.width}x{cfg.height} pictures (seeded PU lists of frames 0..{frames - 1}) "
                         f"through the oracle (oracle/mm_oracle.c, array-at-a-time restatement, glibc libm + SSE "
                         f"packets), single thread, {cpu_s:.1f} s incl. reference padding"}

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
            "config": {"workload": f"{args.config}: {cfg.description}" + (
                           f" [uniform 16x16 PUs, model {mm360.MODEL_NAMES[args.uniform_model]}]"
                           if args.uniform_model is not None else ""), "width": cfg.width, "height": cfg.height,
                       "pus": int(len(pus)), "luma_area": int(area), "models": [mm360.MODEL_NAMES[m] for m in cfg.models],
                       "parallelism": f"replicas x{world} (one picture per GPU)"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": measured_traffic(args),
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


def bench_me(args, cfg, params, rank, world, local, dist):
    """C5: encoder ME candidate evaluation -- every block of the 16x16 PU grid once per model, a
    33x33 integer window each, reprojection + 8-tap + SAD per candidate (mm_sad_window).  Each
    rank evaluates its own picture's windows (weak scaling)."""
    blocks = W.me_blocks(cfg.width, cfg.height, cfg.models, grid=16, seed=5 + rank)
    C = (2 * W.ME_RANGE + 1) ** 2
    n_cand = len(blocks) * C
    cand_px = int((blocks["w"].astype(np.int64) * blocks["h"]).sum()) * C
    ctx = mm360.MMContext(params, device=local)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    ctx.set_epipole(W.CUR_POC, -1, W.GED_EPIPOLE_Q24)
    for poc in W.REF_POCS:
        y, cb, cr = W.ref_planes(cfg.width, cfg.height, poc)
        ctx.upload_ref(poc, torch.from_numpy(y).cuda(), torch.from_numpy(cb).cuda(), torch.from_numpy(cr).cuda())
    ctx.upload_org(W.CUR_POC, torch.from_numpy(W.org_plane(cfg.width, cfg.height)).cuda())
    sads = torch.zeros((len(blocks), C), dtype=torch.int32, device="cuda")
    for _ in range(args.warmup):
        ctx.sad_window(W.CUR_POC, blocks, W.ME_RANGE, 16, out=sads)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kms = []
    for _ in range(args.steps):
        ctx.sad_window(W.CUR_POC, blocks, W.ME_RANGE, 16, out=sads)
        kms.append(ctx.last_timing_ms())
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    total = float(n_cand)
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        at = torch.tensor([total], dtype=torch.float64, device="cuda")
        dist.all_reduce(at, op=dist.ReduceOp.SUM)
        total = float(at.item())
    kernel_ms = float(np.mean(kms))
    alg_bytes = cand_px * 4  # read ref 2 B + read org 2 B per candidate pixel
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle.oracle import Oracle
        refs = {poc: W.ref_planes(cfg.width, cfg.height, poc)[0] for poc in W.REF_POCS}
        org = W.org_plane(cfg.width, cfg.height)
        sample = W.me_blocks(cfg.width, cfg.height, cfg.models, grid=16, seed=5,
                             max_blocks=max(14, int(14 * args.cpu_seconds / 0.06)))
        orc = Oracle(params, [(W.CUR_POC, -1, W.GED_EPIPOLE_Q24)])
        t = time.perf_counter()
        orc.sad_window(W.CUR_POC, sample, W.ME_RANGE, 16, refs, org)
        cpu_s = time.perf_counter() - t
        cpu = {"value": round(len(sample) * C / cpu_s / 1e6, 4), "unit": "Mcandidates/s", "cores": 1, "kind": "port",
               "sample": f"{len(sample)} blocks x {C} candidates of the same workload through the oracle "
                         f"(oracle/mm_oracle.c), single thread, {cpu_s:.2f} s"}
    if rank == 0:
        print(json.dumps({
            "metric": "MM encoder ME candidate evaluations/s (reprojection + 8-tap + SAD) on 2048x1024 ERP",
            "value": round(total * args.steps / elapsed / 1e6, 3),
            "unit": "Mcandidates/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32+int16",
            "data": "synthetic (seeded ERP planes, seeded window centres, SURVEY 8(d) C5)",
            "config": {"workload": f"C5: {cfg.description}", "width": cfg.width, "height": cfg.height,
                       "blocks": int(len(blocks)), "candidates": int(n_cand), "candidate_luma_px": int(cand_px),
                       "models": [mm360.MODEL_NAMES[m] for m in cfg.models],
                       "parallelism": f"replicas x{world} (one picture per GPU)"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                         "kernel": "mm_sad_window (k_me_setup + k_me_sad)", "kernel_ms": round(kernel_ms, 3),
                         "algorithmic_bytes": int(alg_bytes)},
            "cpu_baseline": cpu,
        }), flush=True)
    ctx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
