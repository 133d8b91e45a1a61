"""Benchmark: MC+reprojection Mpixels/s on 6144x3072 ERP (BASELINE.json metric).

One step = one pass of the MM motion-compensation path over one picture's PU list: device-side
planning (PU classification + validation, job bucketing), the per-block setup, the per-sub-block
reprojection of every (PU, list, component) and the 8-tap / 4-tap interpolation + bi-averaging
of every predicted sample, for a synthetic 6144x3072 10-bit 4:2:0 ERP picture whose PU list uses
all five motion models (MPA x3, TAN, 3DT, ROT, GED_CAMPOSE).  Inputs (reference planes, the PU
descriptor lists) are resident in HBM before the timed region; nothing is planned on the host.

Configurations (BASELINE.json configs):
  C3 (default at 1 GPU)  `--pictures` distinct pictures (PU lists of frames 0..P-1), each with its
        own pair of reference pictures (2P resident references, 529 MB of padded pool at P = 4 -- more than the
        256 MB Infinity Cache), predicted in rotation: step s predicts picture s % P.  After
        timing, every picture's output is compared with the CPU oracle (`bit_exact`).
  C4 (default at N > 1 GPUs)  one C3 picture per step, CTU-row sharded: rank r predicts the PUs
        of its stripe (mm360.parallel) straight into its segment of the stripe-major packed
        picture, then ONE in-place RCCL all-gather (Y + Cb + Cr together) rebuilds the picture on
        every rank; picture t's all-gather overlaps picture t+1's prediction (two picture
        buffers).  value = pictures' luma area / max-over-ranks time ("strong" scaling: the
        picture is fixed); `mc_only` is the same loop without the all-gather.
  C5  encoder ME candidate evaluation (Mcandidates/s).

roofline: the dominant kernel is k_mc (interpolation + averaging); its algorithmic bytes (SURVEY
8(d): 6 B uni / 9 B bi per luma pixel) over its per-launch device time, measured with HIP events
on the context stream (mm_last_stage_timing).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C3|C4|C5]
"""
import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "vvc-extension-mm_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import mm360  # noqa: E402
from mm360 import parallel as P  # noqa: E402
from mm360 import workload as W  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "MC+reprojection Mpixels/s on 6144x3072 ERP; bit-exact vs the CPU oracle restatement (parity unpinned)"
POC_STRIDE = 32  # picture f: refs (32 f, 32 f + 16), current POC 32 f + 8
RED_DEVICE = ["cuda"]  # where the timing reductions run: "cpu" under the gloo rehearsal backend


def build_provenance():
    """The measured library's sha256, the tree's source sha256 and whether both match the record
    __graft_entry__.build() wrote when it last recompiled the library (mm360/provenance.py)."""
    from mm360 import provenance
    return provenance.provenance(mm360.LIB_PATH)


def measured_traffic(args, config):
    """HBM bytes per k_mc_dev launch from the committed rocprofv3 FETCH_SIZE / WRITE_SIZE passes
    (profiles/r0N_traffic.json, tools/traffic_json.py), only when that profile was taken with
    this very library (sha256) and the same workload: (bytes, source label), else (None, reason).
    The PMC passes are not run inside the bench: the counters need their own rocprofv3 runs."""
    import glob
    import hashlib
    if config != "C3" or args.uniform_model is not None or args.coherent_mv or args.dmvr_share > 0:
        return None, "no committed profile for this workload"
    sha = hashlib.sha256(open(mm360.LIB_PATH, "rb").read()).hexdigest()
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_traffic.json")), reverse=True):
        d = json.load(open(path))
        if d.get("lib_sha256") == sha and d.get("pictures") == args.pictures:
            return d["traffic_bytes_per_launch"], (f"{os.path.relpath(path, ROOT)} (library sha256 match; "
                                                   f"rocprofv3 FETCH_SIZE / WRITE_SIZE passes, not this run)")
    return None, f"no committed PMC profile of this library (sha256 {sha[:16]})"


def host_info(threads):
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    libc = " ".join(platform.libc_ver())
    return {"cpu_model": model, "nproc": os.cpu_count(), "threads_available": threads, "glibc": libc,
            "threads_note": "the all-threads leg uses one GPU's share of the GPU box's host (16 threads per "
                            "GPU), not the whole machine"}


def cpu_threads():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))  # the GPU box's CPU share is 16 threads per GPU


def picture_set(cfg, n, frame0=0, uniform_model=None, coherent=False, dmvr_share=0.0, dmvr_correlated=False):
    """n pictures: (cur_poc, PU list, {poc: planes}) with disjoint reference pairs.
    dmvr_correlated: both references of a picture carry the same content and the MM_PUF_DMVR PUs
    point both lists at the same place (mv1 = mv0; 30 % of them a quarter sample off in one
    component), so their two predictions agree and the centre cost ends most searches early
    (InterPrediction.cpp:2516-2525), as on content with true bi-directional motion."""
    out = []
    for f in range(n):
        base = POC_STRIDE * (frame0 + f)
        if uniform_model is not None:
            pus = W.pu_list(cfg, frame=frame0 + f, uniform=True, uniform_model=uniform_model)
        else:
            pus = W.pu_list(cfg, frame=frame0 + f, dmvr_share=dmvr_share)
        if coherent:
            pus["mv"][:, 0, :] = (85, -43)
            pus["mv"][:, 1, :] = (-37, 91)
        pus["ref_poc"] = np.where(pus["ref_poc"] >= 0, pus["ref_poc"] + base, -1)
        refs = {base + p: W.ref_planes(cfg.width, cfg.height, base + p) for p in W.REF_POCS}
        if dmvr_correlated:
            p0, p1 = (base + p for p in W.REF_POCS)
            refs[p1] = tuple(x.copy() for x in refs[p0])
            d = np.flatnonzero(W.dmvr_flagged(pus))
            rng = np.random.default_rng(0x4D4D8000 + frame0 + f)
            pus["mv"][d, 1, :] = pus["mv"][d, 0, :]
            off = d[rng.random(len(d)) < 0.3]
            pus["mv"][off, 1, rng.integers(0, 2, size=len(off))] += rng.choice([-4, 4], size=len(off))
        out.append((base + W.CUR_POC, pus, refs))
    return out


def new_ctx(params, local, pictures):
    ctx = mm360.MMContext(params, device=local)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    for cur, _, refs in pictures:
        ctx.set_epipole(cur, -1, W.GED_EPIPOLE_Q24)
        for poc, (y, cb, cr) in refs.items():
            ctx.upload_ref(poc, torch.from_numpy(y).cuda(), torch.from_numpy(cb).cuda(), torch.from_numpy(cr).cuda())
    return ctx


def planes(cfg):
    dy = torch.zeros((cfg.height, cfg.width), dtype=torch.int16, device="cuda")
    dcb = torch.zeros((cfg.height // 2, cfg.width // 2), dtype=torch.int16, device="cuda")
    return dy, dcb, torch.zeros_like(dcb)


def timed(steps, warmup, body, dist, before=None):
    """before(): runs after the warm-up, outside the timed region (e.g. poisons the output buffers
    so that the self-check reads what the timed steps wrote)."""
    for s in range(warmup):
        body(s)
    torch.cuda.synchronize()
    if before is not None:
        before()
        torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(steps):
        body(s)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=RED_DEVICE[0])
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    return elapsed


def cpu_baseline_and_check(args, cfg, params, pictures, gpu_out, n_checked=None):
    """The oracle on the host cores of this box: (a) one thread, as VTM's serial decoder, over a
    bounded sample (~cpu_seconds) of the bench pictures; (b) PU-parallel on all available threads
    (std::thread-style pthreads in the oracle) over the same pictures.  References are padded
    once per picture outside the timing (reported separately).  The all-thread outputs are
    compared with the GPU outputs of every bench picture: bit_exact."""
    from oracle.oracle import Oracle
    orc = Oracle(params, [(cur, -1, W.GED_EPIPOLE_Q24) for cur, _, _ in pictures])
    t = time.perf_counter()
    padded = [orc.padded_refs(refs) for _, _, refs in pictures]
    pad_s = (time.perf_counter() - t) / len(pictures)
    threads = cpu_threads()
    # (b) all threads, every picture once -> bit-exact check (MM_PUF_DMVR PUs: the oracle's serial
    # DMVR restatement after the PU-parallel rest)
    mismatches = 0
    n_checked = len(pictures) if n_checked is None else n_checked
    t_all, area_all = 0.0, 0
    for (cur, pus, refs), pr, got in list(zip(pictures, padded, gpu_out))[:n_checked]:
        t = time.perf_counter()
        want = orc.predict_mixed(cur, pus, refs, cfg.width, cfg.height, prefs=pr, threads=threads)
        t_all += time.perf_counter() - t
        area_all += W.luma_area(pus)
        mismatches += sum(int((g != w).sum()) for g, w in zip(got, want))
    # (a) one thread, bounded sample
    t_one, area_one, n_one = 0.0, 0, 0
    while t_one < args.cpu_seconds:
        cur, pus, refs = pictures[n_one % len(pictures)]
        t = time.perf_counter()
        orc.predict_mixed(cur, pus, refs, cfg.width, cfg.height, prefs=padded[n_one % len(pictures)], threads=1)
        t_one += time.perf_counter() - t
        area_one += W.luma_area(pus)
        n_one += 1
    info = host_info(threads)
    cpu = {"value": round(area_one / t_one / 1e6, 3), "unit": "Mpixels/s", "cores": 1, "kind": "port",
           "sample": f"{n_one} full {cfg.width}x{cfg.height} pictures of the bench workload through the oracle "
                     f"(oracle/mm_oracle.c: array-at-a-time restatement, glibc libm + SSE packets, gcc -O3), "
                     f"one host thread, {t_one:.1f} s; reference padding (extendPicBorder) {pad_s * 1e3:.0f} ms per "
                     f"picture done once outside the timing",
           "all_cores": {"value": round(area_all / t_all / 1e6, 3), "unit": "Mpixels/s", "threads": threads,
                         "share": "per-GPU share of the host (16 threads per GPU on the GPU box)",
                         "sample": f"{len(pictures)} pictures, PU-parallel pthreads, {t_all:.2f} s"},
           "padding_ms_per_picture": round(pad_s * 1e3, 1)}
    cpu.update(info)
    return cpu, mismatches == 0, mismatches


def bench_pictures(args, cfg, params, rank, world, local, dist):
    """C3 (and C2 / uniform-model variants): rotating pictures, one per step."""
    pictures = picture_set(cfg, args.pictures, frame0=rank * args.pictures, uniform_model=args.uniform_model,
                           coherent=args.coherent_mv, dmvr_share=args.dmvr_share,
                           dmvr_correlated=getattr(args, "dmvr_correlated", False))
    ctx = new_ctx(params, local, pictures)
    if args.dmvr_share > 0:
        ctx.set_dmvr(True)
    if args.stripes:
        ctx.set_stripes(args.stripes)
    if args.plan_ahead:
        ctx.set_plan_ahead(True)
    ctx.set_call_timing(False)  # a decoder loop reads no per-call times (stage timing below is separate)
    d_pus = [mm360.pus_to_device(p) for _, p, _ in pictures]
    outs = [planes(cfg) for _ in pictures]
    area = [W.luma_area(p) for _, p, _ in pictures]
    dmvr_area_frac = float(np.mean([W.luma_area(p[W.dmvr_flagged(p)]) / W.luma_area(p) for _, p, _ in pictures]))
    alg = [W.algorithmic_bytes(p) for _, p, _ in pictures]
    P_ = len(pictures)

    def step(s):
        f = s % P_
        ctx.predict_device(pictures[f][0], d_pus[f], *outs[f])

    def poison():
        for o in outs:
            for t in o:
                t.fill_(-1)

    elapsed = timed(args.steps, args.warmup, step, dist, before=poison)
    ctx.synchronize()  # raises if the device planner rejected a PU
    # the timed plan-ahead pictures, copied out before anything else writes the buffers: the
    # bit-exact check below reads these (every sample of a C3 picture is predicted, so a sample the
    # timed steps left unwritten would read -1 and fail the check)
    got = [tuple(t.cpu().numpy() for t in o) for o in outs]
    # k_mc_dev as it runs in the timed loop: the same steps replayed with every k_mc_dev launch
    # bracketed by kernel-bound events (mm_set_kernel_timing: no marker packets; under plan-ahead
    # the stop event is the slot's gate), so its duration includes the overlap with the next
    # picture's planning and reprojection on the auxiliary queue
    loop_k, replay = [], float("nan")
    if hasattr(ctx.lib, "mm_set_kernel_timing"):  # an A/B library (--lib) of an older round may lack it
        ctx.set_kernel_timing(True)
        replay = timed(args.steps, args.warmup, step, None)
        loop_k = ctx.kernel_times_ms()[-args.steps:]
        ctx.set_kernel_timing(False)
    loop_kernel_ms = float(np.mean(loop_k)) if len(loop_k) else None
    steps_area = sum(area[s % P_] for s in range(args.steps))
    total_area = float(steps_area)
    if dist:
        at = torch.tensor([total_area], dtype=torch.float64, device=RED_DEVICE[0])
        dist.all_reduce(at, op=dist.ReduceOp.SUM)
        total_area = float(at.item())
    # per-launch device time of each stage (HIP events between the launches on the context stream)
    ctx.set_stage_timing(True)
    stages = []
    for s in range(args.kernel_steps):
        step(s)
        stages.append(ctx.last_stage_timing_ms())
    ctx.set_stage_timing(False)
    st = np.mean(np.array(stages), axis=0)
    kernel_ms = float(st[3])
    alg_step = float(np.mean([alg[s % P_] for s in range(args.kernel_steps)]))
    alg_loop = float(np.mean([alg[s % P_] for s in range(args.steps)]))
    achieved_iso = alg_step / (kernel_ms * 1e-3) / 1e9
    if loop_kernel_ms is None:
        loop_kernel_ms = kernel_ms
    achieved = alg_loop / (loop_kernel_ms * 1e-3) / 1e9
    traffic, traffic_src = measured_traffic(args, args.config)
    mvp = None
    if args.config == "C3" and not args.no_mvp:
        mvp = mvp_per_picture(ctx, cfg, int(np.mean([list_uses(p) for _, p, _ in pictures])), params,
                              [(cur, -1, W.GED_EPIPOLE_Q24) for cur, _, _ in pictures])
        mvp["in_loop"] = mvp_in_loop(args, ctx, cfg, pictures, d_pus, outs, area)
        sp = mvp["spatial_host"]
        par = sp[f"ms_per_picture_{sp['threads']}_threads"]
        mvp["decoder_bound_ms_per_picture"] = {
            "value": round(max(mvp["in_loop"]["ms_per_picture"], par), 4),
            "note": f"max of the GPU loop with the TMVP batches ({mvp['in_loop']['ms_per_picture']} ms) and the "
                    f"host's spatial conversions on {sp['threads']} threads ({par} ms), which overlap the GPU work "
                    f"of earlier pictures in a decoder"}

    multi = None
    if (args.config == "C3" and world == 1 and args.dmvr_share == 0 and args.uniform_model is None and P_ >= 2
            and not args.no_multi):
        multi = multi_picture_record(args, ctx, pictures, d_pus, area, got)

    cpu, bit_exact, mism = None, None, None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # pictures the timed steps predicted (all of them unless --steps < --pictures)
        cpu, bit_exact, mism = cpu_baseline_and_check(args, cfg, params, pictures, got, min(P_, args.steps))
    if rank == 0:
        line = {
            "metric": METRIC, "value": round(total_area / elapsed / 1e6, 2), "unit": "Mpixels/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32+int16",
            "data": "synthetic (seeded ERP planes + PU lists, SURVEY 8(d))",
            "config": {"workload": f"{args.config}: {cfg.description}" + (
                           f" [uniform 16x16 PUs, model {mm360.MODEL_NAMES[args.uniform_model]}]"
                           if args.uniform_model is not None else "") + (
                           f" [MM-DMVR: {args.dmvr_share:.0%} of the DMVR-eligible bi leaves, "
                           f"{dmvr_area_frac:.1%} of the luma area]" if args.dmvr_share > 0 else ""),
                       "width": cfg.width, "height": cfg.height, "pictures": P_,
                       "pus_per_picture": int(np.mean([len(p) for _, p, _ in pictures])),
                       "luma_area": int(area[0]), "resident_refs": 2 * P_, "plan_ahead": bool(args.plan_ahead),
                       "models": [mm360.MODEL_NAMES[m] for m in cfg.models],
                       "parallelism": "1 GPU" if world == 1 else f"replicas x{world} (own pictures per GPU)"},
            "bit_exact": bit_exact, "mismatching_samples": mism,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": "k_mc_dev", "kernel_ms": round(loop_kernel_ms, 4),
                         "kernel_ms_source": (f"mean of the {len(loop_k)} k_mc_dev launches of a replay of the timed "
                                              f"steps, kernel-bound HIP events on the launch stream "
                                              f"(mm_set_kernel_timing); replay {replay / args.steps * 1e3:.4f} ms "
                                              f"per step vs {elapsed / args.steps * 1e3:.4f} timed"),
                         "algorithmic_bytes": int(alg_loop),
                         "frac_isolated": round(achieved_iso / HBM_PEAK_GBS, 4),
                         "kernel_ms_isolated": round(kernel_ms, 4),
                         "frac_end_to_end": round(alg_loop / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS, 4),
                         "note": "frac: k_mc_dev in the timed plan-ahead loop (beside the next picture's "
                                 "reprojection); frac_isolated: stage-timing pass, stages one after another; "
                                 "frac_end_to_end: algorithmic bytes / ms_per_step"},
            "stages_ms": {"plan": round(float(st[0]), 4), "setup": round(float(st[1]), 4),
                          "reproj": round(float(st[2]), 4), "mc": round(float(st[3]), 4),
                          "pipeline": round(float(st.sum()), 4)},
            "cpu_baseline": cpu,
            "build": build_provenance(),
        }
        if mvp is not None:
            line["mvp"] = mvp
        if multi is not None:
            line["multi_picture"] = multi
        ctx.close()
        return line
    ctx.close()
    return None


def multi_picture_record(args, ctx, pictures, d_pus, area, verified):
    """Beside the headline (not `value`): the same rotating C3 pictures, k = 2 and 4 at a time in
    ONE launch chain (mm_pred_device_multi) -- what a decoder gets for pictures that do not reference
    each other (the leaves of an RA temporal layer, cfg/encoder_randomaccess_vtm.cfg:20-51).  Every
    output equals the headline's own timed output of the same picture (which the bench checks
    against the oracle)."""
    P_ = len(pictures)
    out = {}
    for k in (2, 4):
        if k > P_:
            continue
        outs = [planes(W.CONFIGS[args.config]) for _ in range(P_)]

        def step(s, k=k, outs=outs):
            f0 = (s * k) % P_
            ctx.predict_device_multi([(pictures[(f0 + q) % P_][0], d_pus[(f0 + q) % P_], *outs[(f0 + q) % P_])
                                      for q in range(k)])

        steps = max(2, args.steps // k)
        t = timed(steps, max(1, args.warmup // k), step, None)
        ctx.synchronize()
        same = all(np.array_equal(a.cpu().numpy(), b) for f in range(P_) for a, b in zip(outs[f], verified[f]))
        n_pic = steps * k
        px = sum(area[(s * k + q) % P_] for s in range(steps) for q in range(k))
        out[str(k)] = {"ms_per_picture": round(t / n_pic * 1e3, 4), "value": round(px / t / 1e6, 2),
                       "equals_headline_output": bool(same)}
    out["note"] = ("k independent C3 pictures per mm_pred_device_multi call (one launch chain), plan-ahead as set; "
                   "not part of value: the headline predicts one picture per call")
    return out


def dmvr_record(args, cfg, params, share=0.3, steps=12, warmup=3, correlated=False):
    """C3 with MM-DMVR beside the headline: the same rotating pictures with
    `share` of the DMVR-eligible bi leaves flagged MM_PUF_DMVR (merge / mvRefine PUs), so that each
    picture runs the centre costs, the survivors' 24-offset search and the refined prediction inside
    its own launch sequence (mm_set_dmvr).  Timed like the headline (plan-ahead as set); the timed
    outputs of every picture are checked against the oracle (its serial DMVR restatement)."""
    a = argparse.Namespace(**vars(args))
    a.dmvr_share, a.steps, a.warmup, a.kernel_steps = share, steps, warmup, 2
    a.no_mvp, a.cpu_seconds, a.uniform_model, a.coherent_mv = True, 0.5, None, False
    a.dmvr_correlated = correlated
    line = bench_pictures(a, cfg, params, 0, 1, 0, None)
    cpu = line["cpu_baseline"] or {}
    wl = line["config"]["workload"]
    if correlated:
        wl += (" [correlated references: both lists read the same content at the same place (mv1 = mv0, 30 % "
               "a quarter sample off), so the centre cost ends most searches]")
    return {"workload": wl, "share": share, "value": line["value"], "unit": "Mpixels/s",
            "ms_per_picture": line["ms_per_step"], "steps": steps, "stages_ms": line["stages_ms"],
            "bit_exact": line["bit_exact"], "mismatching_samples": line["mismatching_samples"],
            "bit_exact_sample": f"the {min(a.pictures, steps)} timed pictures vs the oracle",
            "cpu_all_cores_mpix_s": (cpu.get("all_cores") or {}).get("value"),
            "note": "stages_ms.setup holds the DMVR kernels (centre terms and setups, centre costs, the "
                    "survivors' search) and k_setup_dev; not part of value"}


def list_uses(pus):
    """(PU, used list) pairs of a PU list."""
    return int((pus["ref_poc"] >= 0).sum())


def mvp_per_picture(ctx, cfg, n_uses, params, epipoles, reps=10):
    """MM-MVP beside the C3 number, outside its timed region, split the way a
    decoder binds it (MVP): per PU and used list, two spatial candidates (the left and
    above neighbours of addMVPCandUnscaled / the merge list, UnitTools.cpp:2930-2992, 3134-3167) that
    convert a neighbour's FINAL MV and so run one at a time in decoding order on the host
    (mm_mvp_convert_host), and one collocated (TMVP) candidate (UnitTools.cpp:2267-2304) whose
    picture's worth is converted as one device batch (mm_mvp_convert_device, queries and results
    resident in HBM).  Host: one thread over the picture's spatial queries, and 16 threads (the
    per-GPU share of the box's host) each converting a run of CTU rows with its own epipole list --
    the WPP-style parallelism a decoder has -- wall time.  Device: kernel time (HIP events) and wall
    time per call over `reps` back-to-back calls; the synchronous host-buffer call beside it."""
    from concurrent.futures import ThreadPoolExecutor
    n_sp, n_tm = 2 * n_uses, n_uses
    q_sp = np.resize(W.mvp_queries(cfg.width, cfg.height, cfg.models, 20000, seed=3), n_sp)
    q = np.resize(W.mvp_queries(cfg.width, cfg.height, cfg.models, 20000, seed=5), n_tm)
    d_q = mm360.queries_to_device(q)
    d_out = torch.zeros((len(q), 2), dtype=torch.int32, device="cuda")
    ctx.mvp_convert_device(d_q, d_out)  # warm-up (epipole table upload)
    ctx.mvp_status()
    dev = []
    for _ in range(reps):
        ctx.mvp_convert_device(d_q, d_out)
        dev.append(ctx.last_timing_ms())
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        ctx.mvp_convert_device(d_q, d_out)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / reps
    ctx.mvp_status()
    got = d_out.cpu().numpy()  # the last timed call's results
    ctx.mvp_convert(q)  # host-buffer form (warm-up of its buffers)
    host = float("inf")
    for _ in range(3):
        t0 = time.perf_counter()
        ctx.mvp_convert(q)
        host = min(host, time.perf_counter() - t0)
    # spatial candidates on the host: the picture's queries in one call per thread, so the time per
    # query is the conversion's own cost (a C++ decoder calls it per candidate; a ctypes call per query
    # from Python would time the binding instead)
    epi = ctx.epipole_list()
    mm360.mvp_convert_host(params, q_sp[:1000], epi)
    t0 = time.perf_counter()
    host_mv = mm360.mvp_convert_host(params, q_sp, epi)
    host1 = time.perf_counter() - t0
    threads = cpu_threads()
    lists = []
    for _ in range(threads):
        e = mm360.EpipoleList()
        for cur, ref, qq in epipoles:
            e.add(cur, ref, qq, True)
        lists.append(e)
    chunks = np.array_split(np.arange(n_sp), threads)
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(lambda k: mm360.mvp_convert_host(params, q_sp[chunks[k][:100]], lists[k]), range(threads)))
        t0 = time.perf_counter()
        parts = list(ex.map(lambda k: mm360.mvp_convert_host(params, q_sp[chunks[k]], lists[k]), range(threads)))
        host_n = time.perf_counter() - t0
    host_par = np.concatenate(parts)
    # check (after timing): the timed device conversions and both host forms against the oracle
    from oracle.oracle import Oracle
    orc = Oracle(params, epipoles)
    want, want_sp = orc.mvp(q), orc.mvp(q_sp)
    bad = int((got != want).any(axis=1).sum())
    bad_host = int((host_mv != want_sp).any(axis=1).sum()) + int((host_par != want_sp).any(axis=1).sum())
    return {"queries_per_picture": {"spatial": int(n_sp), "tmvp": int(n_tm)},
            "query_model": "per PU and used list: 2 spatial candidates (left, above) converted on the host in "
                           "decoding order + 1 collocated (TMVP) candidate converted in the picture's device batch",
            "spatial_host": {"ms_per_picture_1_thread": round(host1 * 1e3, 3),
                             "us_per_query": round(host1 / n_sp * 1e6, 3),
                             f"ms_per_picture_{threads}_threads": round(host_n * 1e3, 3), "threads": threads,
                             "note": "mm_mvp_convert_host (the product's model bodies compiled for the host, no "
                                     "oracle); the threads split the picture's queries in CTU-row runs, each with "
                                     "its own epipole list (WPP-style); wall time"},
            "tmvp_device": {"ms_per_picture": round(wall * 1e3, 4), "kernel_ms": round(float(np.mean(dev)), 4),
                            "host_buffer_call_ms": round(host * 1e3, 4)},
            "bit_exact": bad == 0 and bad_host == 0, "mismatching_queries": bad + bad_host,
            "bit_exact_sample": "the last timed device batch and both host forms' MVs, vs the oracle",
            "host_per_query_us": round(host1 / n_sp * 1e6, 3), "host_per_query_cores": 1,
            "note": "not part of value; in_loop: C3 with the TMVP batches on their own stream"}


def mvp_in_loop(args, ctx, cfg, pictures, d_pus, outs, area):
    """C3 with MM-MVP in the decode loop: a picture's TMVP conversions (one per PU and used list, one batch)
    run on their own stream (mm_set_mvp_stream), two pictures ahead, while earlier pictures are
    predicted on the context stream; a picture's PU list depends on its conversions, so before its
    prediction call is issued the host waits for them (the plan-ahead contract: a call's list is
    complete when the call is issued; the conversions finished during the previous picture, so the
    wait returns at once): a decoder that derives the next pictures' MVs while the current one is
    motion-compensated.  With plan-ahead off, the prediction waits for its conversions on the
    device instead (an event) and they run one picture ahead.  Also the latency of one CTU row's and one CTU's batch
    (merge lists that chain, UnitTools.cpp:2269-2302, convert in dependent batches): device time of
    the call and host wall time of the synchronous host-buffer call."""
    P_ = len(pictures)
    qs = [np.resize(W.mvp_queries(cfg.width, cfg.height, cfg.models, 20000, seed=11 + f), list_uses(p))
          for f, (_, p, _) in enumerate(pictures)]
    d_q = [mm360.queries_to_device(q) for q in qs]
    d_o = [torch.zeros((len(q), 2), dtype=torch.int32, device="cuda") for q in qs]
    side = torch.cuda.Stream()
    ahead = 2 if args.plan_ahead else 1
    ctx.set_plan_ahead(bool(args.plan_ahead))
    ctx.set_call_timing(False)
    ctx.set_mvp_stream(side.cuda_stream)
    ready = [torch.cuda.Event() for _ in range(P_)]
    main = torch.cuda.current_stream()

    def convert(f):
        ctx.mvp_convert_device(d_q[f], d_o[f])
        ready[f].record(side)

    def step(s):
        f = s % P_
        if s == 0:
            for a in range(ahead):
                convert(a)
        convert((s + ahead) % P_)  # a later picture's MV derivation, overlapping this picture's MC
        if args.plan_ahead:
            ready[f].synchronize()  # the list of call s is complete when the call is issued
        else:
            main.wait_event(ready[f])
        ctx.predict_device(pictures[f][0], d_pus[f], *outs[f])

    elapsed = timed(args.steps, args.warmup, step, None)
    ctx.mvp_status()
    ctx.synchronize()
    ms = elapsed / args.steps * 1e3
    steps_area = sum(area[s % P_] for s in range(args.steps))
    # dependent batches: one CTU row (W / 128 CTUs) and one CTU of conversions
    n_pic = len(qs[0])
    rows = cfg.height // 128
    lat = {}
    ctx.set_mvp_stream(None)
    ctx.set_call_timing(True)
    for name, n in (("ctu_row", max(1, n_pic // rows)), ("ctu", max(1, n_pic // (rows * (cfg.width // 128))))):
        dq, do = d_q[0][:n], d_o[0][:n]  # [queries, 20 words], [queries, 2]
        dev = []
        for _ in range(20):
            ctx.mvp_convert_device(dq, do)
            dev.append(ctx.last_timing_ms())
        ctx.mvp_status()
        host = float("inf")
        for _ in range(20):
            t0 = time.perf_counter()
            ctx.mvp_convert(qs[0][:n])
            host = min(host, time.perf_counter() - t0)
        lat[name] = {"queries": int(n), "device_ms": round(float(np.median(dev[5:])), 4),
                     "host_call_ms": round(host * 1e3, 4)}
    return {"ms_per_picture": round(ms, 4), "mpix_s": round(steps_area / elapsed / 1e6, 2),
            "plan_ahead": bool(args.plan_ahead),
            "note": ("conversions of picture t+2 on their own stream during picture t's prediction; the host "
                     "issues picture t's prediction (plan-ahead) once its conversions are complete"
                     if args.plan_ahead else
                     "conversions of picture t+1 on their own stream during picture t's prediction; "
                     "prediction of t (planning included, plan-ahead off) waits for its conversions"),
            "batch_latency": lat}


def bench_c4(args, cfg, params, rank, world, local, dist):
    """C4: one C3 picture per step, CTU-row sharded over the ranks, one packed all-gather per
    picture, pictures in random-access decode order (mm360.gop): picture k is predicted only after
    the all-gathers of all the pictures it references have landed (a stream wait on their RCCL
    work), so a picture's all-gather overlaps only the prediction of pictures that do not reference
    it.  Every step predicts the same PU list from the same resident reference planes (synthetic
    data); the decode-order dependencies are enforced, the reference samples are not re-read from
    the gathered pictures."""
    from mm360 import gop as G
    (cur, pus, refs), = picture_set(cfg, 1)
    ctx = new_ctx(params, local, [(cur, pus, refs)])
    if args.plan_ahead:  # the stripe list is resident (mm_pred_prepare) before the timed region
        ctx.set_plan_ahead(True)
    ctx.set_call_timing(False)
    mine = P.shard_pus(pus, cfg.height, world, rank)
    ctx.prepare(cur, mine)
    lay = P.StripeLayout(cfg.width, cfg.height, world)
    n_bufs = 4
    bufs = [torch.zeros(lay.total, dtype=torch.int16, device="cuda") for _ in range(n_bufs)]
    ptrs = [lay.dst_pointers(b.data_ptr(), rank) for b in bufs]
    area = W.luma_area(pus)
    # packed transport (include/mm360.h): each rank packs its int16 segment (3 samples per word at 10
    # bits), the all-gather moves 2/3 of the bytes, and every rank unpacks a gathered picture straight
    # into a reference pool slot (margins included) when a picture that references it is predicted --
    # the decoder's "reconstructed picture becomes a reference" step, so its cost is in the loop (the
    # int16 transport, --c4-pack 0, uploads from the int16 stripes the same way)
    pack = bool(args.c4_pack) and world > 1
    nw = ctx.stripe_packed_dwords(world)
    pbufs = [torch.zeros(world * nw, dtype=torch.int32, device="cuda") for _ in range(n_bufs)] if pack else []
    ref_fifo = []  # POCs of the gathered pictures uploaded as references (released after 6)

    def mc_only(s):
        ctx.run_raw(*ptrs[s % 2])

    class Gathered:
        """a packed all-gather in flight: waiting for it also unpacks it into the pool, once"""
        serial = [0]

        def __init__(self, h, b):
            self.h, self.b, self.done = h, b, False

        def wait(self):
            if self.h is not None:
                self.h.wait()
            if not self.done:
                self.done = True
                Gathered.serial[0] += 1
                poc = 100000 + Gathered.serial[0]
                if pack:
                    ctx.upload_ref_packed(poc, pbufs[self.b], world)
                else:
                    ctx.upload_ref_stripes(poc, bufs[self.b], world)
                ref_fifo.append(poc)
                if len(ref_fifo) > 6:
                    ctx.release_ref(ref_fifo.pop(0))

    def gather(b):
        if world == 1:
            return None  # the whole picture is already here
        if pack:
            ctx.pack_samples(bufs[b][rank * lay.seg:(rank + 1) * lay.seg], pbufs[b][rank * nw:(rank + 1) * nw])
            if args.dist_backend == "nccl":
                return Gathered(P.allgather_packed(pbufs[b], lay, async_op=True), b)
            host = pbufs[b].cpu()  # gloo rehearsal: host staging, synchronous
            P.allgather_packed(host, lay)
            pbufs[b].copy_(host)
            return Gathered(None, b)
        if args.dist_backend == "nccl":
            return Gathered(P.allgather_packed(bufs[b], lay, async_op=True), b)
        host = bufs[b].cpu()  # gloo rehearsal: host staging, synchronous
        P.allgather_packed(host, lay)
        bufs[b].copy_(host)
        return Gathered(None, b)

    def loop_for(gop_name, ref_waits=True, gather_all=False):
        """A DependencyLoop whose warm-up steps are the tail of the GOP before the timed one, so
        the timed steps start at a GOP boundary.  ref_waits False: the dependency-free upper bound
        (every all-gather hidden behind the next picture, round 2's loop).  gather_all: all-gather
        every picture, not only the referenced ones."""
        size = len(G.GOPS[gop_name])
        start = (size - args.warmup % size) % size
        return G.DependencyLoop(gop_name, n_bufs, lambda k, poc, rr, b: ctx.run_raw(*ptrs[b]), gather,
                                lambda h: h.wait(), start=start, ref_waits=ref_waits, gather_all=gather_all)

    d_mine = mm360.pus_to_device(mine)

    def batched_loop(gop_name, max_pics=2):
        """The RA loop with the independent pictures that follow each other in decode order (the
        highest-layer leaves: 1 3, 5 7, ...) predicted together by mm_pred_device_multi: one launch
        chain per batch; dependencies and all-gathers as in loop_for.  Returns the time of `steps`
        pictures after `warmup` pictures."""
        lp = loop_for(gop_name)
        start = lp.k

        def pb(items):
            ctx.predict_device_multi_raw([(cur, d_mine, *ptrs[b]) for _, _, _, b in items])

        def run_until(target):
            while lp.k < target:
                lp.step_batch(min(max_pics, target - lp.k), pb)

        run_until(start + args.warmup)
        return timed(1, 0, lambda s: run_until(start + args.warmup + args.steps), dist)

    t_mc = timed(args.steps, args.warmup, mc_only, dist)
    results = {}
    for name, gop_name, ref_waits, gather_all in (("ra32", "ra32", True, False), ("ra32_all", "ra32", True, True),
                                                  ("ra8", "ra8", True, False), ("independent", "ra32", False, True)):
        if world == 1:
            results[name] = t_mc
            continue
        lp = loop_for(gop_name, ref_waits, gather_all)
        results[name] = timed(args.steps, args.warmup, lambda s: lp.step(), dist)
    results["ra32_batched"] = batched_loop("ra32")
    # the line's loop at N > 1: the RA loop with the independent leaves predicted together (one launch
    # chain for two pictures' small stripes); one picture per call is reported beside it
    t_e2e = results["ra32_batched"] if world > 1 else results["ra32"]
    # one more picture into buffer 0, all-gathered, for the bit-exact check below
    mc_only(0)
    h = gather(0) if world > 1 else None
    if h is not None:
        h.wait()
    torch.cuda.synchronize()
    ctx.synchronize()
    gathered_pic = (P.unpack_picture(pbufs[0].cpu().numpy().view(np.uint32), lay, params.bit_depth) if pack
                    else lay.unpack(bufs[0].cpu().numpy()))
    # stage timing of this rank's stripe
    ctx.set_stage_timing(True)
    stages = []
    for s in range(args.kernel_steps):
        mc_only(s)
        stages.append(ctx.last_stage_timing_ms())
    ctx.set_stage_timing(False)
    st = np.mean(np.array(stages), axis=0)
    kernel_ms = float(st[3])
    achieved = W.algorithmic_bytes(mine) / (kernel_ms * 1e-3) / 1e9
    # a gathered picture on this rank vs the oracle's full picture
    bit_exact = None
    if rank == 0 and not args.no_cpu_baseline:
        from oracle.oracle import Oracle
        orc = Oracle(params, [(cur, -1, W.GED_EPIPOLE_Q24)])
        want = orc.predict_padded(orc.padded_refs(refs), cur, pus, cfg.width, cfg.height, cpu_threads())
        # buffer 0 was last written by the gathered check picture
        bit_exact = all(np.array_equal(g, w) for g, w in zip(gathered_pic, want))
    if rank == 0:
        ag_bytes = (world - 1) * (nw * 4 if pack else lay.seg * 2)
        per = lambda t: {"value": round(area * args.steps / t / 1e6, 2), "ms_per_step": round(t / args.steps * 1e3, 4)}
        print(json.dumps({
            "metric": METRIC, "value": round(area * args.steps / t_e2e / 1e6, 2), "unit": "Mpixels/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(t_e2e / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "f32+int16", "data": "synthetic (seeded ERP planes + PU list, SURVEY 8(d))",
            "config": {"workload": f"C4: {cfg.description}, CTU-row sharded across {world} GPU(s), pictures in "
                                   f"the reference's RA GOP-32 decode order (cfg/encoder_randomaccess_vtm.cfg): "
                                   f"each referenced picture is rebuilt on every GPU by one packed RCCL all-gather, "
                                   f"each picture is predicted after its references' all-gathers, unreferenced "
                                   f"(highest temporal layer) pictures stay sharded"
                                   + (f", consecutive independent pictures (the leaves 1 3, 5 7, ...) predicted together "
                                      f"in one launch chain (mm_pred_device_multi)" if world > 1 else ""),
                       "width": cfg.width, "height": cfg.height,
                       "pus": int(len(pus)), "pus_rank0": int(len(mine)), "luma_area": int(area),
                       "stripe_ctu_rows": lay.rows // 128, "allgather_bytes_in_per_rank": int(ag_bytes),
                       "transport": ("packed: 3 samples per 32-bit word (mm_pack_samples), unpacked into the "
                                     "reference pool on every rank when a picture references it "
                                     "(mm_upload_ref_packed)" if pack else
                                     "int16 samples, uploaded into the reference pool on every rank when a "
                                     "picture references it (mm_upload_ref_stripes)"),
                       "gop": "ra32", "timed_pictures": "decode-order pictures 0..steps-1 of a GOP",
                       "plan_ahead": bool(args.plan_ahead), "parallelism": f"ctu-row stripes x{world}"},
            "ra_gop8": dict(per(results["ra8"]), note="same loop, dyadic hierarchical-B GOP-8 decode order"),
            "ra32_batched": dict(per(results["ra32_batched"]),
                                 note="consecutive independent pictures (the highest-layer leaves 1 3, 5 7, ...) "
                                      "predicted together in one launch chain (mm_pred_device_multi); the line's "
                                      "value at N > 1"),
            "ra32_single": dict(per(results["ra32"]), note="same RA loop, one picture per call"),
            "ra32_gather_every_picture": dict(per(results["ra32_all"]),
                                              note="same loop, unreferenced pictures all-gathered too"),
            "independent": dict(per(results["independent"]),
                                note="no reference waits: every all-gather hidden behind the next picture (upper bound)"),
            "mc_only": dict(per(t_mc), note="same loop without the all-gather (references pre-replicated)"),
            "bit_exact": bit_exact,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None, "kernel": "k_mc_dev (rank 0 stripe)",
                         "kernel_ms": round(kernel_ms, 4), "algorithmic_bytes": int(W.algorithmic_bytes(mine))},
            "stages_ms": {"plan": round(float(st[0]), 4), "setup": round(float(st[1]), 4),
                          "reproj": round(float(st[2]), 4), "mc": round(float(st[3]), 4),
                          "pipeline": round(float(st.sum()), 4)},
            "cpu_baseline": None,
        }), flush=True)
    ctx.close()


def bench_c4_emulate(args, cfg, params):
    """C4 rehearsal on ONE GPU (not a bench line): for N = 2, 4, 8 the per-GPU MC time of every
    rank's CTU-row stripe (ranks run one after another here, so the max over ranks is the N-GPU
    step time of the MC part), then the predicted per-picture time of the N-GPU C4 loop, with the
    stripe all-gather (N-1)/N x 56.6 MB inbound per rank modelled at one xGMI link per direction
    (ring, ~153 GB/s) and at all 7 links (direct, 7 x 153 GB/s): hidden behind the next picture's
    MC regardless of dependencies (max(mc, allgather), the upper bound), or in random-access decode
    order (mm360.gop.schedule: a picture waits for its references' all-gathers; the reference's
    GOP-32 and a dyadic GOP-8; only referenced pictures are all-gathered, or every one: _all)."""
    from mm360 import gop as G
    (cur, pus, refs), = picture_set(cfg, 1)
    ctx = new_ctx(params, 0, [(cur, pus, refs)])
    if args.plan_ahead:
        ctx.set_plan_ahead(True)
    area = W.luma_area(pus)
    pic_bytes = cfg.width * cfg.height * 2 * 3 // 2
    dy, dcb, dcr = planes(cfg)
    out = {"note": "one-GPU rehearsal: measured stripe MC times, all-gather times modelled", "n": {},
           "plan_ahead": bool(args.plan_ahead)}
    link = 153e9
    for n in (1, 2, 4, 8):
        worst = 0.0
        issue = 0.0
        for r in range(n):
            mine = P.shard_pus(pus, cfg.height, n, r)
            ctx.prepare(cur, mine)
            t = timed(args.steps, args.warmup, lambda s: ctx.run(dy, dcb, dcr), None)
            worst = max(worst, t / args.steps)
            if r == 0:  # host time to issue one call (no synchronisation inside the loop)
                torch.cuda.synchronize()
                h0 = time.perf_counter()
                for _ in range(args.steps):
                    ctx.run(dy, dcb, dcr)
                issue = (time.perf_counter() - h0) / args.steps
                torch.cuda.synchronize()
        ag = (n - 1) / n * pic_bytes
        ring, mesh = ag / link, ag / (7 * link) if n > 1 else 0.0
        mc = worst * 1e3
        dep = {f"{g}{'_all' if every else ''}_{k}": round(G.schedule(64, mc, a * 1e3, g, every)["ms_per_picture"], 4)
               for g in ("ra32", "ra8") for every in (False, True) for k, a in (("ring", ring), ("mesh", mesh))}
        # packed transport: measured pack (one rank's segment) and unpack-into-the-pool (the gathered
        # picture) kernels on this GPU, around the modelled all-gather of the packed segments
        lay = P.StripeLayout(cfg.width, cfg.height, n)
        nw = ctx.stripe_packed_dwords(n)
        seg = torch.zeros(lay.seg, dtype=torch.int16, device="cuda")
        pk = torch.zeros(n * nw, dtype=torch.int32, device="cuda")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ctx.pack_samples(seg, pk[:nw])
        ctx.upload_ref_packed(999, pk, n)
        e0.record()
        for _ in range(10):
            ctx.pack_samples(seg, pk[:nw])
        e1.record()
        e1.synchronize()
        pack_ms = e0.elapsed_time(e1) / 10
        e0.record()
        for _ in range(10):
            ctx.upload_ref_packed(999, pk, n)
        e1.record()
        e1.synchronize()
        unpack_ms = e0.elapsed_time(e1) / 10
        full16 = torch.zeros(lay.total, dtype=torch.int16, device="cuda")
        ctx.upload_ref_stripes(999, full16, n)
        e0.record()
        for _ in range(10):
            ctx.upload_ref_stripes(999, full16, n)
        e1.record()
        e1.synchronize()
        up16_ms = e0.elapsed_time(e1) / 10
        ctx.release_ref(999)
        ag_p = (n - 1) * nw * 4
        ring_p = pack_ms + ag_p / link * 1e3 + unpack_ms
        mesh_p = pack_ms + ag_p / (7 * link) * 1e3 + unpack_ms
        ring_u, mesh_u = ring * 1e3 + up16_ms, mesh * 1e3 + up16_ms
        dep_p = {f"ra32_{t}_{k}": round(G.schedule(64, mc, a, "ra32")["ms_per_picture"], 4)
                 for t, k, a in (("packed", "ring", ring_p), ("packed", "mesh", mesh_p),
                                 ("int16_upload", "ring", ring_u), ("int16_upload", "mesh", mesh_u))} if n > 1 else {}
        out["n"][n] = {"mc_ms": round(mc, 4), "host_issue_ms": round(issue * 1e3, 4),
                       "allgather_ms": {"ring": round(ring * 1e3, 4), "mesh": round(mesh * 1e3, 4)},
                       "int16_upload_into_pool_ms": round(up16_ms, 4),
                       "packed": {"pack_ms": round(pack_ms, 4), "unpack_into_pool_ms": round(unpack_ms, 4),
                                  "allgather_bytes_in": int(ag_p), "int16_bytes_in": int(ag),
                                  "transfer_ms": {"ring": round(ring_p, 4), "mesh": round(mesh_p, 4)},
                                  "int16_transfer_ms": {"ring": round(ring_u, 4), "mesh": round(mesh_u, 4)},
                                  "note": "pack + modelled all-gather of the packed segments + unpack into the "
                                          "reference pool, the dependent picture's wait"},
                       "pred_ms_per_picture": {"hidden_ring": round(max(worst, ring) * 1e3, 4),
                                               "hidden_mesh": round(max(worst, mesh) * 1e3, 4),
                                               "serial_ring": round((worst + ring) * 1e3, 4), **dep, **dep_p},
                       "pred_mpix_s": {"hidden_ring": round(area / max(worst, ring) / 1e6, 1),
                                       "hidden_mesh": round(area / max(worst, mesh) / 1e6, 1),
                                       "mc_only": round(area / worst / 1e6, 1),
                                       **{k: round(area / (v * 1e-3) / 1e6, 1) for k, v in {**dep, **dep_p}.items()}}}
    # Independent pictures (one temporal layer of the RA GOP) in flight together: k contexts, each
    # with its own stream and resident references, predicting rank 0's stripe concurrently, so that
    # several 1/N-picture launch chains share the GPU.  ms per stripe = elapsed / (steps x k).
    ctx.close()
    conc = {}
    for n in (4, 8):
        mine = P.shard_pus(pus, cfg.height, n, 0)
        conc[n] = {}
        for k in (1, 2, 3, 4):
            ctxs, outs, streams = [], [], []
            for _ in range(k):
                cj = new_ctx(params, 0, [(cur, pus, refs)])
                sj = torch.cuda.Stream()
                cj.set_stream(sj.cuda_stream)
                cj.set_plan_ahead(False)  # plan-ahead's host wait would serialise the contexts' calls
                cj.prepare(cur, mine)
                ctxs.append(cj)
                outs.append(planes(cfg))
                streams.append(sj)
            t = timed(args.steps, args.warmup, lambda st: [c.run(*o) for c, o in zip(ctxs, outs)], None)
            conc[n][k] = round(t / args.steps / k * 1e3, 4)
            for c in ctxs:
                c.synchronize()
                c.close()
    # The same with ONE context and ONE launch chain per k stripes (mm_pred_device_multi: the stripes
    # of k independent pictures planned, reprojected and interpolated together, plan-ahead on)
    multi = {}
    cm = new_ctx(params, 0, [(cur, pus, refs)])
    cm.set_plan_ahead(bool(args.plan_ahead))
    for n in (4, 8):
        mine = P.shard_pus(pus, cfg.height, n, 0)
        d_mine = mm360.pus_to_device(mine)
        multi[n] = {}
        for k in (1, 2, 3, 4):
            outs = [planes(cfg) for _ in range(k)]
            jobs = [(cur, d_mine, *o) for o in outs]
            torch.cuda.synchronize()
            t = timed(args.steps, args.warmup, lambda st: cm.predict_device_multi(jobs), None)
            cm.synchronize()
            multi[n][k] = round(t / args.steps / k * 1e3, 4)
    cm.close()
    # the RA loop with the leaves predicted two at a time (bench_c4's line at N > 1), modelled: each
    # rank's batch costs its single-stripe time x rank 0's measured ratio of two-in-one-chain to one
    for n in (4, 8):
        ratio = multi[n][2] / multi[n][1]
        e = out["n"][n]
        mc = e["mc_ms"]
        for k, a in (("ring", e["allgather_ms"]["ring"]), ("mesh", e["allgather_ms"]["mesh"]),
                     ("packed_ring", e["packed"]["transfer_ms"]["ring"]), ("packed_mesh", e["packed"]["transfer_ms"]["mesh"]),
                     ("int16_upload_ring", e["packed"]["int16_transfer_ms"]["ring"]),
                     ("int16_upload_mesh", e["packed"]["int16_transfer_ms"]["mesh"])):
            v = round(G.schedule(64, mc, a, "ra32", batch_ms={2: mc * ratio})["ms_per_picture"], 4)
            e["pred_ms_per_picture"][f"ra32_batched_{k}"] = v
            e["pred_mpix_s"][f"ra32_batched_{k}"] = round(area / (v * 1e-3) / 1e6, 1)
    out["multi_picture_stripes"] = {
        "ms_per_stripe": multi,
        "note": "rank 0's stripe of k independent pictures predicted by ONE context in ONE launch chain per "
                "step (mm_pred_device_multi, plan-ahead as set): ms per stripe = elapsed / (steps x k)"}
    out["concurrent_stripes"] = {
        "ms_per_stripe": conc,
        "note": "rank 0's stripe predicted by k contexts at once (own streams and resident references, "
                "plan-ahead off: its host wait per call would serialise the contexts' calls from one host "
                "thread): the pictures of one temporal layer do not reference each other, so a decoder may "
                "predict them together; one stripe at a time with plan-ahead takes n[N].mc_ms"}
    print(json.dumps(out), flush=True)


def c5_record(args, steps=3, warmup=1):
    """The C5 configuration (encoder ME candidate evaluation, 2048x1024, all models, 33x33 integer
    window per 16x16 block and model) beside the C3 line: Mcandidates/s over `steps` full windows,
    bit_exact of the device SADs against the oracle on a seeded sample of blocks, and the bound of
    k_me_sad from the committed PMC profile of this very library (VALU, not HBM: every candidate
    reprojects its block), when one exists."""
    import glob
    import hashlib
    cfg = W.CONFIGS["C5"]
    params = mm360.seq_params(cfg.width, cfg.height, cfg.models)
    blocks = W.me_blocks(cfg.width, cfg.height, cfg.models, grid=16, seed=5)
    C = (2 * W.ME_RANGE + 1) ** 2
    ctx = mm360.MMContext(params, device=torch.cuda.current_device())
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    ctx.set_epipole(W.CUR_POC, -1, W.GED_EPIPOLE_Q24)
    refs = {poc: W.ref_planes(cfg.width, cfg.height, poc) for poc in W.REF_POCS}
    for poc, (y, cb, cr) in refs.items():
        ctx.upload_ref(poc, torch.from_numpy(y).cuda(), torch.from_numpy(cb).cuda(), torch.from_numpy(cr).cuda())
    org = W.org_plane(cfg.width, cfg.height)
    ctx.upload_org(W.CUR_POC, torch.from_numpy(org).cuda())
    sads = torch.zeros((len(blocks), C), dtype=torch.int32, device="cuda")
    kms = []

    def step(s):
        ctx.sad_window(W.CUR_POC, blocks, W.ME_RANGE, 16, out=sads)
        kms.append(ctx.last_timing_ms())

    elapsed = timed(steps, warmup, step, None)
    got = sads.cpu().numpy().view(np.uint32)
    tz = tz_step_record(ctx, blocks)
    ctx.close()
    rng = np.random.default_rng(0x4D4D8000)
    pick = np.sort(rng.choice(len(blocks), size=48, replace=False))
    bit_exact = None
    if not args.no_cpu_baseline:
        from oracle.oracle import Oracle
        orc = Oracle(params, [(W.CUR_POC, -1, W.GED_EPIPOLE_Q24)])
        want = orc.sad_window(W.CUR_POC, blocks[pick], W.ME_RANGE, 16, {poc: r[0] for poc, r in refs.items()}, org)
        bit_exact = bool(np.array_equal(got[pick], want))
        tz_pick = (pick[:, None] * 8 + np.arange(8)[None, :]).ravel()
        tz_want = orc.sad_window(W.CUR_POC, tz.pop("_blocks")[tz_pick], 0, 16,
                                 {poc: r[0] for poc, r in refs.items()}, org)
        tz["bit_exact"] = bool(np.array_equal(tz.pop("_sads")[tz_pick], np.asarray(tz_want).view(np.uint32).ravel()))
        tz["bit_exact_sample"] = f"{len(pick)} seeded blocks x 8 candidates vs the oracle"
    else:
        tz.pop("_blocks")
        tz.pop("_sads")
    bound = None  # the committed PMC profile of this very library, if any (tools/c5_pmc_json.py)
    lib_sha = hashlib.sha256(open(mm360.LIB_PATH, "rb").read()).hexdigest()
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_c5_pmc.json")), reverse=True):
        d = json.load(open(path))
        if d.get("lib_sha256") == lib_sha:
            bound = {k: d[k] for k in ("kernel", "valu_insts_per_wave", "valu_active_share", "valu_busy_2cyc",
                                       "note") if k in d}
            break
    n_cand = len(blocks) * C
    return {"workload": f"C5: {cfg.description}", "blocks": int(len(blocks)), "candidates": int(n_cand),
            "tz_step": tz,
            "value": round(n_cand * steps / elapsed / 1e6, 2), "unit": "Mcandidates/s",
            "ms_per_window_set": round(elapsed / steps * 1e3, 3),
            "kernel_ms": round(float(np.mean(kms[warmup:])), 3),
            "bit_exact": bit_exact, "bit_exact_sample": f"{len(pick)} seeded blocks x {C} candidates vs the oracle",
            "bound": bound}


TZ_SQUARE = ((-1, -1), (0, -1), (1, -1), (-1, 0), (1, 0), (-1, 1), (0, 1), (1, 1))  # InterSearch.cpp:492-526


def tz_step_record(ctx, blocks, dist=2, reps=5):
    """The encoder's dependent call pattern (InterSearch.cpp:474-526, xTZ8PointSquareSearch via
    xTZSearchHelp): ONE TZ 8-point square step at distance `dist` around every block's current best
    (here the C5 window centre) for every PU x model of the C5 picture as one device round trip
    including the host's wait for the SADs (the next step's start points depend on them).
    mm_sad_pattern takes the step as one pattern of 8 offsets shared by the blocks (each block's setup
    and each sub-block's model head once for its 8 candidates); the round-5 form -- 8 range-0 blocks
    per block through mm_sad_window -- is timed beside it.  Time per step, and the steps an encoder
    could afford per picture in a 30 fps budget."""
    off = np.array(TZ_SQUARE, dtype=np.int32) * (16 * dist)
    b8 = np.repeat(blocks, 8)
    o8 = np.tile(off, (len(blocks), 1))
    b8["mv_hor"] += o8[:, 0]
    b8["mv_ver"] += o8[:, 1]
    out = torch.zeros((len(blocks), 8), dtype=torch.int32, device="cuda")
    host = torch.empty((len(blocks), 8), dtype=torch.int32, pin_memory=True)  # an encoder's SAD buffer

    def run(fn):
        fn()  # warm-up (buffers)
        host.copy_(out)
        t, tc = [], []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()  # synchronous: returns with the SADs in HBM
            t1 = time.perf_counter()
            host.copy_(out)  # the host needs the SADs to pick the next step's start points
            t.append(time.perf_counter() - t0)
            tc.append(time.perf_counter() - t1)
        return (float(np.median(t)) * 1e3, ctx.last_timing_ms(), float(np.median(tc)) * 1e3,
                host.numpy().copy().view(np.uint32).reshape(len(blocks), 8))

    ms, dev_ms, copy_ms, sads = run(lambda: ctx.sad_pattern(W.CUR_POC, blocks, off, out=out))
    ms0, dev_ms0, _, sads0 = run(lambda: ctx.sad_window(W.CUR_POC, b8, 0, 16, out=out.view(-1, 1)))
    return {"candidates": int(len(b8)), "blocks": int(len(blocks)), "distance": dist,
            "ms_per_step": round(ms, 3), "device_ms": round(dev_ms, 3), "sad_copy_ms": round(copy_ms, 3),
            "host_ms": round(ms - dev_ms - copy_ms, 3),
            "steps_per_33ms": int(33.3 / ms),
            "range0_blocks": {"ms_per_step": round(ms0, 3), "device_ms": round(dev_ms0, 3),
                              "equal": bool(np.array_equal(sads, sads0))},
            "note": "one xTZ8PointSquareSearch step for every PU x model of the picture as one mm_sad_pattern call "
                    "(8 offsets shared by the blocks) + the SAD copy to a pinned host buffer, median of the calls; "
                    "device_ms: the call's stream time (block uploads + kernels), host_ms: planning and call overhead; "
                    "range0_blocks: the same step as 8 range-0 blocks per block through mm_sad_window; "
                    "steps_per_33ms: dependent steps a 30 fps encoder could afford per picture on this path alone",
            "_blocks": b8, "_sads": sads.ravel()}


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
    kms = []

    def step(s):
        ctx.sad_window(W.CUR_POC, blocks, W.ME_RANGE, 16, out=sads)
        kms.append(ctx.last_timing_ms())

    elapsed = timed(args.steps, args.warmup, step, dist)
    total = float(n_cand)
    if dist:
        at = torch.tensor([total], dtype=torch.float64, device=RED_DEVICE[0])
        dist.all_reduce(at, op=dist.ReduceOp.SUM)
        total = float(at.item())
    kernel_ms = float(np.mean(kms[args.warmup:]))
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
        cpu.update(host_info(cpu_threads()))
    if rank == 0:
        print(json.dumps({
            "metric": "MM encoder ME candidate evaluations/s (reprojection + 8-tap + SAD) on 2048x1024 ERP",
            "value": round(total * args.steps / elapsed / 1e6, 3), "unit": "Mcandidates/s",
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default=None, help="C3 (default at 1 GPU), C4 (default at N > 1), C2, C5")
    ap.add_argument("--pictures", type=int, default=4, help="C3: distinct pictures (each with its own references)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-mvp", action="store_true", help="C3: skip the MM-MVP figure beside the line")
    ap.add_argument("--no-c5", action="store_true", help="C3: skip the C5 (encoder ME) sub-record beside the line")
    ap.add_argument("--no-dmvr", action="store_true", help="C3: skip the MM-DMVR sub-record beside the line")
    ap.add_argument("--no-multi", action="store_true",
                    help="C3: skip the multi_picture sub-record (k pictures per launch) beside the line")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="length of the one-thread CPU baseline sample")
    ap.add_argument("--kernel-steps", type=int, default=8, help="extra steps timed per launch with HIP events")
    ap.add_argument("--lib", default=None, help="alternative build of libmm360.so (A/B experiments)")
    ap.add_argument("--stripes", type=int, default=None, help="mm_set_stripes (default: the library's)")
    ap.add_argument("--plan-ahead", type=int, default=1, choices=(0, 1),
                    help="mm_set_plan_ahead: planning of picture t+1 overlaps picture t's interpolation "
                         "(every bench PU list is resident before the timed region)")
    ap.add_argument("--c4-emulate", action="store_true",
                    help="C4 rehearsal on one GPU: per-rank stripe MC times for N = 2, 4, 8 + modelled all-gather")
    ap.add_argument("--coherent-mv", action="store_true",
                    help="experiment: one MV for every PU and list (spatially coherent motion)")
    ap.add_argument("--dmvr-correlated", action="store_true",
                    help="with --dmvr-share: both references and both lists' MVs of the DMVR PUs agree (early exits)")
    ap.add_argument("--dmvr-share", type=float, default=0.0,
                    help="C2/C3: this share of the DMVR-eligible bi leaves are merge/mvRefine PUs that run MM-DMVR "
                         "inside the picture's launch sequence (mm_set_dmvr, MM_PUF_DMVR)")
    ap.add_argument("--uniform-model", type=int, default=None,
                    help="per-model workload: all PUs 16x16 with this MotionModelID (SURVEY 8(d))")
    ap.add_argument("--c4-pack", type=int, default=1, choices=(0, 1),
                    help="C4: all-gather the stripe-packed picture (3 samples per word) and unpack it into the "
                         "reference pool (1), or move int16 samples (0)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (RCCL over xGMI, default) or gloo (rehearsal of N ranks on one GPU: the "
                         "all-gather then stages through host memory)")
    args = ap.parse_args()

    if args.lib:
        mm360.LIB_PATH = os.path.abspath(args.lib)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dist_backend != "nccl":  # gloo rehearsal: ranks may share the box's GPU(s)
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(args.dist_backend)
            RED_DEVICE[0] = "cpu"
    args.config = args.config or ("C3" if world == 1 else "C4")
    cfg = W.CONFIGS["C3" if args.config == "C4" else args.config]
    params = mm360.seq_params(cfg.width, cfg.height, cfg.models)
    if args.config == "C5":
        bench_me(args, cfg, params, rank, world, local, dist)
    elif args.config == "C4" and args.c4_emulate:
        bench_c4_emulate(args, cfg, params)
    elif args.config == "C4":
        bench_c4(args, cfg, params, rank, world, local, dist)
    else:
        line = bench_pictures(args, cfg, params, rank, world, local, dist)
        if line is not None:
            if args.config == "C3" and world == 1 and args.dmvr_share == 0 and not args.no_dmvr:
                line["dmvr"] = dmvr_record(args, cfg, params)
                line["dmvr_correlated"] = dmvr_record(args, cfg, params, correlated=True)
            if args.config == "C3" and world == 1 and not args.no_c5:
                line["c5"] = c5_record(args)
            print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
