// mm_kernels.hip -- gfx950 kernels and the C-ABI (include/mm360.h) of the 360-degree
// multi-model motion-compensation path.
//
// Pipeline of one mm_pred_device (one picture's PU list, all device work, one stream):
//   k_plan_count / k_plan_place   device planning (mm_devplan.h): PU classification and
//              validation, class-sorted PUs, (component, model, packet)-sorted jobs.
//   k_setup    thread per reprojection job (PU x list x {luma, chroma}): the per-block part of
//              reprojectMotionVectorSubblocks (centre transforms, rotation matrices, k, ...).
//   k_reproj   thread per sub-block element of every job: <Model>::modelMotion[Cached] + NaN
//              fallback + fixed-point rounding -> int32 (X, Y) per element.
//   k_mc       thread per luma 4x4 sub-block of every PU: for each used list, the 8-tap luma and
//              4-tap 4:2:0 chroma sub-block predictions (xPredInterBlkMM :776-828) and the
//              addAvg / uni output (xWeightedAverage), written straight into the picture planes.
// (k_setup / k_reproj also serve the parity API mm_reproject on a host-planned block list; the
// _dev variants read their sizes from the device plan.)
// Reference planes stay resident in HBM in one pool, each plane with edge-replicated margins wide
// enough for every in-range window (plane_layout below), so k_mc, the MM-DMVR search and the ME
// SAD kernel read windows without clamping; the host twin clamps addresses instead (same values).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <utility>
#include <vector>

#include "../../include/mm360.h"
#include "mm_effective.h"
#include "mm_pipeline.h"
#include "mm_plan.h"
#include "mm_syntax.h"

using namespace mmpipe;

#define MM_VERSION 300

namespace {

__constant__ int8_t c_luma_taps[16][8] = MM_LUMA_TAPS_INIT;
__constant__ int8_t c_chroma_taps[32][4] = MM_CHROMA_TAPS_INIT;
__constant__ PackedTaps c_packed_taps = make_packed_taps();

__global__ void k_mpa_cache(SeqConst sc, int plane, int cols, int rows, float* px, float* py, uint8_t* vip) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= cols * rows) return;
  mpa_cache_thread(t, sc, plane, cols, rows, px, py, vip);
}

__global__ void k_erp_trig(SeqConst sc, int cols, int rows, float* col, float* row) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 2 * (cols + rows)) return;
  erp_trig_thread(t, sc, cols, rows, col, row);
}

__global__ void k_tan_grid(SeqConst sc, MpaCache cache, TanEntry* out) {
  tan_grid_thread((long)blockIdx.x * blockDim.x + threadIdx.x, sc, cache, out);
}

__global__ void k_setup(SeqConst sc, const JobDev* __restrict__ jobs, int n_jobs, const M3* __restrict__ ged,
                        BlockSetup* __restrict__ out) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_jobs) return;
  setup_thread(t, sc, jobs, ged, out);
}

__global__ void __launch_bounds__(256) k_reproj(SeqConst sc, const JobDev* __restrict__ jobs, int n_jobs,
                                                const int* __restrict__ job_offsets, const int* __restrict__ chunk_start,
                                                int n_elems, const BlockSetup* __restrict__ setups, MpaCache cache,
                                                int32_t* __restrict__ out) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g - (int)__lane_id() >= n_elems) return;  // whole wave past the end
  const int ji = wave_find_item(job_offsets, chunk_start, g, n_jobs);
  if (g >= n_elems) return;
  reproj_thread(g, ji, sc, jobs, job_offsets, setups, cache, out);
}

// --------------------------------------------------------------------------------------------
// Device-planned picture path (mm_pred_device): k_plan_count -> k_plan_place -> k_setup_dev ->
// k_reproj_dev -> k_mc_dev, sizes from PlanMeta (mm_devplan.h).
// --------------------------------------------------------------------------------------------
using namespace mmdev;

// Buffer capacities of the device plan (the host sizes them; k_plan_place enforces them).
struct PlanCaps {
  int pus, sb, jobs, elems;
  int subs, dmvr_elems;  // MM-DMVR sub-PU records and cost elements (0 unless DMVR is enabled)
};
// Where k_plan_place puts the MM-DMVR sub-PU records (mm_dmvr.h SubPuDev), their cost-element
// offsets and the 64-element chunk starts of those elements.
struct DmvrRecs {
  SubPuDev* sub;
  int* off;
  int* chunk;
};

// Workgroups are dispatched round-robin over the 8 XCDs, each with its own L2.  Within every
// group of 8 * XCD_RUN consecutive workgroups, renumbering them XCD-major hands each XCD a run of
// XCD_RUN adjacent workgroups, so neighbouring PUs (overlapping reference windows) share one L2.
// Groups stay small so that the work of every region still spreads over all XCDs (a static
// 1/8 split of the whole grid would load one XCD with the most expensive model bucket).
// Requires gridDim.x % (8 * XCD_RUN) == 0; the grids are sized by the plan capacities and
// workgroups past the device-known totals exit at once.
constexpr int XCD_RUN = 4;
__device__ __forceinline__ int xcd_block() {
  const int b = blockIdx.x, grp = b / (8 * XCD_RUN), r = b % (8 * XCD_RUN);
  return grp * (8 * XCD_RUN) + (r & 7) * XCD_RUN + (r >> 3);
}

// Planning runs without global atomics: k_plan_count (1024-thread blocks) writes each block's
// bucket counts to its own row of `blk`, and those of each of its four 256-PU quarters to their
// rows of `blkq`; every k_plan_place block (256 threads, one quarter) sums the column of each bucket
// over the count blocks (the bucket total) and the part above its own count block, plus the
// quarters before it inside that block (its offset inside the bucket).  PUs therefore land in their
// buckets in input order, quarter by quarter.  Placement uses 256-thread blocks because its
// scattered record stores are bound by the texture-address path of the CUs it runs on: 1024-thread
// blocks put 16 storing waves on each of only n / 1024 CUs (profiles/r02_ab_plan_place.txt).
constexpr int PLAN_BLOCK = 1024;
constexpr int PLACE_BLOCK = 256;
constexpr int PLAN_Q = PLAN_BLOCK / PLACE_BLOCK;  // quarters per count block
constexpr int N_KEYS = DMVR_KEY + 1;  // one row of `blk`: PU buckets, job buckets, the DMVR bucket

// status: the picture's validation word (0 = ok, else ~((pu_index << 8) | code) of the lowest
// failing PU, combined with atomicMax over every stripe of the picture).
__global__ void __launch_bounds__(PLAN_BLOCK) k_plan_count(const PuSegs pus, int n, int pu_base,
                                                    const PicTables t, unsigned long long* __restrict__ status,
                                                    unsigned long long* __restrict__ blk,
                                                    unsigned long long* __restrict__ blkq, int n_quarters) {
  __shared__ unsigned long long s_cnt[PLAN_Q][N_KEYS], s_status;
  const int tid = threadIdx.x, q = tid / PLACE_BLOCK;
  for (int k = tid; k < PLAN_Q * N_KEYS; k += PLAN_BLOCK) lds_put((&s_cnt[0][0])[k], 0ull, 0ull);
  if (tid == 0) lds_put(s_status, 0ull, 0ull);
  __syncthreads();
  const int i = blockIdx.x * blockDim.x + tid;
  if (i < n) {
    const int pic = pu_seg(pus, i);
    const mm_pu_desc u = load_pu(pus, i, pic);
    PuPlan p;
    classify_pu(u, t, &p, pic);
    if (p.code != MM_OK) {
      atomicMax(&s_status, status_word(pu_base + i, p.code));
    } else {
      atomicAdd(&s_cnt[q][p.key], pu_count(p));
#pragma unroll
      for (int k = 0; k < 4; k++)
        if (p.job[k].valid) atomicAdd(&s_cnt[q][N_PU_KEYS + p.job[k].key], job_count(p, k));
      if (p.dmvr) atomicAdd(&s_cnt[q][DMVR_KEY], dmvr_count(p));
    }
  }
  __syncthreads();
  if (tid < N_KEYS) {
    unsigned long long tot = 0;
#pragma unroll
    for (int qq = 0; qq < PLAN_Q; qq++) tot += s_cnt[qq][tid];
    blk[(long)blockIdx.x * N_KEYS + tid] = tot;
  }
  for (int k = tid; k < PLAN_Q * N_KEYS; k += PLAN_BLOCK) {
    const int r = blockIdx.x * PLAN_Q + k / N_KEYS;
    if (r < n_quarters) blkq[(long)r * N_KEYS + k % N_KEYS] = (&s_cnt[0][0])[k];
  }
  if (tid == 0 && s_status) atomicMax(status, s_status);
}

// `next_status` is the other word of the picture ping-pong pair: the first stripe's block 0 zeroes
// it for the next picture, so no memset launch precedes k_plan_count.
__global__ void __launch_bounds__(PLACE_BLOCK) k_plan_place(const PuSegs pus, int n, const PicTables t,
                                                     unsigned long long* __restrict__ status,
                                                     unsigned long long* __restrict__ next_status,
                                                     const unsigned long long* __restrict__ blk, int n_blocks,
                                                     const unsigned long long* __restrict__ blkq,
                                                    PlanMeta* __restrict__ meta, PlanCaps caps,
                                                    JobDev* __restrict__ jobs, int* __restrict__ job_off,
                                                    int* __restrict__ job_chunk, DmvrRecs dm) {
  __shared__ unsigned long long s_job[N_JOB_KEYS];
  __shared__ unsigned long long g_pu[N_PU_KEYS], g_job[N_JOB_KEYS], g_dm;
  __shared__ PlanMeta s_meta;
  __shared__ int s_ok;
  const int tid = threadIdx.x;
  if (blockIdx.x == 0 && tid == 0 && next_status) *next_status = 0ull;
  if (tid < N_JOB_KEYS) lds_put(s_job[tid], 0ull, 0ull);
  // bucket totals and this quarter's offsets inside the buckets: the column sums of blk, split
  // over the block's 4 waves (wave w takes count rows w, w + 4, ...), plus the quarters before this
  // one in its count block (blkq), combined through LDS
  constexpr int NWAVE = PLACE_BLOCK / 64;
  __shared__ unsigned long long s_ptot[NWAVE][N_KEYS], s_ppre[NWAVE][N_KEYS];
  {
    const int lane = tid & 63, w = tid >> 6, b0 = blockIdx.x / PLAN_Q, q0 = b0 * PLAN_Q;
#pragma unroll
    for (int kc = 0; kc < N_KEYS; kc += 64) {
      const int key = kc + lane;
      if (key < N_KEYS) {
        unsigned long long tp = 0, pp = 0;
#pragma unroll 4
        for (int b = w; b < n_blocks; b += NWAVE) {
          const unsigned long long v = blk[(long)b * N_KEYS + key];
          tp += v;
          if (b < b0) pp += v;
        }
        if (q0 + w < (int)blockIdx.x) pp += blkq[(long)(q0 + w) * N_KEYS + key];  // PLAN_Q == NWAVE
        lds_put(s_ptot[w][key], tp, 0ull);
        lds_put(s_ppre[w][key], pp, 0ull);
      }
    }
  }
  static_assert(PLAN_Q == NWAVE, "one wave per preceding quarter");
  __syncthreads();
  unsigned long long tot = 0, pre = 0;
  if (tid < N_KEYS) {
#pragma unroll
    for (int w = 0; w < NWAVE; w++) {
      tot += s_ptot[w][tid];
      pre += s_ppre[w][tid];
    }
    if (tid < N_PU_KEYS)
      lds_put(g_pu[tid], pre, 0ull);
    else if (tid < DMVR_KEY)
      lds_put(g_job[tid - N_PU_KEYS], pre, 0ull);
    else
      lds_put(g_dm, pre, 0ull);
  }
  // PlanMeta = exclusive prefix of the bucket totals: the job buckets are one wave (lanes 6..69
  // are threads N_PU_KEYS..N_KEYS-1, scanned in two waves' halves through LDS), the PU buckets
  // are few
  __shared__ unsigned long long s_tot[N_KEYS];
  if (tid < N_KEYS) lds_put(s_tot[tid], tot, 0ull);
  __syncthreads();
  static_assert(N_JOB_KEYS == 64, "one lane per job bucket");
  if (tid < 64) {
    const unsigned long long v = s_tot[N_PU_KEYS + tid];
    const int items = packed_items(v), elems = packed_elems(v);
    int si = items, se = elems;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int ui = __shfl_up(si, d), ue = __shfl_up(se, d);
      if (tid >= d) {
        si += ui;
        se += ue;
      }
    }
    lds_put(s_meta.job_base[tid], si - items, 0);
    lds_put(s_meta.elem_base[tid], se - elems, 0);
    if (tid == 63) {
      lds_put(s_meta.n_jobs, si, 0);
      lds_put(s_meta.n_elems, se, 0);
    }
    if (tid == 0) {
      int acc = 0, sacc = 0, pb[N_PU_KEYS], sbb[N_PU_KEYS], band[N_BANDS + 1];
#pragma unroll
      for (int k = 0; k < N_PU_KEYS; k++) {
        pb[k] = acc;
        sbb[k] = sacc;
        acc += packed_items(s_tot[k]);
        sacc += packed_elems(s_tot[k]);
      }
      band_cut(sbb, sacc, band);
#pragma unroll
      for (int k = 0; k < N_PU_KEYS; k++) {
        lds_put(s_meta.pu_base[k], pb[k], 0);
        lds_put(s_meta.sb_base[k], sbb[k], 0);
      }
#pragma unroll
      for (int r = 0; r <= N_BANDS; r++) lds_put(s_meta.band[r], band[r], 0);
      lds_put(s_meta.n_pus, acc, 0);
      lds_put(s_meta.n_sb, sacc, 0);
      lds_put(s_meta.n_sub, packed_items(s_tot[DMVR_KEY]), 0);
      lds_put(s_meta.n_dmvr_elems, packed_elems(s_tot[DMVR_KEY]), 0);
    }
  }
  __syncthreads();
  if (tid == 0) {
    const int ok = s_meta.n_pus <= caps.pus && s_meta.n_sb <= caps.sb && s_meta.n_jobs <= caps.jobs &&
           s_meta.n_elems <= caps.elems && s_meta.n_sub <= caps.subs && s_meta.n_dmvr_elems <= caps.dmvr_elems;
    lds_put(s_ok, ok, 0);
    if (blockIdx.x == 0) {
      PlanMeta m = s_meta;
      if (!ok) {  // over capacity (overlapping PUs): nothing is predicted, the call fails
        m.n_pus = m.n_sb = m.n_jobs = m.n_elems = m.n_sub = m.n_dmvr_elems = 0;
        for (int r = 0; r <= N_BANDS; r++) m.band[r] = 0;
        atomicMax(status, status_word(0, MM_ERR_ARG));
      }
      *meta = m;
    }
  }
  __syncthreads();
  if (!s_ok) return;
  const int i = blockIdx.x * PLACE_BLOCK + tid;
  PuPlan p;
  p.code = MM_ERR_ARG;
  mm_pu_desc u;
  unsigned long long lp = 0, lj[4] = {0, 0, 0, 0}, ld = 0;
  if (i < n) {
    const int pic = pu_seg(pus, i);
    u = load_pu(pus, i, pic);
    classify_pu(u, t, &p, pic);
    if (p.code == MM_OK) {
#pragma unroll
      for (int k = 0; k < 4; k++)
        if (p.job[k].valid) lj[k] = atomicAdd(&s_job[p.job[k].key], job_count(p, k));
    }
  }
  // PUs and DMVR sub-PUs are placed in list order inside their buckets by exclusive scans over the
  // block (one per PU bucket) -- not in LDS-atomic arrival order: the sub-block enumeration k_mc
  // walks follows the list (CTU raster, profiles/r03_ab_scan_place.txt), and mm_pred_dmvr returns
  // its refined deltas PU after PU
  {
    __shared__ unsigned long long s_wsum[N_PU_KEYS + 1][PLACE_BLOCK / 64];
    const int lane = tid & 63, w = tid >> 6;
    const bool ok = p.code == MM_OK;
    const unsigned long long v = ok ? pu_count(p) : 0ull;
    const unsigned long long vd = (ok && p.dmvr) ? dmvr_count(p) : 0ull;
    unsigned long long mine = 0, incd = vd;
#pragma unroll
    for (int k = 0; k < N_PU_KEYS; k++) {
      const unsigned long long vk = (ok && p.key == k) ? v : 0ull;
      unsigned long long inc = vk;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const unsigned long long a = __shfl_up(inc, d);
        if (lane >= d) inc += a;
      }
      if (lane == 63) lds_put(s_wsum[k][w], inc, 0ull);
      if (ok && p.key == k) mine = inc - vk;
    }
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const unsigned long long b = __shfl_up(incd, d);
      if (lane >= d) incd += b;
    }
    if (lane == 63) lds_put(s_wsum[N_PU_KEYS][w], incd, 0ull);
    __syncthreads();
    unsigned long long before = 0, befd = 0;
    for (int k = 0; k < w; k++) {
      if (ok) before += s_wsum[p.key][k];
      befd += s_wsum[N_PU_KEYS][k];
    }
    lp = before + mine;
    ld = befd + incd - vd;
  }
  if (p.code != MM_OK) return;
  const unsigned long long bp = g_pu[p.key] + lp;
  const int sb_off = s_meta.sb_base[p.key] + packed_elems(bp);
  int jidx[4], joff[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    jidx[k] = joff[k] = 0;
    if (p.job[k].valid) {
      const int key = p.job[k].key;
      const unsigned long long bj = g_job[key] + lj[k];
      jidx[k] = s_meta.job_base[key] + packed_items(bj);
      joff[k] = s_meta.elem_base[key] + packed_elems(bj);
    }
  }
  const unsigned long long bd = g_dm + ld;
  emit_pu(u, p, sb_off, jidx, joff, jobs, job_off, job_chunk, packed_items(bd), packed_elems(bd), dm.sub, dm.off,
          dm.chunk);
}

// The 256 setups of a block are contiguous in `out`: each thread builds its BlockSetup in LDS and
// the block then streams the whole 22.5 KB image out with 16-byte stores, instead of 22 scattered
// dword stores per thread into 88-byte strided records (every one a partial cache line).
__global__ void __launch_bounds__(256) k_setup_dev(SeqConst sc, const PlanMeta* __restrict__ meta,
                                                   const JobDev* __restrict__ jobs, const PicTables t,
                                                   BlockSetup* __restrict__ out) {
  static_assert(sizeof(BlockSetup) % 8 == 0, "BlockSetup image is copied in 8-byte words");
  __shared__ alignas(16) BlockSetup s_set[256];
  __shared__ M3 s_ged[3 + MAX_SLOTS];  // indexed per lane: staged by stage_arg_words
  const int n_jobs = meta->n_jobs;
  const int base = blockIdx.x * 256;
  if (base >= n_jobs) return;
  stage_arg_words<sizeof(s_ged) / 4>(reinterpret_cast<const uint32_t*>(t.ged), reinterpret_cast<uint32_t*>(s_ged));
  __syncthreads();
  const int i = base + threadIdx.x;
  if (i < n_jobs) {
    BlockSetup b;
    setup_job(jobs[i], sc, s_ged, &b);
    lds_put(s_set[threadIdx.x], b, BlockSetup{});
  }
  __syncthreads();
  const int cnt = min(256, n_jobs - base);
  const int words = cnt * (int)(sizeof(BlockSetup) / 8);
  const uint2* src = reinterpret_cast<const uint2*>(s_set);
  uint2* dst = reinterpret_cast<uint2*>(out + base);
  for (int w = threadIdx.x; w < words; w += 256) dst[w] = src[w];
}

__global__ void __launch_bounds__(256) k_reproj_dev(SeqConst sc, const PlanMeta* __restrict__ meta,
                                                    const JobDev* __restrict__ jobs, const int* __restrict__ job_offsets,
                                                    const int* __restrict__ chunk_start,
                                                    const BlockSetup* __restrict__ setups, MpaCache cache, McRec mc) {
  const int g = xcd_block() * blockDim.x + threadIdx.x;
  const int n_elems = meta->n_elems;
  if (g - (int)__lane_id() >= n_elems) return;  // whole wave past the end
  const int ji = wave_find_item(job_offsets, chunk_start, g, meta->n_jobs);
  if (g >= n_elems) return;
#if MM_REPROJ_BYVAL
  const BlockSetup su = setups[ji];
  reproj_thread_mc(g, ji, sc, jobs, job_offsets, su, cache, mc);
#else
  reproj_thread_mc(g, ji, sc, jobs, job_offsets, setups[ji], cache, mc);
#endif
}

// The tap-pair tables (4 KB) are copied into LDS once per workgroup: every lane indexes them by
// its own phase, and from __constant__ memory those lookups are ~16 vector loads per wave that
// compete with the reference-window loads for the texture-address path.
// amdgpu_waves_per_eu(3): 151 VGPRs, 3 waves per SIMD.  At 4 waves (128 VGPRs) the round-4 body spills
// 7 VGPRs to scratch; 3 spill-free waves are faster (C3 0.1735-0.1743 vs 0.1764-0.1792 ms per picture,
// k_mc 94-96 vs 97-99 us, profiles/r04_ab_occupancy.txt)
//
// Band-per-XCD mapping: the sub-blocks are enumerated bin by bin in picture order and cut into
// N_BANDS = 8 bands of about equal size (mm_devplan.h band_cut).  Workgroup b predicts band b % 8 --
// workgroups b and b + 8 share an XCD under the round-robin dealing (MI355X_MICROARCH.md, workgroup
// dispatch; speed only, results do not depend on it) -- taking the band's 256-sub-block blocks
// b / 8, b / 8 + gridDim / 8, ... (one block per workgroup with MC_BLOCKS_PER_WG = 1), so each XCD
// walks one band of the picture in decode order and keeps the reference rows that the band's
// neighbouring PUs share in its own L2.  Every workgroup stages the tap tables and the reference
// table in LDS once for all its blocks.
static_assert(N_BANDS == 8, "one band per XCD");
#ifndef MM_MC_WAVES
#define MM_MC_WAVES 3
#endif
template <bool UNI_HP>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MM_MC_WAVES))) k_mc_dev(Geometry geo, const PlanMeta* __restrict__ meta, McRec mc,
                                                const PicTables t, const DstPlanes dst) {
  const int band = blockIdx.x & 7, stride = (int)(gridDim.x >> 3) * 256;
  const int n_sb = meta->n_sb;  // (second guard: a band never reaches past the plan's sub-blocks)
  const int b0 = meta->band[band], b1 = min(meta->band[band + 1], n_sb);
  __shared__ PackedTaps s_taps;
  __shared__ RefDev s_ref[MAX_SLOTS];
  __shared__ DstPlanes s_dst;  // the pictures' planes, indexed per lane at the stores
  static_assert(sizeof(PackedTaps) % 16 == 0 && sizeof(PackedTaps) / 16 <= 256, "one 16-byte word per thread");
  const int first = b0 + (int)(blockIdx.x >> 3) * 256;
  if (first >= b1) return;  // whole workgroup past the band's end
#if defined(MM_MC_PRIO) && defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_s_setprio(MM_MC_PRIO);  // A/B: issue priority over the next picture's reprojection waves
#endif
  if (threadIdx.x < sizeof(PackedTaps) / 16)
    lds_put(reinterpret_cast<uint4*>(&s_taps)[threadIdx.x], reinterpret_cast<const uint4*>(&c_packed_taps)[threadIdx.x], make_uint4(~0u, ~0u, ~0u, ~0u));
  stage_ref_table<MAX_SLOTS>(t.pool_slot4, t.pool, s_ref);
  // (probe poison 0: a store through an unstaged plane pointer would fault rather than read garbage,
  // so the plane words get no poison store; the probe checks the taps and reference table)
  for (int k = threadIdx.x; k < (int)(sizeof(DstPlanes) / 4); k += blockDim.x)
    reinterpret_cast<uint32_t*>(&s_dst)[k] = reinterpret_cast<const uint32_t*>(&dst)[k];
  __syncthreads();
  const Taps taps{c_luma_taps, c_chroma_taps, &s_taps, t.pool};
  // s_ref: each lane looks its slots' pool offsets up in LDS; indexing the kernel-argument copy
  // per lane was a dependent global load between the record loads and the window loads
  // software-pipelined records: the next iteration's 24 bytes are in flight while this one predicts
  int g = first + (int)threadIdx.x;
  McIn cur = mc_rec_load(mc, min(g, b1 - 1));
  for (; g - (int)threadIdx.x < b1; g += stride) {
    const int gn = g + stride;
    McIn nxt;
    if (gn - (int)threadIdx.x < b1) nxt = mc_rec_load(mc, min(gn, b1 - 1));
    if (g < b1) mc_thread_in<UNI_HP>(g, cur, geo, taps, mc, s_ref, s_dst);
    cur = nxt;
  }
}
// k_mc grid: enough workgroups for MC_BLOCKS_PER_WG blocks of its band each (the band sizes are only
// known on the device; bands are at most ceil(sub-block capacity / 8) long).  One block per workgroup
// measured faster than a persistent 8 x 128 grid (profiles/r03_ab_mc_grid.txt): the dispatcher
// balances the workgroups over the CUs, and workgroups of the next picture's planning kernels that
// hold CU slots under plan-ahead no longer fix a late start to a persistent workgroup's whole share.
constexpr int MC_BLOCKS_PER_WG = 1;
// Plan-ahead events bound to kernel dispatches (hipExtLaunchKernelGGL stop events): ev_plan completes
// with k_setup_dev and a slot's gate with its k_mc_dev, so no marker packet sits between two
// pictures on the context stream (profiles/r03_ab_kernel_events.txt).
constexpr bool KERNEL_EVENTS = true;
constexpr bool GATE_NO_FENCE = true;
#ifndef MM_PLAN_HOST_WAIT
#define MM_PLAN_HOST_WAIT 0  // see launch_stripe
#endif
constexpr bool PLAN_AHEAD_HOST_WAIT = MM_PLAN_HOST_WAIT;
#ifndef MM_REPROJ_AHEAD
#define MM_REPROJ_AHEAD 1  // see launch_stripe
#endif
#ifndef MM_MC_LDS
#define MM_MC_LDS 0  // A/B knob: dynamic LDS per k_mc_dev workgroup, to cap its workgroups per CU
#endif
#ifndef MM_REPROJ_LDS
#define MM_REPROJ_LDS 0  // A/B knob: dynamic LDS per k_reproj_dev workgroup, to cap its workgroups per CU
#endif

// --------------------------------------------------------------------------------------------
// Encoder candidate windows (mm_sad_window, mm_me.h)
// --------------------------------------------------------------------------------------------
using namespace mmme;

__global__ void __launch_bounds__(256) k_me_setup(SeqConst sc, MeWindow w, const MeBlockDev* __restrict__ blocks,
                                                  int n_jobs, const PicTables t, BlockSetup* __restrict__ out) {
  __shared__ M3 s_ged[3 + MAX_SLOTS];  // indexed per lane: staged by stage_arg_words
  stage_arg_words<sizeof(s_ged) / 4>(reinterpret_cast<const uint32_t*>(t.ged), reinterpret_cast<uint32_t*>(s_ged));
  __syncthreads();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_jobs) return;
  me_setup_thread(i, sc, w, blocks, s_ged, out);
}

// thread per (block, window row j, sub-block e) looping over the row's candidates (mm_me.h
// me_elem_init / me_cand_sad); per candidate the sub-block SADs of a block are summed across the
// lanes that hold it (segmented shuffle scan) and added to sads[] by its last lane.
// chunk c of a batch's elements -> the block holding element 64 c (binary search of the block
// offsets); the device form of mm_plan.h build_chunks
__global__ void __launch_bounds__(256) k_me_chunks(const int* __restrict__ off, int n_items, long n_elems,
                                                   int* __restrict__ chunk) {
  const long c = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c * 64 >= n_elems) return;
  const long g = c * 64;
  int lo = 0, hi = n_items - 1;  // largest i with off[i] <= g
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (off[mid] <= g)
      lo = mid;
    else
      hi = mid - 1;
  }
  chunk[c] = lo;
}

// Orders one wave's LDS accesses (its lanes run in lockstep; LDS serves a wave's accesses in order)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

#ifndef MM_ME_WAVES
#define MM_ME_WAVES 4  // waves per SIMD of k_me_sad (its body alone would take 162 VGPRs: 3 waves)
#endif
// Window staging (MM_ME_LDS): a wave's lanes are consecutive window rows j of one block (16 lanes per
// row for a 16x16 block), so the 8-tap windows of all their candidates -- each candidate one sample
// step from the last -- fall in one box of about (block + 2 range + 8) x (block + 4 + 8) samples.  The
// wave loads that box into its LDS once and every candidate's window rows are then LDS reads
// instead of texture-path loads.  The box comes from each lane's first and last candidate plus
// ME_WIN_SLACK samples; a candidate whose window is not inside it (curved motion) and lanes of
// another block read the pool as before, so results never depend on the box.
#ifndef MM_ME_LDS
#define MM_ME_LDS 1
#endif
constexpr int ME_WIN_W = 88, ME_WIN_H = 48;           // staged box per wave: samples x rows
constexpr int ME_WIN_STRIDE = ME_WIN_W / 2 + 1;       // dwords per LDS row (odd: rows start on different banks)
[[maybe_unused]] constexpr int ME_WIN_SLACK = 2;
#ifndef MM_ME_LDS_TAPS
#define MM_ME_LDS_TAPS 1  // the packed tap pairs in LDS (each candidate's tap rows are position-dependent loads)
#endif
static_assert(MM_ME_WAVES * (4 * ME_WIN_H * ME_WIN_STRIDE * 4 + MAX_SLOTS * (int)sizeof(RefDev) +
                             (MM_ME_LDS_TAPS ? (int)sizeof(PackedLumaTaps) : 0)) <= 160 * 1024,
              "the workgroups of one CU fit its LDS");
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MM_ME_WAVES))) k_me_sad(SeqConst sc, Geometry geo, MeWindow w,
                                                const MeBlockDev* __restrict__ blocks, int n_blocks,
                                                const int* __restrict__ blk_off, const int* __restrict__ chunk,
                                                int n_elems, const BlockSetup* __restrict__ setups, MpaCache cache,
                                                const PicTables t, const int16_t* __restrict__ org, int org_stride,
                                                uint32_t* __restrict__ sads) {
  __shared__ RefDev s_ref[MAX_SLOTS];  // indexed per lane: staged by stage_ref_table
#if MM_ME_LDS && defined(__HIP_DEVICE_COMPILE__)
  __shared__ uint32_t s_win[4][ME_WIN_H * ME_WIN_STRIDE];  // per wave
#endif
  stage_ref_table<MAX_SLOTS>(t.pool_slot4, t.pool, s_ref);
#if MM_ME_LDS_TAPS && defined(__HIP_DEVICE_COMPILE__)
  // every candidate reads its (phase, parity) luma tap rows at a position-dependent address: from
  // LDS instead of a dependent constant-memory load ahead of each candidate's filter
  __shared__ PackedLumaTaps s_lt;
  static_assert(sizeof(PackedLumaTaps) / 16 <= 256, "one 16-byte word per thread");
  if (threadIdx.x < sizeof(PackedLumaTaps) / 16)
    lds_put(reinterpret_cast<uint4*>(&s_lt)[threadIdx.x], reinterpret_cast<const uint4*>(&c_packed_taps)[threadIdx.x],
            make_uint4(~0u, ~0u, ~0u, ~0u));
  [[maybe_unused]] const PackedLumaTaps* lt = &s_lt;
#else
  [[maybe_unused]] const PackedLumaTaps* lt = reinterpret_cast<const PackedLumaTaps*>(&c_packed_taps);  // its leading members
#endif
  __syncthreads();
  const int g = xcd_block() * blockDim.x + threadIdx.x;
  const int lane = __lane_id();
  if (g - lane >= n_elems) return;  // whole wave past the end
  const int bi = wave_find_item(blk_off, chunk, g, n_blocks);
  const bool active = g < n_elems;
  [[maybe_unused]] const Taps taps{c_luma_taps, c_chroma_taps, &c_packed_taps, t.pool};  // MM_ME_LDS 0 / host
  MeElem el;
  int j = 0, key = -1 - lane;  // inactive lanes: distinct keys that never merge
  if (active) {
    me_elem_init(g, bi, sc, w, blocks, setups, cache, org, org_stride, &el, &j);
    key = blocks[bi].sad_off + j * w.side;
  }
#if MM_ME_LDS && defined(__HIP_DEVICE_COMPILE__)
  // the box of the wave's last active lane's block, from its lanes' first and last candidates
  const uint64_t act = __ballot(active);
  const int bref = __shfl(bi, 63 - __clzll(act));
  const bool mine = active && bi == bref;
  int xmin = INT_MAX, xmax = INT_MIN, ymin = INT_MAX, ymax = INT_MIN;
  if (mine) {
#pragma unroll 1
    for (int q = 0; q < 2; q++) {
      int32_t fx, fy;
      me_cand_pos(el, q ? w.side - 1 : 0, j, bi, sc, w, setups, &fx, &fy);
      const int xPos = fx >> 4, yPos = fy >> 4;
      if (!me_out_of_range(xPos, yPos, geo)) {
        xmin = min(xmin, xPos);
        xmax = max(xmax, xPos);
        ymin = min(ymin, yPos);
        ymax = max(ymax, yPos);
      }
    }
  }
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    xmin = min(xmin, __shfl_xor(xmin, d));
    xmax = max(xmax, __shfl_xor(xmax, d));
    ymin = min(ymin, __shfl_xor(ymin, d));
    ymax = max(ymax, __shfl_xor(ymax, d));
  }
  const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const bool any = xmin <= xmax;  // some lane of the block has an in-range extreme candidate
  if (!any) xmin = xmax = ymin = ymax = 0;
  xmin += w.box_lx;  // a pattern's other candidates (0 for a window)
  xmax += w.box_hx;
  ymin += w.box_ly;
  ymax += w.box_hy;
  // columns [bx0, bx0 + 8 cw) hold every window (12 samples from its even start) of a position in
  // [xmin - SLACK, xmax + SLACK]; rows [by0, by0 + rows) every window's rows yPos - 3 .. yPos + 7
  const int bx0 = (xmin - ME_WIN_SLACK - 3) & ~1, by0 = ymin - ME_WIN_SLACK - 3;
  const int cw = (xmax + ME_WIN_SLACK + 9 - bx0 + 7) >> 3, rows = ymax + ME_WIN_SLACK + 8 - by0;
  const bool staged = any && cw * 8 <= ME_WIN_W && rows <= ME_WIN_H;
  if (staged) {  // wave-uniform
    const RefDev r = s_ref[__builtin_amdgcn_readfirstlane(blocks[bref].slot)];
    const char* src = t.pool.base + r.off_y + (long)(by0 * r.stride_y + bx0) * 2;
    for (int c4 = lane; c4 < rows * cw; c4 += 64) {
      const int rr = c4 / cw, c = c4 - rr * cw;
      typedef uint32_t u4a4 __attribute__((ext_vector_type(4), aligned(4)));
      const u4a4 q = *reinterpret_cast<const u4a4*>(src + ((long)rr * r.stride_y + 8 * c) * 2);
      uint32_t* dp = &s_win[wv][rr * ME_WIN_STRIDE + 4 * c];
      dp[0] = q.x;
      dp[1] = q.y;
      dp[2] = q.z;
      dp[3] = q.w;
    }
  }
  wave_lds_sync();
  const MeWin win{s_win[wv], ME_WIN_STRIDE, bx0, by0, bx0 + 8 * cw, by0 + rows};
  const bool use_win = staged && mine;
  const RefDev rme = s_ref[active ? blocks[bi].slot : 0];
  const int sub_shift = active ? blocks[bi].sub_shift : 0;
#endif
#pragma unroll 1
  for (int i = 0; i < w.side; i++) {  // uniform trip count (shuffles below)
    uint32_t v = 0;
#if MM_ME_LDS && defined(__HIP_DEVICE_COMPILE__)
    if (active) {
      // the whole setup by value: its seven 8-byte words are loaded together ahead of the tail (as a
      // reference into global memory the fields were loaded where used: C5 1,194 vs 1,228 Mcand/s)
      const BlockSetup su = setups[(long)bi * w.C + (long)j * w.side + i];
      v = me_cand_sad_win(el, su, i, j, sc, geo, t.pool, lt, rme, sub_shift, win, use_win);
    }
#else
    if (active) v = me_cand_sad(el, i, j, bi, sc, geo, taps, w, blocks, setups, s_ref);
#endif
    const int idx = active ? key + i : key;
#if defined(__HIP_DEVICE_COMPILE__)
    if (w.seg16) {  // lanes 16 k .. 16 k + 15 hold one (block, row): four DPP sums, no LDS round trips
      v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
      v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
      v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
      v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);  // row_mirror
      if (active && (lane & 15) == 0) atomicAdd(&sads[idx], v);
      continue;
    }
#endif
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t vu = __shfl_up(v, d);
      const int iu = __shfl_up(idx, d);
      if (lane >= d && iu == idx) v += vu;
    }
    const int inext = __shfl_down(idx, 1);
    if (active && (lane == 63 || inext != idx)) atomicAdd(&sads[idx], v);
  }
}

// --------------------------------------------------------------------------------------------
// MM-DMVR inside the device-planned picture (MM_PUF_DMVR PUs, mm_dmvr.h): k_plan_place placed the
// sub-PU records; these run between k_plan_place and k_setup_dev.  Their sizes live on the device
// (the DMVR share of a device-resident list is unknown to the host), so they loop over a fixed grid
// instead of capacity-sized grids of mostly idle workgroups.
// --------------------------------------------------------------------------------------------
using namespace mmdmvr;
constexpr int DMVR_GRID = 2048;  // workgroups of 256 of the grid-stride setup kernel

// The picture's DMVR survivors (sub-PUs whose centre cost does not end the search)
struct DmvrWork {
  unsigned* count;            // survivors (k_dmvr_centre_dev)
  uint32_t* ccost;            // centre cost (xDMVRCost at the merge MVs) per sub-PU
  int* surv_s;                // sub-PU of survivor k
  const CentreTerms* cterms;  // centre terms [2 s + l] (k_dmvr_setup_dev)
};

// thread per (sub-PU, list): the centre terms and the centre setup (the other 24 offsets' setups are
// derived from the terms by the search, for the survivors only); also clears the survivor count for
// k_dmvr_centre_dev
__global__ void __launch_bounds__(256) k_dmvr_setup_dev(SeqConst sc, const PlanMeta* __restrict__ meta,
                                                        const SubPuDev* __restrict__ sp, const PicTables t,
                                                        BlockSetup* __restrict__ out, CentreTerms* __restrict__ cterms,
                                                        unsigned* __restrict__ count) {
  __shared__ M3 s_ged[3 + MAX_SLOTS];  // indexed per lane: staged by stage_arg_words
  stage_arg_words<sizeof(s_ged) / 4>(reinterpret_cast<const uint32_t*>(t.ged), reinterpret_cast<uint32_t*>(s_ged));
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x == 0) *count = 0u;
  const int n_jobs = meta->n_sub * 2;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n_jobs; i += gridDim.x * blockDim.x)
    dmvr_centre_setup_thread(i, sc, sp, s_ged, out, cterms);
}

// The centre cost of every sub-PU (InterPrediction.cpp:2510-2525): 32 lanes per sub-PU, lane
// 2 e + l list l of luma 4x4 sub-block e -- its position at the merge MV and rows 0 and 2 of its
// 14-bit prediction; the L0 lane takes its partner's L1 rows by shuffle for the SAD, summed over
// the 32 lanes.  minCost = cost - cost/4 < dx*dy ends the search: the sub-PU keeps its merge MVs
// (dmvr_apply with a zero delta).  Otherwise it joins the survivor list, whose entries the
// workgroup's survivors take together with one atomic (a counter bumped per sub-PU serialised ~14 K
// device-scope atomics, ~100 µs; a separate one-workgroup scan kernel took 25 µs).  The list order
// varies from run to run; each survivor decides alone, so results do not.
__global__ void __launch_bounds__(256) k_dmvr_centre_dev(SeqConst sc, Geometry geo, const PlanMeta* __restrict__ meta,
                                                         const SubPuDev* __restrict__ sp,
                                                         const BlockSetup* __restrict__ setups, MpaCache cache,
                                                         const PicTables t, DmvrWork w, JobDev* __restrict__ jobs,
                                                         int32_t* __restrict__ mvd) {
#if defined(__HIP_DEVICE_COMPILE__)  // device-only filter paths (mm_filter.h predict_rows02, PtrRows)
  __shared__ PackedTaps s_taps;
  __shared__ RefDev s_ref[MAX_SLOTS];  // indexed per lane: staged by stage_ref_table
  __shared__ int s_surv[8], s_pre[8], s_base;
  const int tid = threadIdx.x;
  if (tid < sizeof(PackedTaps) / 16)
    lds_put(reinterpret_cast<uint4*>(&s_taps)[tid], reinterpret_cast<const uint4*>(&c_packed_taps)[tid], make_uint4(~0u, ~0u, ~0u, ~0u));
  stage_ref_table<MAX_SLOTS>(t.pool_slot4, t.pool, s_ref);
  if (tid < 8) lds_put(s_surv[tid], 0, 0);
  __syncthreads();
  const int n_sub = meta->n_sub;
  const RefPool pool = t.pool;
  for (int base = blockIdx.x * 256; base < n_sub * 32; base += gridDim.x * 256) {  // uniform trip count
    const int g = base + tid, s = g >> 5, e = (g >> 1) & 15, l = g & 1;
    int16_t p[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    SubPuDev u;
    if (s < n_sub) u = sp[s];
    if (s < n_sub && e < u.n) {
      int32_t fx, fy;
      dmvr_position(sc, u, setups[2 * s + l], cache, e, &fx, &fy);
      const int xPos = fx >> 4, yPos = fy >> 4;
      if (!sb_out_of_range(xPos, yPos, geo.W, geo.H, geo.maxCUw, geo.maxCUh, 4, 4)) {
        const RefDev& r = s_ref[l ? u.slot[1] : u.slot[0]];
        const int x0 = (xPos - 3) & ~1;
        const PtrRows rows{pool.base + r.off_y + (long)((yPos - 3) * r.stride_y + x0) * 2, r.stride_y * 2};
        predict_rows02(rows, s_taps.lh[fx & 15][(xPos - 3) & 1], s_taps.lv[fy & 15], geo.bd, p);
      }
    }
    uint32_t v = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint32_t mine = (uint32_t)(uint16_t)p[2 * j] | ((uint32_t)(uint16_t)p[2 * j + 1] << 16);
      const uint32_t other = __shfl_xor(mine, 1);
      v += (uint32_t)abs((int)(int16_t)(mine & 0xffffu) - (int)(int16_t)(other & 0xffffu)) +
           (uint32_t)abs((int)(int16_t)(mine >> 16) - (int)(int16_t)(other >> 16));
    }
    v = l ? 0u : v;  // each pair counted once
#pragma unroll
    for (int d = 1; d < 32; d <<= 1) v += __shfl_xor(v, d);
    // survivors of this workgroup's 8 sub-PUs: one atomic per workgroup allocates their list entries
    const int slot = tid >> 5;
    int survives = 0;
    if (s < n_sub && (g & 31) == 0) {
      w.ccost[s] = v;
      survives = v - (v >> 2) >= (uint32_t)(u.w * u.h) ? 1 : 0;
      if (!survives) dmvr_apply(s, u, 0, 0, jobs, mvd);  // notZeroCost = false: no refinement (:2520-2525)
      lds_put(s_surv[slot], survives, 0);
    }
    __syncthreads();
    if (tid == 0) {
      int ns = 0;
#pragma unroll
      for (int k = 0; k < 8; k++) {
        lds_put(s_pre[k], ns, 0);  // survivors before sub-PU k of the workgroup
        ns += (base + 32 * k < n_sub * 32) ? s_surv[k] : 0;
      }
      lds_put(s_base, ns ? (int)atomicAdd(w.count, (unsigned)ns) : 0, 0);
    }
    __syncthreads();
    if (survives) w.surv_s[s_base + s_pre[slot]] = s;
    __syncthreads();  // s_surv / s_pre / s_base reused by the next iteration
  }
#endif
}

// The search of one surviving sub-PU per wave (xProcessDMVRProjected, InterPrediction.cpp:2526-2580).
// Each wave of a workgroup takes its own survivors and its own LDS region; the workgroup shares only
// the tap tables and the GED rotations.  Lane L = part * 2n + 2 e + l serves luma 4x4 sub-block e of
// list l at the part's 24 / P offsets (P = 64 / 2n parts: 2 for a 16x16 sub-PU, 4 for 16x8 / 8x16):
//   0. the 24 non-centre offsets' setups of both lists (lanes 0..47) into the wave's LDS -- only the
//      MV part, from the centre terms k_dmvr_setup_dev stored (mm_models.h setup_from_centre);
//   1. the lane's positions at its offsets, kept in registers -- the model's MV-independent head once,
//      the tail per offset (mm_dmvr.h dmvr_positions_offsets) -- and per list the bounding box of the
//      in-range windows (wave shuffles);
//   2. the union of every offset's luma window, per list, staged once into the wave's LDS (16-byte
//      loads): the 24 x n windows of a list lie within about (dx + 11) x (dy + 11) samples, so each
//      staged sample serves ~50 window reads; a union larger than the LDS window (strong warping, the
//      ERP seam) reads the pool directly instead;
//   3. per offset, rows 0 and 2 of the lane's 14-bit prediction; the L0 lane takes its partner's L1
//      rows by shuffle for the SAD, summed over the part's n sub-blocks (xor shuffles);
//   4. the decision (the centre cost from k_dmvr_centre_dev, first strict minimum, error surface) and
//      the refined MVs into the sub-PU's jobs (lane 0).
// The phases of one survivor are ordered by wave-level fences only, so a wave waiting on its window
// loads never holds the others of its workgroup.  C3 at a 30 % share (profiles/r05_ab_dmvr.txt):
// 0.674-0.685 ms per picture, against 0.689-0.695 for round 4's split (positions written to HBM by a
// separate reprojection kernel and read back; 0.9 GB of work buffers per context); 0.715-0.730 at 3
// waves with the setups computed in full here (162 VGPRs, 44 K instructions); 0.77-0.82 for a first
// form with one survivor per 256-thread workgroup and five workgroup barriers per survivor.
constexpr int DMVR_WAVES = 4;                  // waves (survivors in flight) per workgroup
constexpr int DMVR_SEARCH_WG = 64 * DMVR_WAVES;
constexpr int DMVR_LANE_OFFS = 12;             // offsets per lane of a 16x16 sub-PU (24 / 2 parts)
#ifndef MM_DMVR_WIN_W
#define MM_DMVR_WIN_W 40  // a 16x16 sub-PU's 24 offsets span ~(16 + 4 + 11)^2 samples; larger unions read the pool
#define MM_DMVR_WIN_H 32
#endif
constexpr int DMVR_WIN_W = MM_DMVR_WIN_W;  // staged union window per list: samples x rows
constexpr int DMVR_WIN_H = MM_DMVR_WIN_H;
constexpr int DMVR_WIN_STRIDE = DMVR_WIN_W / 2 + 1;  // dwords per LDS row: odd, so rows start on different banks
struct DmvrWaveLds {
  uint32_t win[2][DMVR_WIN_H * DMVR_WIN_STRIDE];
  BlockSetup set[N_OFF - 1][2];  // the survivor's 24 non-centre offsets x 2 lists
  uint32_t cost[N_OFF];
};
static_assert(2 * (N_OFF - 1) <= 64, "one lane per (offset, list) setup");
static_assert((N_OFF - 1) % 4 == 0 && (N_OFF - 1) / 2 == DMVR_LANE_OFFS, "24 offsets split over 2 or 4 parts");


#ifndef MM_DMVR_SEARCH_WAVES
#define MM_DMVR_SEARCH_WAVES 4  // waves per SIMD = workgroups per CU (LDS): 128 VGPRs, spill-free
#endif
constexpr int DMVR_SEARCH_GRID = 256 * MM_DMVR_SEARCH_WAVES;  // grid-stride over the survivors
static_assert(MM_DMVR_SEARCH_WAVES * (sizeof(DmvrWaveLds) * DMVR_WAVES + sizeof(PackedTaps) + (3 + MAX_SLOTS) * sizeof(M3)) <=
                  160 * 1024,
              "the workgroups of one CU fit its LDS");
__global__ void __launch_bounds__(DMVR_SEARCH_WG) __attribute__((amdgpu_waves_per_eu(MM_DMVR_SEARCH_WAVES))) k_dmvr_search_dev(
    SeqConst sc, Geometry geo, const SubPuDev* __restrict__ sp, MpaCache cache, const PicTables t, DmvrWork w,
    JobDev* __restrict__ jobs, int32_t* __restrict__ mvd) {
#if defined(__HIP_DEVICE_COMPILE__)  // device-only filter paths (mm_filter.h predict_rows02, PtrRows, LdsRows)
  __shared__ PackedTaps s_taps;
  __shared__ M3 s_ged[3 + MAX_SLOTS];  // indexed per lane: staged by stage_arg_words
  __shared__ DmvrWaveLds s_wave[DMVR_WAVES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  DmvrWaveLds& L = s_wave[wv];
  static_assert(sizeof(PackedTaps) % 16 == 0 && sizeof(PackedTaps) / 16 <= DMVR_SEARCH_WG, "one 16-byte word per thread");
  if (tid < sizeof(PackedTaps) / 16)
    lds_put(reinterpret_cast<uint4*>(&s_taps)[tid], reinterpret_cast<const uint4*>(&c_packed_taps)[tid], make_uint4(~0u, ~0u, ~0u, ~0u));
  stage_arg_words<sizeof(s_ged) / 4>(reinterpret_cast<const uint32_t*>(t.ged), reinterpret_cast<uint32_t*>(s_ged));
  __syncthreads();  // s_taps, s_ged: the only LDS the waves share
#if defined(MM_DMVR_PROBE_NOSEARCH)  // timing probe (wrong results): no survivor is searched
  const int n_surv = 0;
#else
  const int n_surv = (int)*w.count;
#endif
  const RefPool pool = t.pool;
  for (int k = blockIdx.x * DMVR_WAVES + wv; k < n_surv; k += gridDim.x * DMVR_WAVES) {
    const int s = w.surv_s[k];
    const SubPuDev u = sp[s];
    const int n = u.n, log2n = 31 - __clz(n);                       // n: 8 or 16
    const int n_offs = DMVR_LANE_OFFS >> (4 - log2n);               // 12 or 6 offsets per lane
    const int part = lane >> (log2n + 1), e = (lane >> 1) & (n - 1), l = lane & 1;
    // the sub-PU's slots are uniform: scalar loads of the kernel argument's table
    const int slot0 = __builtin_amdgcn_readfirstlane(u.slot[0]), slot1 = __builtin_amdgcn_readfirstlane(u.slot[1]);
    const uint32_t off_y[2] = {t.ref[slot0].off_y, t.ref[slot1].off_y};
    const int stride_y[2] = {t.ref[slot0].stride_y, t.ref[slot1].stride_y};
    if (lane < 2 * (N_OFF - 1)) {  // 0. the 24 non-centre offsets' setups of both lists
      BlockSetup b;
      dmvr_offset_setup(sc, u, dmvr_outer_offset(lane >> 1), lane & 1, w.cterms[2 * s + (lane & 1)], s_ged, &b);
      lds_put(L.set[lane >> 1][lane & 1], b, BlockSetup{});
    }
    if (lane == 0) lds_put(L.cost[N_OFF / 2], w.ccost[s], 0u);
    wave_lds_sync();
    // 1. this lane's positions, and the in-range box of its list
    int32_t pfx[DMVR_LANE_OFFS] = {}, pfy[DMVR_LANE_OFFS] = {};
    int xmin = INT_MAX, xmax = INT_MIN, ymin = INT_MAX, ymax = INT_MIN;
#if defined(MM_DMVR_PROBE_NOTAIL)  // timing probe (wrong results): translational positions, no model
    auto positions = [&](auto out) {
      const int col = e / u.rows, row = e - col * u.rows, sg = l ? -1 : 1;
      for (int j = 0; j < n_offs; j++) {
        const int o = dmvr_outer_offset(part * n_offs + j);
        out(j, 16 * (u.x + 4 * col) + u.mv[l][0] + sg * 16 * mmdmvr::off_x(o), 16 * (u.y + 4 * row) + u.mv[l][1] + sg * 16 * mmdmvr::off_y(o));
      }
    };
#else
    auto positions = [&](auto out) {
      dmvr_positions_offsets(sc, u, l, e, cache, [&](int j) -> const BlockSetup& { return L.set[part * n_offs + j][l]; },
                             n_offs, out);
    };
#endif
    positions([&](int j, int32_t fx, int32_t fy) {
#pragma unroll
                             for (int q = 0; q < DMVR_LANE_OFFS; q++)
                               if (q == j) {
                                 pfx[q] = fx;
                                 pfy[q] = fy;
                               }
                             const int xPos = fx >> 4, yPos = fy >> 4;
                             if (!sb_out_of_range(xPos, yPos, geo.W, geo.H, geo.maxCUw, geo.maxCUh, 4, 4)) {
                               xmin = min(xmin, xPos);
                               xmax = max(xmax, xPos);
                               ymin = min(ymin, yPos);
                               ymax = max(ymax, yPos);
                             }
                           });
#pragma unroll
    for (int d = 2; d < 64; d <<= 1) {  // over the lanes of the same list (same parity)
      xmin = min(xmin, __shfl_xor(xmin, d));
      xmax = max(xmax, __shfl_xor(xmax, d));
      ymin = min(ymin, __shfl_xor(ymin, d));
      ymax = max(ymax, __shfl_xor(ymax, d));
    }
    // 2. stage the union windows: columns [bx0, bx0 + 8 cw), rows [by0, by0 + rows)
    int bx0[2], by0[2];
    bool staged[2];
#pragma unroll
    for (int ll = 0; ll < 2; ll++) {
      const int bxmin = __shfl(xmin, ll), bxmax = __shfl(xmax, ll), bymin = __shfl(ymin, ll), bymax = __shfl(ymax, ll);
      bx0[ll] = (bxmin - 3) & ~1;
      by0[ll] = bymin - 3;
      const int cw = (bxmax + 9 - bx0[ll] + 7) >> 3, rows = bymax - bymin + 11;  // 16-byte chunks per row, rows
      staged[ll] = bxmin <= bxmax && cw * 8 <= DMVR_WIN_W && rows <= DMVR_WIN_H;
#if defined(MM_DMVR_PROBE_NOSTAGE)  // A/B: no union window in LDS, every row from the pool (same results)
      staged[ll] = false;
#endif
      if (staged[ll]) {
        const char* src = pool.base + off_y[ll] + (long)(by0[ll] * stride_y[ll] + bx0[ll]) * 2;
        for (int c4 = lane; c4 < rows * cw; c4 += 64) {
          const int r = c4 / cw, c = c4 - r * cw;
          typedef uint32_t u4a4 __attribute__((ext_vector_type(4), aligned(4)));
          const u4a4 q = *reinterpret_cast<const u4a4*>(src + ((long)r * stride_y[ll] + 8 * c) * 2);
          uint32_t* dp = &L.win[ll][r * DMVR_WIN_STRIDE + 4 * c];
          lds_put(dp[0], q.x, ~0u);
          dp[1] = q.y;
          dp[2] = q.z;
          dp[3] = q.w;
        }
      }
    }
    wave_lds_sync();
    // 3. rows 0 and 2 of the lane's prediction per offset; SAD against the partner list's, per offset
    const uint32_t* win = L.win[l];
    const int wbx0 = l ? bx0[1] : bx0[0], wby0 = l ? by0[1] : by0[0];
    const bool wstaged = l ? staged[1] : staged[0];
    const uint32_t woff = l ? off_y[1] : off_y[0];
    const int wstride = l ? stride_y[1] : stride_y[0];
#pragma unroll 1
    for (int j = 0; j < n_offs; j++) {
      int32_t fx = pfx[0], fy = pfy[0];
#pragma unroll
      for (int q = 1; q < DMVR_LANE_OFFS; q++)
        if (q == j) {
          fx = pfx[q];
          fy = pfy[q];
        }
      const int xPos = fx >> 4, yPos = fy >> 4;
      int16_t p[8];
      if (sb_out_of_range(xPos, yPos, geo.W, geo.H, geo.maxCUw, geo.maxCUh, 4, 4)) {
#pragma unroll
        for (int i = 0; i < 8; i++) p[i] = 0;
      } else {
        const uint32_t* ht = s_taps.lh[fx & 15][(xPos - 3) & 1];
        const uint32_t* vt = s_taps.lv[fy & 15];
        const int x0 = (xPos - 3) & ~1;
#if defined(MM_DMVR_PROBE_NOFILTER)  // timing probe (wrong results): one window word, no filter
        if (wstaged) {
          const uint32_t q = win[(yPos - 3 - wby0) * DMVR_WIN_STRIDE + ((x0 - wbx0) >> 1)] ^ ht[0] ^ vt[0];
#pragma unroll
          for (int i = 0; i < 8; i++) p[i] = (int16_t)(q >> i);
        } else {
#else
        if (wstaged) {
          const LdsRows rows{&win[(yPos - 3 - wby0) * DMVR_WIN_STRIDE + ((x0 - wbx0) >> 1)], DMVR_WIN_STRIDE};
          predict_rows02(rows, ht, vt, geo.bd, p);
        } else {
#endif
          const PtrRows rows{pool.base + woff + (long)((yPos - 3) * wstride + x0) * 2, wstride * 2};
          predict_rows02(rows, ht, vt, geo.bd, p);
        }
      }
      uint32_t v = 0;
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const uint32_t mine = (uint32_t)(uint16_t)p[2 * i] | ((uint32_t)(uint16_t)p[2 * i + 1] << 16);
        const uint32_t other = __shfl_xor(mine, 1);
        v += (uint32_t)abs((int)(int16_t)(mine & 0xffffu) - (int)(int16_t)(other & 0xffffu)) +
             (uint32_t)abs((int)(int16_t)(mine >> 16) - (int)(int16_t)(other >> 16));
      }
      for (int d = 2; d < 2 * n; d <<= 1) v += __shfl_xor(v, d);  // the part's n sub-blocks (same list)
      if ((lane & (2 * n - 1)) == 0) lds_put(L.cost[dmvr_outer_offset(part * n_offs + j)], v, 0u);
    }
    wave_lds_sync();
    // 4. the decision and the refined MVs
    if (lane == 0) {
      int tdx, tdy;
      dmvr_decide(u, L.cost, &tdx, &tdy);
      dmvr_apply(s, u, tdx, tdy, jobs, mvd);
    }
    wave_lds_sync();  // the decision's reads before the next survivor's setups
  }
#endif
}

// --------------------------------------------------------------------------------------------
// MM-MVP (mm_mvp_convert, mm_mvp.h)
// --------------------------------------------------------------------------------------------
// One workgroup converts 256 queries.  The two model evaluations of a query (the candidate's
// modelMotion, then the desired model's equivalent MV) each branch on a model id, and a wave of
// arbitrary queries would run every model's code one after another.  So between the steps the
// workgroup regroups its queries through LDS: step 1 runs on the queries ordered by the candidate's
// model, step 2 on them ordered by the desired model (a counting sort of 256 keys each time), and
// each wave then runs one or two models' code.  Early returns and failing queries take no slot.
constexpr int MVP_BLOCK = 256;
constexpr int MVP_KEYS = NUM_MODELS;
__device__ __forceinline__ void mvp_regroup(int key, int* s_cnt, int* s_perm, int* n_work) {
  const int tid = threadIdx.x;
  if (tid < MVP_KEYS) lds_put(s_cnt[tid], 0, 0);
  __syncthreads();
  int rank = 0;
  if (key >= 0) rank = atomicAdd(&s_cnt[key], 1);
  __syncthreads();
  if (tid == 0) {
    int acc = 0;
    for (int k = 0; k < MVP_KEYS; k++) {
      const int c = s_cnt[k];
      lds_put(s_cnt[k], acc, 0);
      acc += c;
    }
    lds_put(s_cnt[MVP_KEYS], acc, 0);
  }
  __syncthreads();
  if (key >= 0) lds_put(s_perm[s_cnt[key] + rank], tid, 0);
  __syncthreads();
  *n_work = s_cnt[MVP_KEYS];
}

// Queries sorted by (candidate model, desired model) before k_mvp_dev: a launch over the bench's
// query mix took 74 us, the same queries in model order 41 us -- workgroups that run one model
// pair keep its code in the instruction cache (tools/mvp_probe.py).  A counting sort in two small
// kernels: k_mvp_bucket counts the keys of its 256 queries in LDS and takes each key's range with
// one atomic per key and workgroup (the order inside a key varies from run to run; each query
// converts alone, so results do not); k_mvp_place adds the keys' starts.  Each key has MVP_SUBS
// counters, workgroup b adding to counter b % MVP_SUBS: one counter per key took all ~600
// workgroups' atomics on the keys' 121 addresses (k_mvp_bucket 17 us on the bench mix, profiles/
// r04_mvp_sort.txt).  The counters alternate between calls: a call's k_mvp_bucket clears the next
// call's set.
constexpr int MVP_BINS = NUM_MODELS * NUM_MODELS;
constexpr int MVP_SUBS = 8;
constexpr int MVP_COUNTERS = MVP_BINS * MVP_SUBS;  // [key][sub]
constexpr int MVP_SORT_MIN = 32768;  // batches at least this large are sorted (mm_mvp_convert_device)
static_assert(MVP_BINS <= MVP_BLOCK, "k_mvp_place gives every key one thread");
__device__ __forceinline__ int mvp_key(const mm_mvp_query& x) {
  const bool ok = x.model_orig >= 0 && x.model_orig < NUM_MODELS && x.model_desired >= 0 && x.model_desired < NUM_MODELS;
  return ok ? x.model_orig * NUM_MODELS + x.model_desired : 0;
}
__global__ void __launch_bounds__(MVP_BLOCK) k_mvp_bucket(const mm_mvp_query* __restrict__ q, int n,
                                                          unsigned* __restrict__ bins, unsigned* __restrict__ next_bins,
                                                          int* __restrict__ local) {
  __shared__ unsigned s_h[MVP_BINS], s_base[MVP_BINS];
  const int tid = threadIdx.x, i = blockIdx.x * MVP_BLOCK + tid, sub = blockIdx.x % MVP_SUBS;
  for (int b = tid; b < MVP_BINS; b += MVP_BLOCK) lds_put(s_h[b], 0u, 0u);
  if (blockIdx.x == 0)
    for (int b = tid; b < MVP_COUNTERS; b += MVP_BLOCK) next_bins[b] = 0u;
  __syncthreads();
  int key = 0;
  unsigned rank = 0;
  if (i < n) {
    key = mvp_key(q[i]);
    rank = atomicAdd(&s_h[key], 1u);
  }
  __syncthreads();
  for (int b = tid; b < MVP_BINS; b += MVP_BLOCK)
    if (s_h[b]) lds_put(s_base[b], atomicAdd(&bins[b * MVP_SUBS + sub], s_h[b]), 0u);
  __syncthreads();
  if (i < n) local[i] = (int)(s_base[key] + rank);
}
__global__ void __launch_bounds__(MVP_BLOCK) k_mvp_place(const mm_mvp_query* __restrict__ q, int n,
                                                         const unsigned* __restrict__ bins,
                                                         const int* __restrict__ local, int* __restrict__ perm) {
  __shared__ unsigned s_cnt[MVP_COUNTERS], s_key[MVP_BINS];
  const int tid = threadIdx.x, i = blockIdx.x * MVP_BLOCK + tid, sub = blockIdx.x % MVP_SUBS;
  for (int k = tid; k < MVP_COUNTERS; k += MVP_BLOCK) lds_put(s_cnt[k], bins[k], 0u);
  __syncthreads();
  // this workgroup's counter of key b starts after the key's earlier counters (thread b) ...
  if (tid < MVP_BINS) {
    unsigned acc = 0;
    for (int j = 0; j < MVP_SUBS; j++) {
      const unsigned c = s_cnt[tid * MVP_SUBS + j];
      if (j == sub) s_cnt[tid * MVP_SUBS] = acc;  // (slot j = 0 is read before it is overwritten)
      acc += c;
    }
    lds_put(s_key[tid], acc, 0u);
  }
  __syncthreads();
  // ... and after all earlier keys (one thread scans the MVP_BINS = 121 key totals)
  if (tid == 0) {
    unsigned acc = 0;
    for (int b = 0; b < MVP_BINS; b++) {
      const unsigned t = s_key[b];
      lds_put(s_key[b], acc, 0u);
      acc += t;
    }
  }
  __syncthreads();
  if (i < n) {
    const int key = mvp_key(q[i]);
    perm[s_key[key] + s_cnt[key * MVP_SUBS] + local[i]] = i;
  }
}

__global__ void __launch_bounds__(MVP_BLOCK) k_mvp_dev(SeqConst sc, const mm_mvp_query* __restrict__ q, int n,
                                                       const int* __restrict__ order, uint32_t active, mmmvp::EpiTable et,
                                                       int32_t* __restrict__ out, unsigned long long* __restrict__ status) {
  using namespace mmmvp;
  __shared__ mm_mvp_query s_q[MVP_BLOCK];
  __shared__ float s_sx[MVP_BLOCK], s_sy[MVP_BLOCK];
  __shared__ int s_perm[MVP_BLOCK], s_cnt[MVP_KEYS + 1], s_ok[MVP_BLOCK], s_qi[MVP_BLOCK];
  __shared__ unsigned long long s_status;
  const int tid = threadIdx.x, i0 = blockIdx.x * MVP_BLOCK, i = i0 + tid;
  if (tid == 0) lds_put(s_status, 0ull, 0ull);
  __syncthreads();  // s_status is zeroed before any wave's atomicMax (waves 1-3 may run ahead of wave 0)
  int key = -1;
  if (i < n) {
    const int qi = order ? order[i] : i;  // the query this thread converts (model order)
    lds_put(s_qi[tid], qi, 0);
    const mm_mvp_query x = q[qi];
    lds_put(s_q[tid], x, mm_mvp_query{});
    int32_t o[2] = {0, 0};
    int code = mvp_validate(x, active);
    if (code == MM_OK && !mvp_early(x, et, o, &code)) key = x.model_orig;
    if (key < 0) {
      out[2 * qi] = o[0];
      out[2 * qi + 1] = o[1];
    }
    if (code) atomicMax(&s_status, status_word(qi, code));
  }
  int nw;
  mvp_regroup(key, s_cnt, s_perm, &nw);
  // step 1 in candidate-model order
  if (tid < nw) {
    const int k = s_perm[tid];
    float sx = 0.0f, sy = 0.0f;
    const bool ok = mvp_candidate_motion(sc, s_q[k], et, &sx, &sy);
    if (!ok) {
      const int qk = s_qi[k];
      atomicMax(&s_status, status_word(qk, MM_ERR_NOEPIPOLE));
      out[2 * qk] = out[2 * qk + 1] = 0;
    }
    lds_put(s_sx[k], sx, __int_as_float(0x7fc00000));
    s_sy[k] = sy;
    lds_put(s_ok[k], ok ? 1 : 0, 0);
  }
  __syncthreads();
  const int key2 = (key >= 0 && s_ok[tid]) ? s_q[tid].model_desired : -1;
  mvp_regroup(key2, s_cnt, s_perm, &nw);
  // step 2 in desired-model order
  if (tid < nw) {
    const int k = s_perm[tid];
    int32_t o[2] = {0, 0};
    const int qk = s_qi[k];
    if (!mvp_desired_mv(sc, s_q[k], et, s_sx[k], s_sy[k], o)) atomicMax(&s_status, status_word(qk, MM_ERR_NOEPIPOLE));
    out[2 * qk] = o[0];
    out[2 * qk + 1] = o[1];
  }
  __syncthreads();
  if (tid == 0 && s_status) atomicMax(status, s_status);
}

// InterpolationFilter::filter<N, isVertical, isFirst, isLast> / filterCopy on a raw block
// (parity API mm_filter; InterpolationFilter.cpp:392-644)
__global__ void k_filter(int comp, int vertical, const int16_t* src, int src_stride, int16_t* dst, int dst_stride,
                         int w, int h, int frac, int is_first, int is_last, int bd) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= w * h) return;
  int r = t / w, c = t % w;
  const int NT = comp ? 4 : 8;
  const int8_t* cf = comp ? c_chroma_taps[frac] : c_luma_taps[frac];
  const int maxv = (1 << bd) - 1;
  int v;
  if (frac == 0) {
    int s = src[(long)r * src_stride + c];
    const int sh = if_internal_frac_bits(bd);
    if (is_first == is_last)
      v = s;
    else if (is_first)
      v = (int16_t)((int16_t)(s << sh) - (int16_t)IF_INTERNAL_OFFS);
    else
      v = clip_pel((int16_t)((s + IF_INTERNAL_OFFS + (1 << (sh - 1))) >> sh), maxv);
  } else {
    FiltParam fp = filt_param(is_first != 0, is_last != 0, bd);
    const long cs = vertical ? src_stride : 1;
    const int16_t* p = src + (long)r * src_stride + c - (NT / 2 - 1) * cs;
    int sum = 0;
    for (int k = 0; k < NT; k++) sum += p[k * cs] * cf[k];
    v = (int16_t)((sum + fp.offset) >> fp.shift);
    if (fp.clip) v = clip_pel(v, maxv);
  }
  dst[(long)r * dst_stride + c] = (int16_t)v;
}

}  // namespace

// ============================================================================================
// Host side: context and C-ABI
// ============================================================================================
using namespace mmplan;

struct RefHost {
  int16_t* y = nullptr;
  int16_t* cb = nullptr;
  int16_t* cr = nullptr;
  int stride_y = 0, stride_c = 0;
  int slot = -1;  // picture slot in the context's reference pool (-1: own allocation, e.g. originals)
};

struct mm_ctx;
static hipError_t dev_alloc(mm_ctx* c, void** p, size_t bytes);
static void dev_free(mm_ctx* c, void* p);

// The buffers that grow with the pictures come from the device's stream-ordered pool
// (hipMallocAsync / hipFreeAsync on the context stream, dev_alloc / dev_free): hipFree -- and
// hipFreeAsync of memory hipMalloc returned -- waits for every queue of the device (a busy kernel on
// another stream held it for the kernel's whole 266 ms, tools/ubench/free_sync.hip), so a context that
// grew or was destroyed would stall every other context in flight; a pool free is ordered on the
// context stream only (0.02 ms, its stream done in 0.1 ms beside the same kernel).
template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t cap = 0;
  // fresh (optional): set when the buffer was (re)allocated by this call
  hipError_t ensure(mm_ctx* c, size_t n, bool* fresh = nullptr) {
    if (fresh) *fresh = false;
    if (n <= cap && p) return hipSuccess;
    // Growing replaces a buffer that work still queued on the context's streams may use (the host
    // runs pictures ahead of the GPU): the old allocation is freed in stream order behind that work
    // (dev_free), nothing waits on the host.  Growth is geometric (x1.5), so a list that creeps up
    // picture by picture reallocates a few times, not every picture.
    size_t want = std::max<size_t>(n, 1);
    if (p) want = std::max(want, cap + cap / 2);
    void* q = nullptr;
    const hipError_t e = dev_alloc(c, &q, want * sizeof(T));
    if (e != hipSuccess) return e;
    if (p) dev_free(c, p);
    p = static_cast<T*>(q);
    cap = want;
    if (fresh) *fresh = true;
    return hipSuccess;
  }
  void release(mm_ctx* c) {
    if (p) dev_free(c, p);
    p = nullptr;
    cap = 0;
  }
};

// Buffers of one device-planned stripe of a picture.
struct PlanSlot {
  DevBuf<int> job_off, job_chunk;
  DevBuf<JobDev> jobs;
  DevBuf<BlockSetup> setup;
  DevBuf<unsigned long long> blk;   // per-count-block bucket counts (k_plan_count rows)
  DevBuf<unsigned long long> blkq;  // per-quarter bucket counts
  DevBuf<PlanMeta> meta;
  DevBuf<mm_int2> mc_meta;
  DevBuf<uint32_t> mc_lpos[2], mc_cpos[2];
  DevBuf<mm_int2> mc_far[2][2];
  DevBuf<SubPuDev> dmvr_sub;  // MM-DMVR sub-PU records (k_plan_place) and their element offsets / chunks
  DevBuf<int> dmvr_off, dmvr_chunk;
  // MM-DMVR work of the slot's picture: centre setups [2 s + l], refined deltas, survivor list
  DevBuf<BlockSetup> dmvr_setup;
  DevBuf<CentreTerms> dmvr_cterms;
  DevBuf<int> dmvr_mvd, dmvr_surv_s;
  DevBuf<unsigned> dmvr_count;
  DevBuf<uint32_t> dmvr_ccost;
  int n_ensured = 0;  // largest stripe size the buffers were sized for (they only grow)
  int pics_ensured = 1;  // pictures per call the sub-block capacity covers (mm_pred_device_multi)
  bool dmvr_ensured = false;
  PlanCaps caps{};
  void release(mm_ctx* c) {
    dmvr_sub.release(c);
    dmvr_off.release(c);
    dmvr_chunk.release(c);
    dmvr_setup.release(c);
    dmvr_cterms.release(c);
    dmvr_mvd.release(c);
    dmvr_surv_s.release(c);
    dmvr_count.release(c);
    dmvr_ccost.release(c);
    job_off.release(c);
    job_chunk.release(c);
    jobs.release(c);
    setup.release(c);
    blk.release(c);
    blkq.release(c);
    meta.release(c);
    mc_meta.release(c);
    for (int l = 0; l < 2; l++) {
      mc_lpos[l].release(c);
      mc_cpos[l].release(c);
      for (int k = 0; k < 2; k++) mc_far[l][k].release(c);
    }
  }
};

// Stripes a device-planned picture is cut into (mm_set_stripes)
#ifndef MM_DEFAULT_STRIPES
#define MM_DEFAULT_STRIPES 1
#endif

// C-ABI handle of an EpipoleList: standalone (owned) or a context's own list
struct mm_epipole_list {
  mmepi::EpipoleList* l;
  bool owned;
  // mm_mvp_convert_host: the available entries in key order (the device table's layout), rebuilt
  // when the list's version moves
  std::vector<mmmvp::EpiDev> host;
  unsigned long long host_version = ~0ull;
};

struct mm_ctx {
  mm_seq_params prm{};
  SeqConst sc{};
  Geometry geo{};
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  std::map<int, RefHost> refs;
  // Reference pool: every resident reference picture in one allocation of pool_cap picture slots
  // (Y | interleaved CbCr, rows 128-byte aligned); kernels address planes by 32-bit byte offsets from
  // the pool base (RefDev::off_y / off_cb, mm_filter.h RefPool), so the pool stays below 2 GiB.
  char* pool = nullptr;
  int16_t* chroma_stage = nullptr;  // host-sourced Cb | Cr planes on their way into the pool
  size_t pic_bytes = 0;
  int pool_cap = 0;
  std::vector<int> pool_free;
  EpipoleMap epipoles;                            // the context's EpipoleList (mm_epipole.h)
  mm_epipole_list epi_handle{&epipoles, false};   // its C-ABI handle (mm_get_epipole_list)
  float* trig = nullptr;  // separable toSphere table of the frame grid (MpaCache::trig_col / trig_row)
  TanEntry* tan_grid = nullptr;  // TAN's first step per grid point (MpaCache::tan_grid), when TAN is active
  float* mpa_px = nullptr;  // the three MPA planes back to back (MpaCache)
  float* mpa_py = nullptr;
  uint8_t* mpa_vip = nullptr;
  Plan plan;  // host plan of the parity API mm_reproject
  DevBuf<JobDev> d_jobs;
  DevBuf<int> d_job_off, d_job_chunk, d_pu_off, d_pu_chunk;
  DevBuf<BlockSetup> d_setup;
  DevBuf<int32_t> d_reproj;
  DevBuf<M3> d_ged;
  // device-planned prediction (mm_pred_device / mm_pred_run)
  DevBuf<mm_pu_desc> d_pu_in;  // PU list copied in by mm_pred / mm_pred_prepare
  PlanSlot slot[2];             // device-planned stripes alternate between the two buffer sets
  hipStream_t aux = nullptr;    // odd stripes run here, overlapping the even stripes' kernels
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  int n_stripes = MM_DEFAULT_STRIPES;
  // plan-ahead (mm_set_plan_ahead): a picture's planning + setup run on `aux` once its slot's gate
  // (the previous user's k_mc_dev) is done, concurrently with the previous call's kernels; the
  // context stream waits for ev_plan before the reprojection
  bool plan_ahead = false;
  int ahead_par = 0;                               // slot of the next plan-ahead picture
  int last_slot = 0;  // plan slot of the last call's (first) stripe: where its MM-DMVR deltas are
  hipEvent_t ev_gate[2] = {nullptr, nullptr};      // ev_gate[s]: the last k_mc_dev using slot s is done
  // mm_set_kernel_timing: every k_mc_dev launch bracketed by a kernel-bound start / stop event pair
  // from this ring (hipExtLaunchKernelGGL), read back by mm_kernel_times; under plan-ahead the stop
  // event doubles as the slot's gate (gate[s] points at it), so the timed loop records no extra packet
  static constexpr int KT_RING = 256;
  bool kt_on = false;
  int kt_n = 0;                                    // launches recorded since the last mm_kernel_times
  hipEvent_t kt_ev[KT_RING][2] = {};
  hipEvent_t gate[2] = {nullptr, nullptr};         // the event the next planning of slot s waits for
  hipEvent_t ev_plan = nullptr;
  // validation status words, one per picture, ping-pong: a picture reports into d_status[pic_par]
  // and its first stripe zeroes the other word for the next picture
  DevBuf<unsigned long long> d_status;
  int pic_par = 0;
  unsigned long long* last_status = nullptr;  // word of the last device-planned picture
  int prep_poc = 0, prep_n = 0;
  bool prepared = false;
  bool status_pending = false;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  std::map<int, RefHost> orgs;  // original luma pictures for mm_sad_window
  DevBuf<MeBlockDev> d_me_blocks;
  // MM-DMVR of the device-planned picture (mm_set_dmvr / mm_pred_dmvr): its buffers are the plan
  // slot's (PlanSlot::dmvr_*); the search runs on the context stream
  bool dmvr = false;
  // MM-MVP: the device copy of the epipole list (refreshed when its version moves, staged through a
  // pinned buffer on the context stream), the host-buffer API's query / result buffers and the
  // deferred status word (sticky until mm_mvp_status reads it)
  // Two device tables alternate per list version: a refresh writes the table the current version
  // does not use, after the conversions that read it (two versions back) have completed on the MVP
  // stream (ev_epi_done), so a refresh never rewrites a table an in-flight conversion reads.
  DevBuf<mmmvp::EpiDev> d_epi[2];
  int epi_buf = 0;                                   // table of the current version
  bool epi_used[2] = {false, false};                 // ev_epi_done[b] recorded
  hipEvent_t ev_epi_done[2] = {nullptr, nullptr};    // MVP-stream conversions reading table b are done
  mmmvp::EpiDev* h_epi = nullptr;
  size_t h_epi_cap = 0;
  hipEvent_t ev_epi = nullptr;
  unsigned long long epi_version = ~0ull;
  int epi_n = 0;
  hipStream_t mvp_stream = nullptr;  // mm_set_mvp_stream; mvp_on_own = false: the context stream
  bool mvp_on_own = false;
  bool epi_fresh = false;  // an epipole-table copy on the context stream the MVP stream has not waited for
  DevBuf<mm_mvp_query> d_mvp_q;
  DevBuf<int32_t> d_mvp_out;
  DevBuf<unsigned long long> d_mvp_status;  // sticky: every conversion since the last mm_mvp_status
  DevBuf<unsigned> d_mvp_bins;  // 2 x MVP_COUNTERS key counters (alternating sorted calls)
  int mvp_sort_par = 0;
  DevBuf<int> d_mvp_local, d_mvp_perm;
  bool mvp_pending = false;
  DevBuf<int> d_me_off, d_me_chunk;
  bool stage_timing = false;
  // mm_set_call_timing: ev0 / ev1 around every picture call (on by default); `timed`: the last
  // launch sequence recorded them
  bool call_timing = true;
  bool timed = false;
  hipEvent_t ev_stage[3] = {nullptr, nullptr, nullptr};  // after planning, setup, reprojection
  hipEvent_t ev_mem = nullptr;  // dev_alloc / dev_free fences between the context's streams
};

static hipStream_t mvp_stream_of(const mm_ctx* c) { return c->mvp_on_own ? c->mvp_stream : c->stream; }

// `to` waits for the work queued so far on `from` (GPU-side; a null handle is the null stream, which
// the context stream may be)
static void order_after(mm_ctx* c, hipStream_t to, hipStream_t from) {
  if (from == to) return;
  if (!c->ev_mem && hipEventCreateWithFlags(&c->ev_mem, hipEventDisableTiming) != hipSuccess) {
    (void)hipStreamSynchronize(from);  // no event: drain `from` instead (this context's stream only)
    return;
  }
  if (hipEventRecord(c->ev_mem, from) != hipSuccess || hipStreamWaitEvent(to, c->ev_mem, 0) != hipSuccess)
    (void)hipStreamSynchronize(from);
}

// A buffer from the stream-ordered pool, usable by work queued after this call on every stream of
// the context (the auxiliary and MVP streams wait for the allocation's point on the context stream).
static hipError_t dev_alloc(mm_ctx* c, void** p, size_t bytes) {
  const hipError_t e = hipMallocAsync(p, bytes, c->stream);
  if (e != hipSuccess) return e;
  order_after(c, c->aux, c->stream);
  if (c->mvp_on_own) order_after(c, c->mvp_stream, c->stream);
  return hipSuccess;
}

// Frees a pool buffer once every piece of work queued so far on the context's streams has run: the
// context stream waits for the auxiliary and MVP streams, then frees in its own order.
static void dev_free(mm_ctx* c, void* p) {
  order_after(c, c->stream, c->aux);
  if (c->mvp_on_own) order_after(c, c->stream, c->mvp_stream);
  (void)hipFreeAsync(p, c->stream);
}

static int read_status(mm_ctx* c, int* first_bad);


static int fail(mm_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}
#define HIPCHK(ctx, x)                                                                                    \
  do {                                                                                                    \
    hipError_t e_ = (x);                                                                                  \
    if (e_ != hipSuccess) return fail(ctx, MM_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)
#define RCCHK(x)         \
  do {                   \
    int rc_ = (x);       \
    if (rc_) return rc_; \
  } while (0)

template <typename T>
static int upload(mm_ctx* c, DevBuf<T>& d, const std::vector<T>& h) {
  HIPCHK(c, d.ensure(c, h.size()));
  if (!h.empty()) HIPCHK(c, hipMemcpyAsync(d.p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice, c->stream));
  return MM_OK;
}

static MpaCache make_cache(mm_ctx* c) {
  MpaCache mc{};
  mc.px = c->mpa_px;
  mc.py = c->mpa_py;
  mc.vip = c->mpa_vip;
  mc.cols = c->geo.W / 4;
  mc.rows = c->geo.H / 4;
  mc.trig_col = c->trig;
  mc.tan_grid = c->tan_grid;
  mc.trig_row = c->trig ? c->trig + 4 * mc.cols : nullptr;
  return mc;
}

static int upload_jobs(mm_ctx* c) {
  RCCHK(upload(c, c->d_jobs, c->plan.jobs));
  RCCHK(upload(c, c->d_job_off, c->plan.job_off));
  RCCHK(upload(c, c->d_job_chunk, c->plan.job_chunk));
  RCCHK(upload(c, c->d_ged, c->plan.ged));
  HIPCHK(c, c->d_setup.ensure(c, c->plan.jobs.size()));
  HIPCHK(c, c->d_reproj.ensure(c, 2 * (size_t)c->plan.n_elems));
  return MM_OK;
}

static int run_reproj_kernels(mm_ctx* c) {
  const int n_jobs = (int)c->plan.jobs.size(), n_elems = c->plan.n_elems;
  if (n_jobs == 0 || n_elems == 0) return MM_OK;
  hipLaunchKernelGGL(k_setup, dim3((n_jobs + 255) / 256), dim3(256), 0, c->stream, c->sc, c->d_jobs.p, n_jobs,
                     c->d_ged.p, c->d_setup.p);
  hipLaunchKernelGGL(k_reproj, dim3((n_elems + 255) / 256), dim3(256), 0, c->stream, c->sc, c->d_jobs.p, n_jobs,
                     c->d_job_off.p, c->d_job_chunk.p, n_elems, c->d_setup.p, make_cache(c), c->d_reproj.p);
  HIPCHK(c, hipGetLastError());
  return MM_OK;
}

extern "C" {

int mm_get_version(void) { return MM_VERSION; }

int mm_derive_effective_blocks(const mm_tool_flags* tools, const mm_pu_motion* pus, int n, const mm_pu_desc* sub,
                               mm_pu_desc* out_mc, int cap_mc, int* n_mc, mm_pu_desc* out_dmvr, int cap_dmvr,
                               int* n_dmvr) {
  if (!tools || n < 0 || (n > 0 && !pus) || !n_mc || !n_dmvr) return MM_ERR_ARG;
  std::vector<mm_pu_desc> mc, dmvr;
  mmeff::Deriver d(*tools, &mc, &dmvr);
  for (int i = 0; i < n; i++) {
    const int rc = d.run(pus[i], sub);
    if (rc) return rc;
  }
  *n_mc = (int)mc.size();
  *n_dmvr = (int)dmvr.size();
  if ((int)mc.size() > cap_mc || (int)dmvr.size() > cap_dmvr || (!mc.empty() && !out_mc) ||
      (!dmvr.empty() && !out_dmvr))
    return MM_ERR_ARG;
  std::copy(mc.begin(), mc.end(), out_mc);
  std::copy(dmvr.begin(), dmvr.end(), out_dmvr);
  return MM_OK;
}

const char* mm_last_error(mm_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int mm_create(const mm_seq_params* p, int device, mm_ctx** out_ctx) {
  if (!p || !out_ctx) return MM_ERR_ARG;
  *out_ctx = nullptr;
  if (p->width <= 0 || p->height <= 0 || (p->width & 7) || (p->height & 7)) return MM_ERR_ARG;
  if (p->width > 16384 || p->height > 16384) return MM_ERR_ARG;  // 16-bit positions in the plan records
  if (p->chroma_format != 0 && p->chroma_format != 1) return MM_ERR_ARG;
  if (p->bit_depth < 8 || p->bit_depth > 12) return MM_ERR_ARG;
  if (p->mm_offset4x4 < 0 || p->mm_offset4x4 > 4) return MM_ERR_ARG;
  if (p->max_cu_width < 8 || p->max_cu_height < 8) return MM_ERR_ARG;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return MM_ERR_NODEV;
  if (device < 0 || device >= ndev) return MM_ERR_ARG;
  if (hipSetDevice(device) != hipSuccess) return MM_ERR_HIP;
  mm_ctx* c = new mm_ctx();
  c->prm = *p;
  c->device = device;
  c->sc = seq_const(*p);
  c->geo.W = p->width;
  c->geo.H = p->height;
  c->geo.chroma = p->chroma_format == 1;
  c->geo.Wc = p->width >> 1;
  c->geo.Hc = p->height >> 1;
  c->geo.maxCUw = p->max_cu_width;
  c->geo.maxCUh = p->max_cu_height;
  c->geo.maxCUwc = p->max_cu_width >> 1;
  c->geo.maxCUhc = p->max_cu_height >> 1;
  c->geo.bd = p->bit_depth;
  c->geo.vec_store = 0;
  c->geo.hp = 0;
  c->geo.store = 3;
  c->geo.padded = 1;
  // Every event the library records is a device-scope release: it orders work between the
  // context and auxiliary streams and times it, and never publishes device memory to the host
  // (status words and results reach the host through copies).  The default system-scope release
  // writes back the L2 after each picture's 57 MB of output: ~5 us per event, ~17 us per picture
  // with the three events a call records (profiles/r03_ab_event_scope.txt).
  constexpr unsigned TIMED = hipEventReleaseToDevice, SYNC = hipEventDisableTiming | hipEventReleaseToDevice;
  // the plan-ahead slot gates order the next planning after a k_mc_dev (a write-after-read on the
  // slot's records) and publish nothing, so they skip the release: with one, the gate's completion
  // writes k_mc_dev's dirty output lines back from every XCD's L2 before either queue moves on
  constexpr unsigned GATE = GATE_NO_FENCE ? hipEventDisableTiming | hipEventDisableSystemFence : SYNC;
  if (hipEventCreateWithFlags(&c->ev0, TIMED) != hipSuccess || hipEventCreateWithFlags(&c->ev1, TIMED) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_stage[0], TIMED) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_stage[1], TIMED) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_stage[2], TIMED) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_fork, SYNC) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_join, SYNC) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_gate[0], GATE) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_gate[1], GATE) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_plan, SYNC) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_epi, SYNC) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_epi_done[0], SYNC) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_epi_done[1], SYNC) != hipSuccess ||
      hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking) != hipSuccess ||
      hipEventRecord(c->ev_gate[0], c->stream) != hipSuccess || hipEventRecord(c->ev_gate[1], c->stream) != hipSuccess) {
    mm_destroy(c);
    return MM_ERR_HIP;
  }
  c->gate[0] = c->ev_gate[0];
  c->gate[1] = c->ev_gate[1];
  // MPA frame caches (MVReprojection::init -> MotionPlaneAdaptiveMotionModel::fillCache)
  const int cols = p->width / 4, rows = p->height / 4, n = cols * rows;
  const unsigned mpa_bits = p->active_models & (7u << MPA_FRONT_BACK);
  if (mpa_bits && (dev_alloc(c, reinterpret_cast<void**>(&c->mpa_px), 3 * (size_t)n * sizeof(float)) != hipSuccess ||
                   dev_alloc(c, reinterpret_cast<void**>(&c->mpa_py), 3 * (size_t)n * sizeof(float)) != hipSuccess ||
                   dev_alloc(c, reinterpret_cast<void**>(&c->mpa_vip), 3 * (size_t)n) != hipSuccess)) {
    mm_destroy(c);
    return MM_ERR_HIP;
  }
  for (int pl = 0; pl < 3; pl++) {
    if (!(p->active_models & (1u << (MPA_FRONT_BACK + pl)))) continue;
    hipLaunchKernelGGL(k_mpa_cache, dim3((n + 255) / 256), dim3(256), 0, c->stream, c->sc, MPA_FRONT_BACK + pl, cols,
                       rows, c->mpa_px + (size_t)pl * n, c->mpa_py + (size_t)pl * n, c->mpa_vip + (size_t)pl * n);
  }
  // separable toSphere table (MpaCache::trig_col / trig_row): 2 flavours x (cols + rows) pairs
  if (dev_alloc(c, reinterpret_cast<void**>(&c->trig), (size_t)4 * (cols + rows) * sizeof(float)) != hipSuccess) {
    mm_destroy(c);
    return MM_ERR_HIP;
  }
  hipLaunchKernelGGL(k_erp_trig, dim3((2 * (cols + rows) + 255) / 256), dim3(256), 0, c->stream, c->sc, cols, rows,
                     c->trig, c->trig + 4 * cols);
  // TAN's first step per grid point and flavour, 2 x 16 B x (W/4 x H/4) (37.7 MB at 6144x3072): it
  // depends on the grid point only, so TAN elements load it instead of computing sqrt + acosf +
  // atan2f + a sin/cos pair each (profiles/r03_ab_tan_grid.txt)
  if (p->active_models & (1u << TANGENTIAL)) {
    const long nt = 2L * cols * rows;
    if (dev_alloc(c, reinterpret_cast<void**>(&c->tan_grid), (size_t)nt * sizeof(TanEntry)) != hipSuccess) {
      mm_destroy(c);
      return MM_ERR_HIP;
    }
    MpaCache tc = make_cache(c);
    tc.tan_grid = nullptr;
    hipLaunchKernelGGL(k_tan_grid, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, c->stream, c->sc, tc, c->tan_grid);
  }
  if (c->d_status.ensure(c, 2) != hipSuccess || hipMemsetAsync(c->d_status.p, 0, 2 * sizeof(unsigned long long), c->stream) != hipSuccess ||
      c->d_mvp_status.ensure(c, 1) != hipSuccess ||
      hipMemsetAsync(c->d_mvp_status.p, 0, sizeof(unsigned long long), c->stream) != hipSuccess ||
      c->d_mvp_bins.ensure(c, 2 * MVP_COUNTERS) != hipSuccess ||
      hipMemsetAsync(c->d_mvp_bins.p, 0, 2 * MVP_COUNTERS * sizeof(unsigned), c->stream) != hipSuccess ||
      hipGetLastError() != hipSuccess || hipStreamSynchronize(c->stream) != hipSuccess) {
    mm_destroy(c);
    return MM_ERR_HIP;
  }
  *out_ctx = c;
  return MM_OK;
}

int mm_destroy(mm_ctx* c) {
  if (!c) return MM_ERR_ARG;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  if (c->aux) (void)hipStreamSynchronize(c->aux);
  if (c->mvp_on_own) (void)hipStreamSynchronize(c->mvp_stream);
  for (void* q : {(void*)c->pool, (void*)c->chroma_stage, (void*)c->trig, (void*)c->tan_grid, (void*)c->mpa_px,
                  (void*)c->mpa_py, (void*)c->mpa_vip})
    if (q) dev_free(c, q);
  c->d_jobs.release(c);
  c->d_job_off.release(c);
  c->d_job_chunk.release(c);
  c->d_pu_off.release(c);
  c->d_pu_chunk.release(c);
  c->d_setup.release(c);
  c->d_reproj.release(c);
  c->d_pu_in.release(c);
  c->d_status.release(c);
  for (int k = 0; k < 2; k++) c->slot[k].release(c);
  c->d_ged.release(c);
  for (auto& kv : c->orgs)
    if (kv.second.y) dev_free(c, kv.second.y);
  c->d_me_blocks.release(c);
  c->d_mvp_q.release(c);
  c->d_mvp_out.release(c);
  c->d_mvp_status.release(c);
  c->d_mvp_bins.release(c);
  c->d_mvp_local.release(c);
  c->d_mvp_perm.release(c);
  for (int b = 0; b < 2; b++) {
    c->d_epi[b].release(c);
    if (c->ev_epi_done[b]) (void)hipEventDestroy(c->ev_epi_done[b]);
  }
  if (c->h_epi) (void)hipHostFree(c->h_epi);
  if (c->ev_epi) (void)hipEventDestroy(c->ev_epi);
  c->d_me_off.release(c);
  c->d_me_chunk.release(c);
  for (auto& e : c->ev_stage)
    if (e) (void)hipEventDestroy(e);
  (void)hipStreamSynchronize(c->stream);  // the pool frees above
  if (c->ev_mem) (void)hipEventDestroy(c->ev_mem);
  if (c->aux) (void)hipStreamDestroy(c->aux);
  if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
  if (c->ev_join) (void)hipEventDestroy(c->ev_join);
  for (auto& e : c->ev_gate)
    if (e) (void)hipEventDestroy(e);
  for (auto& pr : c->kt_ev)
    for (auto& e : pr)
      if (e) (void)hipEventDestroy(e);
  if (c->ev_plan) (void)hipEventDestroy(c->ev_plan);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  delete c;
  return MM_OK;
}

int mm_set_stream(mm_ctx* c, void* s) {
  if (!c) return MM_ERR_ARG;
  // work queued on the old stream may still use the context's buffers, which are freed and fenced in
  // the context stream's order from now on
  (void)hipStreamSynchronize(c->stream);
  c->stream = (hipStream_t)s;
  return MM_OK;
}

static int read_mvp_status(mm_ctx* c, int* first_bad);
int mm_synchronize(mm_ctx* c) {
  if (!c) return MM_ERR_ARG;
  const int rc = read_status(c, nullptr);
  const int rm = read_mvp_status(c, nullptr);
  return rc ? rc : rm;
}

int mm_set_epipole(mm_ctx* c, int cur, int ref, const int32_t q24[3]) {
  if (!c || !q24) return MM_ERR_ARG;
  c->epipoles.add({q24[0], q24[1], q24[2]}, cur, ref, true);  // DecLib.cpp:2048, 3141: available
  return MM_OK;
}

// ---- EpipoleList (mm_epipole.h) ------------------------------------------------------------
mm_epipole_list* mm_epipole_list_create(void) { return new mm_epipole_list{new mmepi::EpipoleList(), true}; }

void mm_epipole_list_destroy(mm_epipole_list* e) {
  if (!e || !e->owned) return;  // a context's list lives and dies with the context
  delete e->l;
  delete e;
}

mm_epipole_list* mm_get_epipole_list(mm_ctx* c) { return c ? &c->epi_handle : nullptr; }

int mm_epipole_add(mm_epipole_list* e, int cur, int ref, const int32_t q24[3], int make_available) {
  if (!e || !q24) return MM_ERR_ARG;
  e->l->add({q24[0], q24[1], q24[2]}, cur, ref, make_available != 0);
  return MM_OK;
}

int mm_epipole_make_available(mm_epipole_list* e, int cur) {
  if (!e) return MM_ERR_ARG;
  e->l->make_available(cur);
  return MM_OK;
}

int mm_epipole_has(mm_epipole_list* e, int cur, int ref) { return e && e->l->has(cur, ref) ? 1 : 0; }

int mm_epipole_find(mm_epipole_list* e, int cur, int ref, int32_t q24[3]) {
  if (!e || !q24) return MM_ERR_ARG;
  mmepi::Q3 q;
  if (!e->l->find(cur, ref, &q)) return MM_ERR_NOEPIPOLE;
  for (int i = 0; i < 3; i++) q24[i] = q[i];
  return MM_OK;
}

int mm_epipole_derive_predictor(mm_epipole_list* e, int cur, int32_t q24[3]) {
  if (!e || !q24) return MM_ERR_ARG;
  mmepi::Q3 q;
  const int rc = e->l->derive_predictor(cur, &q);
  if (rc) return rc;
  for (int i = 0; i < 3; i++) q24[i] = q[i];
  return MM_OK;
}

int mm_epipole_count(mm_epipole_list* e) { return e ? e->l->count() : -1; }

// Reference picture layout in the pool: each plane carries edge-replicated margins (the role of
// VTM's extendPicBorder, Picture.cpp:988-1048) wide enough for every window k_mc reads from an
// in-range sub-block (sb_out_of_range admits positions up to maxCU outside the picture; the
// 8-tap luma window reaches 4 samples beyond, the 4-tap chroma one 2), so k_mc never clamps.
// Margins are 64 samples aligned so plane origins stay 128-byte aligned; +8 samples spare.
// The chroma plane is interleaved: one dword Cb | Cr << 16 per position (chroma_layout's stride
// counts positions, its bytes are those of the two planes), so one window row segment of k_mc's
// chroma filter serves both components (mm_filter.h predict_chroma_pool_il).
struct PlaneLayout {
  int mx, my, stride;  // margin columns / rows, row stride (samples)
  size_t bytes;        // whole padded plane
};
static PlaneLayout plane_layout(int w, int h, int max_cu_w, int max_cu_h, int reach_x, int reach_y) {
  PlaneLayout l;
  l.mx = (max_cu_w + reach_x + 8 + 63) & ~63;
  l.my = max_cu_h + reach_y + 8;
  l.stride = (w + 2 * l.mx + 63) & ~63;
  l.bytes = (size_t)2 * l.stride * (h + 2 * l.my);
  return l;
}
static PlaneLayout luma_layout(const mm_ctx* c) {
  return plane_layout(c->geo.W, c->geo.H, c->geo.maxCUw, c->geo.maxCUh, 4, 3);
}
static PlaneLayout chroma_layout(const mm_ctx* c) {
  PlaneLayout l = plane_layout(c->geo.Wc, c->geo.Hc, c->geo.maxCUwc, c->geo.maxCUhc, 2, 1);
  l.bytes *= 2;  // interleaved Cb | Cr dwords
  return l;
}

static void place_ref(mm_ctx* c, RefHost& r) {
  const PlaneLayout ly = luma_layout(c), lc = chroma_layout(c);
  r.stride_y = ly.stride;
  r.stride_c = lc.stride;
  char* base = c->pool + (size_t)r.slot * c->pic_bytes;
  r.y = reinterpret_cast<int16_t*>(base + 2 * ((size_t)ly.my * ly.stride + ly.mx));
  // cb: position (0, 0) of the interleaved chroma plane (Cb | Cr << 16 dwords); no separate Cr plane
  r.cb = c->geo.chroma ? reinterpret_cast<int16_t*>(base + ly.bytes + 4 * ((size_t)lc.my * lc.stride + lc.mx)) : nullptr;
  r.cr = nullptr;
}

// Fills a plane's margins from its nearest edge sample (corners from the corner sample), one
// 4-sample (8-byte) chunk per thread: the top/bottom bands over the full padded width, then the
// left/right bands.  Chunks never straddle the picture edge (w, mx multiples of 4).
__global__ void __launch_bounds__(256) k_pad_plane(int16_t* __restrict__ o, int stride, int w, int h, int mx, int my) {
  typedef uint32_t u2 __attribute__((ext_vector_type(2)));
  const int fq = (w + 2 * mx) >> 2, sq = (2 * mx) >> 2;  // chunks per band row
  long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long tb = (long)2 * my * fq;
  int x, y;
  if (t < tb) {
    const int r = (int)(t / fq);
    x = 4 * (int)(t - (long)r * fq) - mx;
    y = r < my ? r - my : h + r - my;
  } else {
    t -= tb;
    if (t >= (long)h * sq) return;
    y = (int)(t / sq);
    const int k = 4 * (int)(t - (long)y * sq);
    x = k < mx ? k - mx : w + k - mx;
  }
  const int16_t* src = o + (long)(y < 0 ? 0 : (y >= h ? h - 1 : y)) * stride;
  u2 v;
  if (x >= 0 && x < w) {
    v = *reinterpret_cast<const u2*>(src + x);
  } else {
    const uint32_t e = (uint16_t)src[x < 0 ? 0 : w - 1];
    v.x = v.y = e | (e << 16);
  }
  *reinterpret_cast<u2*>(o + (long)y * stride + x) = v;
}

// The interleaved chroma plane with its margins from the two source planes, one 4-position (16-byte)
// chunk per thread over the whole padded plane: position (x, y) holds Cb | Cr << 16 of the source
// sample at (x, y) clamped to the picture -- what pad_plane's edge replication gives each plane.
__global__ void __launch_bounds__(256) k_pad_chroma_il(uint32_t* __restrict__ o, int stride, int w, int h, int mx,
                                                       int my, const int16_t* __restrict__ cb,
                                                       const int16_t* __restrict__ cr, long src_stride) {
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  const int fq = (w + 2 * mx) >> 2;  // chunks per padded row
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)fq * (h + 2 * my)) return;
  const int r = (int)(t / fq);
  const int x = 4 * (int)(t - (long)r * fq) - mx, y = r - my;
  const long sy = (long)(y < 0 ? 0 : (y >= h ? h - 1 : y)) * src_stride;
  uint32_t v[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int sx = x + k < 0 ? 0 : (x + k >= w ? w - 1 : x + k);
    v[k] = (uint32_t)(uint16_t)cb[sy + sx] | ((uint32_t)(uint16_t)cr[sy + sx] << 16);
  }
  *reinterpret_cast<u4*>(o + (long)y * stride + x) = u4{v[0], v[1], v[2], v[3]};
}

static int pad_chroma_il(mm_ctx* c, int16_t* origin, const int16_t* cb, const int16_t* cr, long src_stride) {
  const PlaneLayout l = chroma_layout(c);
  const int w = c->geo.Wc, h = c->geo.Hc;
  const long n = (long)((w + 2 * l.mx) >> 2) * (h + 2 * l.my);
  hipLaunchKernelGGL(k_pad_chroma_il, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream,
                     reinterpret_cast<uint32_t*>(origin), l.stride, w, h, l.mx, l.my, cb, cr, src_stride);
  HIPCHK(c, hipGetLastError());
  return MM_OK;
}

static int pad_plane(mm_ctx* c, int16_t* origin, const PlaneLayout& l, int w, int h) {
  const long n = (long)2 * l.my * ((w + 2 * l.mx) >> 2) + (long)h * ((2 * l.mx) >> 2);
  hipLaunchKernelGGL(k_pad_plane, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream, origin, l.stride, w, h,
                     l.mx, l.my);
  HIPCHK(c, hipGetLastError());
  return MM_OK;
}

}  // extern "C" (the packing kernels below are templates)

// ---- C4 transport: stripe-packed pictures (mm_pack_samples, mm_upload_ref_packed) -------------
// The stripe-major picture of mm360/parallel.py StripeLayout, K = 32 / bd samples per dword
// (mm360.h).  Packing reads the rank's int16 segment once; unpacking fills a pool slot's padded
// planes position by position from the clamped source sample -- the interior and the margins in one
// pass each (k_pad_plane's and k_pad_chroma_il's edge replication), so the gathered picture is
// never materialised as int16 planes.
constexpr int MAX_STRIPES = 64;
struct StripePack {
  int W, H, world, rows;  // rows: luma rows per segment (the largest stripe)
  int K, bd;
  long seg, seg_dw;  // int16 samples / packed dwords per segment
  int y0[MAX_STRIPES + 1];  // first luma row of stripe r; y0[world] = H
};
// StripeLayout's stripes: CTU rows split evenly, r gets [n_ctu r / world, n_ctu (r + 1) / world)
static StripePack stripe_pack(const mm_ctx* c, int world, int ctu) {
  StripePack s{};
  s.W = c->geo.W;
  s.H = c->geo.H;
  s.world = world;
  s.bd = c->geo.bd;
  s.K = 32 / s.bd;
  const int n_ctu = (s.H + ctu - 1) / ctu;
  for (int r = 0; r <= world; r++) s.y0[r] = std::min(s.H, (n_ctu * r / world) * ctu);
  for (int r = 0; r < world; r++) s.rows = std::max(s.rows, s.y0[r + 1] - s.y0[r]);
  s.seg = (long)s.rows * s.W + 2L * (s.rows / 2) * (s.W / 2);
  s.seg_dw = (s.seg + s.K - 1) / s.K;
  return s;
}

__global__ void __launch_bounds__(256) k_pack_samples(const uint16_t* __restrict__ src, long n,
                                                      uint32_t* __restrict__ dst, int K, int bd) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;  // one output dword
  const long i0 = t * K;
  if (i0 >= n) return;
  const uint32_t mask = (1u << bd) - 1u;
  uint32_t w = 0;
  for (int k = 0; k < K; k++)
    if (i0 + k < n) w |= ((uint32_t)src[i0 + k] & mask) << (k * bd);
  dst[t] = w;
}

// sample j of segment r of the packed picture (32-bit indices: a segment holds < 2^31 samples; K a
// compile-time constant, so j / K is a multiply-high, not a 64-bit division)
// K == 1: the int16 stripe-major picture itself (mm_upload_ref_stripes)
template <int K>
__device__ __forceinline__ uint32_t packed_sample(const uint32_t* __restrict__ p, const StripePack& s, int r, int j) {
  if constexpr (K == 1) {
    return (uint32_t)reinterpret_cast<const uint16_t*>(p)[(long)r * s.seg + j];
  } else {
    const int q = j / K;
    return (p[(long)r * s.seg_dw + q] >> ((j - q * K) * s.bd)) & ((1u << s.bd) - 1u);
  }
}
// Samples j0 .. j0 + 3 of segment r (one run inside a plane row): with K >= 3 they lie in two
// consecutive dwords, so an interior chunk takes two loads and one division instead of four each
template <int K>
__device__ __forceinline__ void packed_run4(const uint32_t* __restrict__ p, const StripePack& s, int r, int j0,
                                            uint32_t* v) {
  if constexpr (K < 3) {
#pragma unroll
    for (int k = 0; k < 4; k++) v[k] = packed_sample<K>(p, s, r, j0 + k);
  } else {
    const int q = j0 / K, o = j0 - q * K;
    const uint32_t* w = p + (long)r * s.seg_dw + q;
    const uint32_t d0 = w[0];
    const uint32_t d1 = o + 3 >= K ? w[1] : 0u;  // dword q + 1 only when sample j0 + 3 lies in it
    const uint32_t mask = (1u << s.bd) - 1u;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int t = o + k;  // 0 .. 2K - 1
      v[k] = ((t < K ? d0 : d1) >> ((t < K ? t : t - K) * s.bd)) & mask;
    }
  }
}

// the stripe holding luma row y (uniform loop over the table)
__device__ __forceinline__ int stripe_of(const StripePack& s, int y) {
  int r = 0;
  for (int k = 1; k < s.world; k++) r += y >= s.y0[k] ? 1 : 0;
  return r;
}

// One 4-sample chunk of the padded luma plane per thread: (x, y) over [-mx, W + mx) x [-my, H + my)
template <int K>
__global__ void __launch_bounds__(256) k_unpack_luma(int16_t* __restrict__ o, int stride, int mx, int my,
                                                     const uint32_t* __restrict__ p, StripePack s) {
  typedef uint32_t u2 __attribute__((ext_vector_type(2)));
  const int fq = (s.W + 2 * mx) >> 2;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= fq * (s.H + 2 * my)) return;
  const int row = t / fq;
  const int x = 4 * (t - row * fq) - mx, y = row - my;
  const int yc = y < 0 ? 0 : (y >= s.H ? s.H - 1 : y);
  const int r = stripe_of(s, yc);
  const int base = (yc - s.y0[r]) * s.W;
  uint32_t v[4];
  if (x >= 0 && x + 3 < s.W) {
    packed_run4<K>(p, s, r, base + x, v);
  } else {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int xc = x + k < 0 ? 0 : (x + k >= s.W ? s.W - 1 : x + k);
      v[k] = packed_sample<K>(p, s, r, base + xc);
    }
  }
  *reinterpret_cast<u2*>(o + (long)y * stride + x) = u2{v[0] | (v[1] << 16), v[2] | (v[3] << 16)};
}

// One 4-position chunk of the padded interleaved chroma plane (Cb | Cr << 16) per thread
template <int K>
__global__ void __launch_bounds__(256) k_unpack_chroma_il(uint32_t* __restrict__ o, int stride, int mx, int my,
                                                          const uint32_t* __restrict__ p, StripePack s) {
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  const int w = s.W / 2, h = s.H / 2;
  const int fq = (w + 2 * mx) >> 2;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= fq * (h + 2 * my)) return;
  const int row = t / fq;
  const int x = 4 * (t - row * fq) - mx, y = row - my;
  const int yc = y < 0 ? 0 : (y >= h ? h - 1 : y);
  const int r = stripe_of(s, 2 * yc);  // chroma rows [y0 / 2, y1 / 2) of stripe r (y0 even)
  const int luma = s.rows * s.W, chroma = (s.rows / 2) * w;
  const int base = luma + (yc - s.y0[r] / 2) * w;
  uint32_t v[4];
  if (x >= 0 && x + 3 < w) {
    uint32_t b[4], c[4];
    packed_run4<K>(p, s, r, base + x, b);
    packed_run4<K>(p, s, r, base + chroma + x, c);
#pragma unroll
    for (int k = 0; k < 4; k++) v[k] = b[k] | (c[k] << 16);
  } else {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int xc = x + k < 0 ? 0 : (x + k >= w ? w - 1 : x + k);
      v[k] = packed_sample<K>(p, s, r, base + xc) | (packed_sample<K>(p, s, r, base + chroma + xc) << 16);
    }
  }
  *reinterpret_cast<u4*>(o + (long)y * stride + x) = u4{v[0], v[1], v[2], v[3]};
}

extern "C" {

// A free picture slot of the reference pool; grows the pool (copying the resident pictures) when
// full.  The copy and the old allocation's release are ordered behind the context's queued work on
// its own streams (dev_free), so no launch still reads the old allocation and nothing waits on the
// host.
static int take_pool_slot(mm_ctx* c, int* slot) {
  if (!c->pic_bytes) c->pic_bytes = luma_layout(c).bytes + (c->geo.chroma ? chroma_layout(c).bytes : 0);
  if (c->pool_free.empty()) {
    const size_t limit = ((size_t)1 << 31) - 1;
    const int max_cap = (int)std::min<size_t>(limit / c->pic_bytes, 64);
    if (c->pool_cap >= max_cap)
      return fail(c, MM_ERR_ARG, "reference pool full (" + std::to_string(c->pool_cap) + " pictures, < 2 GiB)");
    const int cap = std::min(max_cap, std::max(4, 2 * c->pool_cap));
    char* np = nullptr;
    HIPCHK(c, dev_alloc(c, reinterpret_cast<void**>(&np), (size_t)cap * c->pic_bytes));
    if (c->pool) {
      order_after(c, c->stream, c->aux);
      HIPCHK(c, hipMemcpyAsync(np, c->pool, (size_t)c->pool_cap * c->pic_bytes, hipMemcpyDeviceToDevice, c->stream));
      dev_free(c, c->pool);
    }
    c->pool = np;
    for (int k = cap - 1; k >= c->pool_cap; k--) c->pool_free.push_back(k);
    c->pool_cap = cap;
    for (auto& kv : c->refs) place_ref(c, kv.second);
  }
  *slot = c->pool_free.back();
  c->pool_free.pop_back();
  return MM_OK;
}

static RefPool pool_of(const mm_ctx* c) {
  const PlaneLayout ly = luma_layout(c), lc = chroma_layout(c);
  RefPool p{};
  p.base = c->pool;
  p.bytes = (uint32_t)((size_t)c->pool_cap * c->pic_bytes);
  p.pic_bytes = (uint32_t)c->pic_bytes;
  p.y0 = (uint32_t)(2 * ((size_t)ly.my * ly.stride + ly.mx));
  p.cb0 = c->geo.chroma ? (uint32_t)(ly.bytes + 4 * ((size_t)lc.my * lc.stride + lc.mx)) : 0u;
  p.stride_y = ly.stride;
  p.stride_c = lc.stride;
  return p;
}

// A picture's tables for the device: the pool and, per table slot, its pool slot (packed bytes;
// stage_ref_table rebuilds the RefDev offsets from them), checked against the host offsets.
static int device_tables(mm_ctx* c, PicTables* t) {
  t->pool = pool_of(c);
  for (int k = 0; k < MAX_SLOTS / 4; k++) t->pool_slot4[k] = 0u;
  for (int s = 0; s < t->n_slots; s++) {
    const RefDev& r = t->ref[s];
    const uint32_t ps = (r.off_y - t->pool.y0) / t->pool.pic_bytes;
    if (ps > 255u || ps * t->pool.pic_bytes + t->pool.y0 != r.off_y ||
        (c->geo.chroma && ps * t->pool.pic_bytes + t->pool.cb0 != r.off_cb) || r.stride_y != t->pool.stride_y ||
        (c->geo.chroma && r.stride_c != t->pool.stride_c))
      return fail(c, MM_ERR_HIP, "reference outside the pool layout");
    t->pool_slot4[s >> 2] |= ps << (8 * (s & 3));
  }
  return MM_OK;
}

// Reference slots of a picture: every resident reference, POC order, with its pool offsets
static std::vector<std::pair<int, RefDev>> ref_slots(const mm_ctx* c) {
  std::vector<std::pair<int, RefDev>> refs;
  for (auto& kv : c->refs) {
    const RefHost& h = kv.second;
    const uint32_t oy = (uint32_t)((const char*)h.y - c->pool);
    const uint32_t oc = h.cb ? (uint32_t)((const char*)h.cb - c->pool) : 0u;
    refs.emplace_back(kv.first, RefDev{h.y, h.cb, h.cr, h.stride_y, h.stride_c, oy, oc});
  }
  return refs;
}

int mm_upload_ref(mm_ctx* c, int poc, const int16_t* y, ptrdiff_t sy, const int16_t* cb, const int16_t* cr,
                  ptrdiff_t sc_, int src_dev) {
  if (!c || !y) return MM_ERR_ARG;
  if (c->geo.chroma && (!cb || !cr)) return fail(c, MM_ERR_ARG, "chroma planes required for 4:2:0");
  HIPCHK(c, hipSetDevice(c->device));
  if (!c->refs.count(poc)) {
    int slot = -1;
    RCCHK(take_pool_slot(c, &slot));
    RefHost& r = c->refs[poc];
    r.slot = slot;
    place_ref(c, r);
  }
  RefHost& r = c->refs[poc];
  const int W = c->geo.W, H = c->geo.H, Wc = c->geo.Wc, Hc = c->geo.Hc;
  hipMemcpyKind k = src_dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
  HIPCHK(c, hipMemcpy2DAsync(r.y, r.stride_y * 2, y, sy * 2, W * 2, H, k, c->stream));
  RCCHK(pad_plane(c, r.y, luma_layout(c), W, H));
  if (c->geo.chroma) {
    // device sources are interleaved straight from their planes; host ones through a device copy
    const int16_t *scb = cb, *scr = cr;
    long ss = (long)sc_;
    if (!src_dev) {
      if (!c->chroma_stage) HIPCHK(c, dev_alloc(c, reinterpret_cast<void**>(&c->chroma_stage), (size_t)4 * Wc * Hc));
      int16_t* st = c->chroma_stage;
      HIPCHK(c, hipMemcpy2DAsync(st, Wc * 2, cb, sc_ * 2, Wc * 2, Hc, k, c->stream));
      HIPCHK(c, hipMemcpy2DAsync(st + (size_t)Wc * Hc, Wc * 2, cr, sc_ * 2, Wc * 2, Hc, k, c->stream));
      scb = st;
      scr = st + (size_t)Wc * Hc;
      ss = Wc;
    }
    RCCHK(pad_chroma_il(c, r.cb, scb, scr, ss));
  }
  if (!src_dev) HIPCHK(c, hipStreamSynchronize(c->stream));  // host source buffers may be reused at once
  return MM_OK;
}

int mm_release_ref(mm_ctx* c, int poc) {
  if (!c) return MM_ERR_ARG;
  auto it = c->refs.find(poc);
  if (it == c->refs.end()) return fail(c, MM_ERR_NOREF, "reference POC not uploaded");
  c->pool_free.push_back(it->second.slot);  // stream-ordered: later uploads into the slot follow
  c->refs.erase(it);                        // every launch already queued on the context stream
  return MM_OK;
}

int64_t mm_stripe_packed_dwords(mm_ctx* c, int world, int ctu) {
  if (!c || world < 1 || world > MAX_STRIPES || ctu < 8 || (ctu & 7)) return -1;
  return stripe_pack(c, world, ctu).seg_dw;
}

int mm_pack_samples(mm_ctx* c, const int16_t* d_src, int64_t n, uint32_t* d_dst) {
  if (!c || n < 0 || (n > 0 && (!d_src || !d_dst))) return MM_ERR_ARG;
  if (n == 0) return MM_OK;
  HIPCHK(c, hipSetDevice(c->device));
  const int K = 32 / c->geo.bd;
  const long nd = (long)((n + K - 1) / K);
  hipLaunchKernelGGL(k_pack_samples, dim3((unsigned)((nd + 255) / 256)), dim3(256), 0, c->stream,
                     reinterpret_cast<const uint16_t*>(d_src), (long)n, d_dst, K, c->geo.bd);
  HIPCHK(c, hipGetLastError());
  return MM_OK;
}

// k: the samples per word of the source (1: the int16 stripe-major picture, mm_upload_ref_stripes)
static int upload_ref_stripes(mm_ctx* c, int poc, const uint32_t* d_packed, int world, int ctu, bool int16) {
  if (!c || !d_packed || world < 1 || world > MAX_STRIPES || ctu < 8 || (ctu & 7)) return MM_ERR_ARG;
  if (!c->geo.chroma) return fail(c, MM_ERR_ARG, "the stripe-packed picture is 4:2:0");
  HIPCHK(c, hipSetDevice(c->device));
  if (!c->refs.count(poc)) {
    int slot = -1;
    RCCHK(take_pool_slot(c, &slot));
    RefHost& r = c->refs[poc];
    r.slot = slot;
    place_ref(c, r);
  }
  const RefHost& r = c->refs[poc];
  StripePack s = stripe_pack(c, world, ctu);
  if (int16) s.K = 1;
  const PlaneLayout ly = luma_layout(c), lc = chroma_layout(c);
  const long nl = (long)((s.W + 2 * ly.mx) >> 2) * (s.H + 2 * ly.my);
  const long nc = (long)((s.W / 2 + 2 * lc.mx) >> 2) * (s.H / 2 + 2 * lc.my);
  auto launch = [&](auto kl, auto kc) {
    hipLaunchKernelGGL(kl, dim3((unsigned)((nl + 255) / 256)), dim3(256), 0, c->stream, r.y, ly.stride, ly.mx, ly.my,
                       d_packed, s);
    hipLaunchKernelGGL(kc, dim3((unsigned)((nc + 255) / 256)), dim3(256), 0, c->stream,
                       reinterpret_cast<uint32_t*>(r.cb), lc.stride, lc.mx, lc.my, d_packed, s);
  };
  if (s.K == 1)
    launch(k_unpack_luma<1>, k_unpack_chroma_il<1>);
  else if (s.K == 4)
    launch(k_unpack_luma<4>, k_unpack_chroma_il<4>);
  else if (s.K == 3)
    launch(k_unpack_luma<3>, k_unpack_chroma_il<3>);
  else
    launch(k_unpack_luma<2>, k_unpack_chroma_il<2>);
  HIPCHK(c, hipGetLastError());
  return MM_OK;
}
int mm_upload_ref_packed(mm_ctx* c, int poc, const uint32_t* d_packed, int world, int ctu) {
  return upload_ref_stripes(c, poc, d_packed, world, ctu, false);
}
int mm_upload_ref_stripes(mm_ctx* c, int poc, const int16_t* d_stripes, int world, int ctu) {
  return upload_ref_stripes(c, poc, reinterpret_cast<const uint32_t*>(d_stripes), world, ctu, true);
}

int mm_reproject(mm_ctx* c, const mm_block_desc* blocks, int n, int32_t* out_xy) {
  if (!c || n < 0 || (n > 0 && (!blocks || !out_xy))) return MM_ERR_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  Planner pl(seq_info(c->prm), c->epipoles, &c->plan);
  int rc = pl.plan_blocks(blocks, n);
  if (rc) return fail(c, rc, c->plan.err);
  if (c->plan.n_elems == 0) return MM_OK;
  RCCHK(upload_jobs(c));
  RCCHK(run_reproj_kernels(c));
  HIPCHK(c, hipMemcpyAsync(out_xy, c->d_reproj.p, (size_t)c->plan.n_elems * 2 * sizeof(int32_t), hipMemcpyDeviceToHost,
                           c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return MM_OK;
}

// ---- device-planned prediction ----------------------------------------------------------

static int round_grid(long v) { return (int)((v + 8 * XCD_RUN - 1) / (8 * XCD_RUN) * (8 * XCD_RUN)); }

// Buffers for a stripe of n PUs: a PU list predicts each luma sample of the picture at most
// once, so sub-blocks are bounded by the picture's sub-block count (and by n * 1024, 128x128
// PUs); a PU has at most 4 jobs and 4 reprojection elements per luma sub-block (2 lists x
// {luma, chroma}).  k_plan_place refuses a list beyond these capacities (overlapping PUs).
// With MM-DMVR a PU is placed as up to 64 sub-PUs (128x128 / 16x16); a sub-PU covers at least 128
// luma samples (PU::checkDMVRCondition), so the picture bounds them by W * H / 128, and their cost
// elements (N_OFF per luma sub-block) by N_OFF times the picture's sub-blocks.
// fits (dry run): set to false when any buffer would have to grow; nothing is allocated or changed.
// slot_fits is this dry run, so a call whose capacities (the DMVR-derived ones included) exceed any
// buffer takes the synchronised growth branch of launch_pictures (round-5 advisor: a small DMVR call,
// a larger plain one and a medium DMVR one used to pass the old n / pics / dmvr test and grow the
// jobs and DMVR buffers unsynchronised).
static int ensure_slot_buffers(mm_ctx* c, PlanSlot& S, int n, bool dmvr, int pics = 1, bool* fits = nullptr) {
  PlanCaps k;
  pics = std::max(pics, S.pics_ensured);  // (buffers only grow)
  const long area_sb = (long)(c->geo.W / 4) * (c->geo.H / 4) * pics;  // each picture predicts each sample once
  const int subs = dmvr ? (int)std::min<long>((long)n * 64, (long)c->geo.W * c->geo.H / 128 * pics) : 0;
  k.pus = n + subs;
  k.jobs = 4 * k.pus;
  k.sb = (int)std::min<long>((long)n * 1024, area_sb);
  k.elems = 4 * k.sb;
  k.subs = subs;
  k.dmvr_elems = dmvr ? (int)std::min<long>((long)N_OFF * area_sb, (long)subs * N_OFF * 16) : 0;
  if (fits) *fits = true;
  // grow (or, dry run, check) one buffer; fresh: it was (re)allocated
  auto need = [&](auto& b, size_t want, bool* fresh = nullptr) -> hipError_t {
    if (fresh) *fresh = false;
    if (fits) {
      if (!b.p || want > b.cap) *fits = false;
      return hipSuccess;
    }
    return b.ensure(c, want, fresh);
  };
  if (dmvr) {
    HIPCHK(c, need(S.dmvr_sub, k.subs));
    HIPCHK(c, need(S.dmvr_off, k.subs));
    HIPCHK(c, need(S.dmvr_chunk, (size_t)k.dmvr_elems / 64 + 1));
    // per slot, sized by the sub-PUs: centre setups and centre terms (2 x (56 + 44) B), delta, centre
    // cost, survivor index -- about 220 B per sub-PU (32 MB at 6144x3072; the other offsets' setups,
    // positions and costs of the survivors live in the search kernel's registers and LDS)
    HIPCHK(c, need(S.dmvr_setup, (size_t)k.subs * 2));
    HIPCHK(c, need(S.dmvr_cterms, (size_t)k.subs * 2));
    HIPCHK(c, need(S.dmvr_mvd, 2 * (size_t)k.subs));
    HIPCHK(c, need(S.dmvr_count, 1));
    HIPCHK(c, need(S.dmvr_ccost, k.subs));
    HIPCHK(c, need(S.dmvr_surv_s, k.subs));
  }
  bool fresh_jobs = false;
  HIPCHK(c, need(S.jobs, k.jobs, &fresh_jobs));
  if (fresh_jobs) HIPCHK(c, hipMemsetAsync(S.jobs.p, 0, S.jobs.cap * sizeof(JobDev), c->stream));
  HIPCHK(c, need(S.job_off, k.jobs));
  HIPCHK(c, need(S.job_chunk, k.elems / 64 + 1));
  HIPCHK(c, need(S.setup, k.jobs));
  HIPCHK(c, need(S.meta, 1));
  HIPCHK(c, need(S.blk, (size_t)((n + PLAN_BLOCK - 1) / PLAN_BLOCK) * N_KEYS));
  HIPCHK(c, need(S.blkq, (size_t)((n + PLACE_BLOCK - 1) / PLACE_BLOCK) * N_KEYS));
  // The records k_reproj/k_mc exchange are zeroed once when allocated: every record a plan
  // counts is written before it is read (classify_pu decides counts and emission alike), and a
  // record that never was written still holds in-picture values (position 0, slot 0), never
  // uninitialised memory that k_mc would use as a destination offset.
  bool fresh = false;
  HIPCHK(c, need(S.mc_meta, k.sb, &fresh));
  if (fresh) HIPCHK(c, hipMemsetAsync(S.mc_meta.p, 0, S.mc_meta.cap * sizeof(mm_int2), c->stream));
  for (int l = 0; l < 2; l++) {
    HIPCHK(c, need(S.mc_lpos[l], k.sb, &fresh));
    if (fresh) HIPCHK(c, hipMemsetAsync(S.mc_lpos[l].p, 0, S.mc_lpos[l].cap * sizeof(uint32_t), c->stream));
    HIPCHK(c, need(S.mc_cpos[l], k.sb, &fresh));
    if (fresh) HIPCHK(c, hipMemsetAsync(S.mc_cpos[l].p, 0, S.mc_cpos[l].cap * sizeof(uint32_t), c->stream));
    for (int q = 0; q < 2; q++) {  // touched only by the sub-blocks whose positions are far
      HIPCHK(c, need(S.mc_far[l][q], k.sb, &fresh));
      if (fresh) HIPCHK(c, hipMemsetAsync(S.mc_far[l][q].p, 0, S.mc_far[l][q].cap * sizeof(mm_int2), c->stream));
    }
  }
  if (fits) return MM_OK;
  S.caps = k;
  if (dmvr) S.dmvr_ensured = true;
  S.n_ensured = std::max(S.n_ensured, n);
  S.pics_ensured = pics;
  return MM_OK;
}
static bool slot_fits(mm_ctx* c, PlanSlot& S, int n, bool dmvr, int pics = 1) {
  bool fits = false;
  return ensure_slot_buffers(c, S, n, dmvr, pics, &fits) == MM_OK && fits;
}

// One stripe (PUs [base, base + n) of the picture's list) through k_plan_count + k_plan_place +
// k_setup_dev + k_reproj_dev + k_mc_dev on `st`.  Stage events only in single-stripe timing mode.
// status: the picture's status word; next_status (first stripe only): the word to zero for the
// next picture.
static int launch_stripe(mm_ctx* c, PlanSlot& S, hipStream_t st, const PicTables& t, const Geometry& geo,
                         const PuSegs& d_in, int n, int base, unsigned long long* status,
                         unsigned long long* next_status, const DstPlanes& dst, bool plan_ahead = false,
                         bool want_mvd = false, hipEvent_t mc_done = nullptr, hipEvent_t* gate_out = nullptr) {
  // plan-ahead: `st` is the auxiliary stream for the planning kernels; the rest runs on the
  // context stream (which may be the null stream, so a flag, not a null handle, says so)
  hipStream_t st_back = c->stream;
  bool back = plan_ahead;
  const PlanCaps& k = S.caps;
  const int gp = (n + PLAN_BLOCK - 1) / PLAN_BLOCK;
  const int gs = (k.jobs + 255) / 256;
  const int gr = round_grid((k.elems + 255) / 256);
  const int gm = 8 * std::max(1, (((k.sb + 7) / 8 + 255) / 256 + MC_BLOCKS_PER_WG - 1) / MC_BLOCKS_PER_WG);
  const int gq = (n + PLACE_BLOCK - 1) / PLACE_BLOCK;
  hipLaunchKernelGGL(k_plan_count, dim3(gp), dim3(PLAN_BLOCK), 0, st, d_in, n, base, t, status, S.blk.p, S.blkq.p, gq);
  const DmvrRecs dm{S.dmvr_sub.p, S.dmvr_off.p, S.dmvr_chunk.p};
  hipLaunchKernelGGL(k_plan_place, dim3(gq), dim3(PLACE_BLOCK), 0, st, d_in, n, t, status, next_status, S.blk.p, gp,
                     S.blkq.p, S.meta.p, k, S.jobs.p, S.job_off.p, S.job_chunk.p, dm);
  if (c->stage_timing) HIPCHK(c, hipEventRecord(c->ev_stage[0], st));
  if (t.dmvr) {
    // MM-DMVR reads the reference pictures: from here on the context stream (plan-ahead gates only
    // the PU list, not the references)
    if (back) {
      HIPCHK(c, hipEventRecord(c->ev_plan, st));
      HIPCHK(c, hipStreamWaitEvent(st_back, c->ev_plan, 0));
      st = st_back;
      back = false;
    }
    const int gd = (int)std::min<long>(DMVR_GRID, ((long)k.subs * 2 + 255) / 256 + 1);
    const DmvrWork dw{S.dmvr_count.p, S.dmvr_ccost.p, S.dmvr_surv_s.p, S.dmvr_cterms.p};
    int32_t* mvd = want_mvd ? S.dmvr_mvd.p : nullptr;
    hipLaunchKernelGGL(k_dmvr_setup_dev, dim3(gd), dim3(256), 0, st, c->sc, S.meta.p, S.dmvr_sub.p, t, S.dmvr_setup.p,
                       S.dmvr_cterms.p, dw.count);
    const int gcen = (int)std::min<long>(DMVR_GRID, ((long)k.subs * 32 + 255) / 256);
    hipLaunchKernelGGL(k_dmvr_centre_dev, dim3(std::max(1, gcen)), dim3(256), 0, st, c->sc, geo, S.meta.p, S.dmvr_sub.p,
                       S.dmvr_setup.p, make_cache(c), t, dw, S.jobs.p, mvd);
    hipLaunchKernelGGL(k_dmvr_search_dev, dim3(std::max(1, std::min(DMVR_SEARCH_GRID, (k.subs + DMVR_WAVES - 1) / DMVR_WAVES))), dim3(DMVR_SEARCH_WG),
                       0, st, c->sc, geo, S.dmvr_sub.p, make_cache(c), t, dw, S.jobs.p, mvd);
  }
  McRec mc;
  mc.meta = S.mc_meta.p;
  for (int l = 0; l < 2; l++) {
    mc.lpos[l] = S.mc_lpos[l].p;
    mc.cpos[l] = S.mc_cpos[l].p;
    for (int q = 0; q < 2; q++) mc.far[l][q] = S.mc_far[l][q].p;
  }
  // reprojection ahead (plan-ahead, no MM-DMVR): k_reproj_dev also runs on the auxiliary stream, so
  // it overlaps the previous picture's k_mc_dev -- VALU-bound reprojection beside the texture-path-
  // bound interpolation.  Its McRec writes go to this call's plan slot, whose previous reader (the
  // k_mc_dev of two calls back) the slot gate already orders before the planning.
  const bool reproj_ahead = back && MM_REPROJ_AHEAD;
  // the setups and the reprojection; `stop`: an event bound to the kernel's completion
  // (hipExtLaunchKernelGGL), or null.  (Building the setups inside the reprojection kernel -- each
  // workgroup its run of jobs into LDS -- measured 0.191 vs 0.172-0.174 ms per picture:
  // profiles/r05_ab_overlap.txt.)
  auto setup = [&](hipStream_t s_, hipEvent_t stop) {
    hipExtLaunchKernelGGL(k_setup_dev, dim3(gs), dim3(256), 0, s_, nullptr, stop, 0, c->sc, S.meta.p, S.jobs.p, t,
                          S.setup.p);
  };
  auto reproj = [&](hipStream_t s_, hipEvent_t stop) {
    hipExtLaunchKernelGGL(k_reproj_dev, dim3(gr), dim3(256), MM_REPROJ_LDS, s_, nullptr, stop, 0, c->sc, S.meta.p, S.jobs.p,
                          S.job_off.p, S.job_chunk.p, S.setup.p, make_cache(c), mc);
  };
  if (back) {
    // plan-ahead: ev_plan completes with the last kernel of this picture on `aux` (the reprojection
    // ahead, or the setups), bound to its dispatch when KERNEL_EVENTS
    hipEvent_t stop = KERNEL_EVENTS ? c->ev_plan : nullptr;
    if (reproj_ahead) {
      setup(st, nullptr);
      reproj(st, stop);
    } else {
      setup(st, stop);
    }
    if (!stop) HIPCHK(c, hipEventRecord(c->ev_plan, st));
    // Round 3 had the host wait for this picture's planning before it issued the context stream's
    // wait, so that the runtime put no cross-queue barrier packet between two pictures' kernels (C3
    // 0.178-0.180 -> 0.173-0.175 ms, profiles/r03_ab_hostsync.txt, when ev_plan completed with the
    // short k_setup_dev).  With the reprojection ahead, ev_plan completes with k_reproj_dev, which runs
    // as long as the previous picture's k_mc_dev: the wait put the host's wake-up (~20 us in the
    // kernel trace) between k_reproj_dev and k_mc_dev and kept the next call's planning from being
    // issued.  Without it: 0.1712-0.1727 vs 0.1724-0.1750 ms per picture (profiles/r05_ab_overlap.txt).
    if (PLAN_AHEAD_HOST_WAIT) HIPCHK(c, hipEventSynchronize(c->ev_plan));
    HIPCHK(c, hipStreamWaitEvent(st_back, c->ev_plan, 0));
    st = st_back;
  } else {
    setup(st, nullptr);
  }
  if (c->stage_timing) HIPCHK(c, hipEventRecord(c->ev_stage[1], st));
  if (!reproj_ahead) reproj(st, nullptr);
  if (c->stage_timing) HIPCHK(c, hipEventRecord(c->ev_stage[2], st));
  // mc_done (plan-ahead): the slot's gate, complete when this k_mc is; *gate_out = the event the
  // slot's next planning waits for (mc_done, or the kernel-timing stop event bound to this k_mc)
  hipEvent_t start = nullptr, stop = KERNEL_EVENTS ? mc_done : nullptr;
  if (c->kt_on) {
    hipEvent_t* pr = c->kt_ev[c->kt_n % mm_ctx::KT_RING];
    start = pr[0];
    stop = pr[1];
    c->kt_n++;
  }
  if (geo.hp)
    hipExtLaunchKernelGGL(k_mc_dev<true>, dim3(gm), dim3(256), MM_MC_LDS, st, start, stop, 0, geo, S.meta.p, mc, t, dst);
  else
    hipExtLaunchKernelGGL(k_mc_dev<false>, dim3(gm), dim3(256), MM_MC_LDS, st, start, stop, 0, geo, S.meta.p, mc, t, dst);
  if (mc_done && (c->kt_on || !KERNEL_EVENTS)) {
    if (c->kt_on && gate_out)
      *gate_out = stop;  // bound to this k_mc_dev: no marker packet in the timed loop
    else
      HIPCHK(c, hipEventRecord(mc_done, st));
  } else if (gate_out) {
    *gate_out = mc_done;
  }
  HIPCHK(c, hipGetLastError());
  return MM_OK;
}

// One picture, bracketed by ev0/ev1 on the context stream.  The PU list (raster CTU order) is cut
// into n_stripes contiguous stripes; even stripes run on the context stream with slot 0, odd ones
// on the auxiliary stream with slot 1, so one stripe's latency-bound planning kernels overlap the
// other's interpolation.  PUs write disjoint samples, so stripes are independent; the auxiliary
// stream forks from and joins back into the context stream.  Validation errors of every stripe
// go to the picture's status word and are reported by mm_pred_status.
// only_list / hp / store: mm_pred_list (-1 / 0 / 3 for the normal prediction).
// dmvr: MM_PUF_DMVR PUs allowed (the context's mm_set_dmvr, or mm_pred_dmvr); want_mvd: keep the
// refined delta of every DMVR sub-PU, in placement order, in the slot's dmvr_mvd.
// status_base: added to the PU index a validation failure reports (a run of a split multi-picture call)
static int launch_pictures(mm_ctx* c, const mm_pic_job* pics, int n_pics, int only_list = -1, int hp = 0,
                           int store = 3, bool may_plan_ahead = false, bool dmvr = false, bool want_mvd = false,
                           int status_base = 0) {
  std::vector<std::pair<int, RefDev>> refs;
  refs = ref_slots(c);
  PicTables t;
  std::string err;
  int cur[MAX_PICS];
  for (int q = 0; q < n_pics; q++) cur[q] = pics[q].cur_poc;
  int rc = build_pic_tables(seq_info(c->prm), c->epipoles, cur, n_pics, refs, &t, &err);
  if (rc) return fail(c, rc, err);
  RCCHK(device_tables(c, &t));
  t.only_list = only_list;
  t.dmvr = dmvr ? 1 : 0;
  Geometry geo = c->geo;
  geo.hp = hp;
  geo.store = store;
  // destinations of the pictures (unused entries repeat picture 0's, so every pointer is valid)
  DstPlanes dst{};
  int n = 0;
  geo.vec_store = 1;
  for (int q = 0; q < MAX_PICS; q++) {
    const mm_pic_job& p = pics[q < n_pics ? q : 0];
    dst.y[q] = p.dst_y;
    dst.cb[q] = p.dst_cb;
    dst.cr[q] = p.dst_cr;
    dst.sy[q] = (int)p.dst_stride_y;
    dst.sc[q] = (int)p.dst_stride_c;
    if (q < n_pics) {
      n += p.n;
      const bool vy = !p.dst_y || ((uintptr_t)p.dst_y % 8 == 0 && p.dst_stride_y % 4 == 0);
      const bool vc = !geo.chroma || !p.dst_cb ||
                      ((uintptr_t)p.dst_cb % 4 == 0 && (uintptr_t)p.dst_cr % 4 == 0 && p.dst_stride_c % 2 == 0);
      if (!(vy && vc)) geo.vec_store = 0;
    }
  }
  // one stripe under stage timing, with DMVR (its setup / cost buffers are per plan slot, one picture's) and for
  // several pictures
  const int K = (c->stage_timing || dmvr || n_pics > 1)
                    ? 1
                    : std::max(1, std::min(c->n_stripes, (n + PLAN_BLOCK - 1) / PLAN_BLOCK));
  const int per = (n + K - 1) / K;
  // PU lists of stripe s of a single picture, or of every picture
  auto segs_of = [&](int base, int m) {
    PuSegs g{};
    g.n_pics = K > 1 ? 1 : n_pics;
    int acc = 0;
    for (int q = 0; q < MAX_PICS; q++) {
      const mm_pic_job& p = pics[q < g.n_pics ? q : 0];
      g.p[q] = K > 1 ? p.d_pus + base : p.d_pus;
      g.base[q] = acc;
      if (q < g.n_pics) acc += K > 1 ? m : p.n;
    }
    g.base[MAX_PICS] = acc;
    return g;
  };
  unsigned long long* status = c->d_status.p + c->pic_par;
  unsigned long long* next_status = c->d_status.p + (c->pic_par ^ 1);
  if (may_plan_ahead && c->plan_ahead && K == 1 && !c->stage_timing) {
    // Plan-ahead: planning + setup of this picture on `aux`, gated only by the k_mc_dev of the
    // slot's previous user (two calls back), so they overlap the previous picture's kernels.
    if (!slot_fits(c, c->slot[0], per, dmvr, n_pics) || !slot_fits(c, c->slot[1], per, dmvr, n_pics)) {
      // growing frees buffers the other stream may still use, and zeroes on the context stream
      HIPCHK(c, hipStreamSynchronize(c->aux));
      HIPCHK(c, hipStreamSynchronize(c->stream));
      for (int s = 0; s < 2; s++) RCCHK(ensure_slot_buffers(c, c->slot[s], per, dmvr, n_pics));
      HIPCHK(c, hipStreamSynchronize(c->stream));
    } else {
      for (int s = 0; s < 2; s++) RCCHK(ensure_slot_buffers(c, c->slot[s], per, dmvr, n_pics));  // caps only
    }
    // the slot's previous user (two calls back) has finished its k_mc_dev
    HIPCHK(c, hipStreamWaitEvent(c->aux, c->gate[c->ahead_par], 0));
    c->timed = c->call_timing;
    if (c->timed) HIPCHK(c, hipEventRecord(c->ev0, c->stream));
    RCCHK(launch_stripe(c, c->slot[c->ahead_par], c->aux, t, geo, segs_of(0, n), n, status_base, status, next_status, dst, true,
                        want_mvd, c->ev_gate[c->ahead_par], &c->gate[c->ahead_par]));
    c->last_slot = c->ahead_par;
    c->ahead_par ^= 1;
    if (c->timed) HIPCHK(c, hipEventRecord(c->ev1, c->stream));
    c->last_status = status;
    c->pic_par ^= 1;
    c->status_pending = true;
    return MM_OK;
  }
  for (int s = 0; s < std::min(K, 2); s++) {
    // growth of buffers a plan-ahead call on the auxiliary stream may still use
    if (!slot_fits(c, c->slot[s], per, dmvr, n_pics)) HIPCHK(c, hipStreamSynchronize(c->aux));
    RCCHK(ensure_slot_buffers(c, c->slot[s], per, dmvr, n_pics));
  }
  // each event a call records costs the context stream ~4 us (profiles/r03_ab_event_scope.txt)
  c->timed = c->call_timing || c->stage_timing;
  if (c->timed) HIPCHK(c, hipEventRecord(c->ev0, c->stream));
  c->last_slot = 0;
  if (K > 1) {
    HIPCHK(c, hipEventRecord(c->ev_fork, c->stream));
    HIPCHK(c, hipStreamWaitEvent(c->aux, c->ev_fork, 0));
  }
  for (int s = 0; s < K; s++) {
    const int base = s * per, m = std::min(per, n - base);
    if (m <= 0) break;
    RCCHK(launch_stripe(c, c->slot[s & 1], (s & 1) ? c->aux : c->stream, t, geo, segs_of(base, m), m, status_base + base, status,
                        s == 0 ? next_status : nullptr, dst, false, want_mvd));
  }
  if (K > 1) {
    HIPCHK(c, hipEventRecord(c->ev_join, c->aux));
    HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_join, 0));
  }
  if (c->timed) HIPCHK(c, hipEventRecord(c->ev1, c->stream));
  // a following plan-ahead call starts its planning only after this whole call (both slots used);
  // while plan-ahead is off, mm_set_plan_ahead records the gates when it is switched on
  if (c->plan_ahead) {  // both slots may have been used by this call's stripes
    HIPCHK(c, hipEventRecord(c->ev_gate[0], c->stream));
    HIPCHK(c, hipEventRecord(c->ev_gate[1], c->stream));
    c->gate[0] = c->ev_gate[0];
    c->gate[1] = c->ev_gate[1];
  }
  c->last_status = status;
  c->pic_par ^= 1;
  c->status_pending = true;
  return MM_OK;
}
// one picture
static int launch_device_plan(mm_ctx* c, int cur_poc, const mm_pu_desc* d_in, int n, int16_t* dy, ptrdiff_t sdy,
                              int16_t* dcb, int16_t* dcr, ptrdiff_t sdc, int only_list = -1, int hp = 0,
                              int store = 3, bool may_plan_ahead = false, bool dmvr = false,
                              bool want_mvd = false) {
  const mm_pic_job p{cur_poc, d_in, n, dy, sdy, dcb, dcr, sdc};
  return launch_pictures(c, &p, 1, only_list, hp, store, may_plan_ahead, dmvr, want_mvd);
}

int mm_set_plan_ahead(mm_ctx* c, int on) {
  if (!c) return MM_ERR_ARG;
  if (on && !c->plan_ahead) {  // calls made while it was off recorded no gate: gate on the current position
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipEventRecord(c->ev_gate[0], c->stream));
    HIPCHK(c, hipEventRecord(c->ev_gate[1], c->stream));
    c->gate[0] = c->ev_gate[0];
    c->gate[1] = c->ev_gate[1];
  }
  c->plan_ahead = on != 0;
  return MM_OK;
}

int mm_set_call_timing(mm_ctx* c, int on) {
  if (!c) return MM_ERR_ARG;
  c->call_timing = on != 0;
  return MM_OK;
}

int mm_set_stripes(mm_ctx* c, int stripes) {
  if (!c || stripes < 1 || stripes > 64) return MM_ERR_ARG;
  c->n_stripes = stripes;
  return MM_OK;
}

// Synchronise and decode the deferred validation status of the last device-planned call.
static int decode_status(mm_ctx* c, unsigned long long w, int* first_bad, const char* item);
static int read_status(mm_ctx* c, int* first_bad) {
  if (first_bad) *first_bad = -1;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (!c->status_pending) return MM_OK;
  c->status_pending = false;
  unsigned long long w = 0;
  HIPCHK(c, hipMemcpy(&w, c->last_status, sizeof(w), hipMemcpyDeviceToHost));
  return decode_status(c, w, first_bad, "PU");
}
static int decode_status(mm_ctx* c, unsigned long long w, int* first_bad, const char* item) {
  if (!w) return MM_OK;
  const unsigned long long v = ~w;
  const int code = (int)(v & 0xff), pu = (int)(v >> 8);
  if (first_bad) *first_bad = pu;
  static const char* what[] = {"ok", "PU outside the picture, not 4x4 aligned, using no (or not the requested) list, "
                                     "invalid BCW index, or the list covers more than the picture",
                               "HIP error", "reference POC not uploaded", "no epipole for (curPOC, refPOC)",
                               "invalid, CLASSIC or inactive motion model", "no device"};
  return fail(c, code, std::string(item) + " " + std::to_string(pu) + ": " + (code >= 0 && code <= 6 ? what[code] : "error"));
}

int mm_pred_device(mm_ctx* c, int cur_poc, const mm_pu_desc* d_pus, int n, int16_t* dy, ptrdiff_t sdy, int16_t* dcb,
                   int16_t* dcr, ptrdiff_t sdc) {
  if (!c || n < 0 || (n > 0 && !d_pus) || !dy || (c->geo.chroma && (!dcb || !dcr))) return MM_ERR_ARG;
  if (n == 0) return MM_OK;
  HIPCHK(c, hipSetDevice(c->device));
  return launch_device_plan(c, cur_poc, d_pus, n, dy, sdy, dcb, dcr, sdc, -1, 0, 3, true, c->dmvr);
}

int mm_pred_device_multi(mm_ctx* c, const mm_pic_job* pics, int n_pics) {
  if (!c || n_pics < 1 || n_pics > MAX_PICS || !pics) return MM_ERR_ARG;
  long n = 0;
  for (int q = 0; q < n_pics; q++) {
    const mm_pic_job& p = pics[q];
    if (p.n < 0 || (p.n > 0 && !p.d_pus) || !p.dst_y || (c->geo.chroma && (!p.dst_cb || !p.dst_cr))) return MM_ERR_ARG;
    n += p.n;
  }
  if (n > INT32_MAX / 2) return MM_ERR_ARG;
  if (n == 0) return MM_OK;
  HIPCHK(c, hipSetDevice(c->device));
  // One launch chain holds MAX_SLOTS distinct camera-pose epipoles (PicTables::ged): pictures whose
  // (cur, ref) epipoles together exceed that are cut into consecutive runs, each its own chain
  // (round-5 advisor: four RA leaves with five distinct references each used to fail the call).
  const auto refs = ref_slots(c);
  int cur[MAX_PICS];
  for (int q = 0; q < n_pics; q++) cur[q] = pics[q].cur_poc;
  // A run's deferred status word is overwritten by the next run's planning, so every run but the last
  // is checked before the next one is issued (host synchronisation only on this rare path).
  int pu_base = 0;
  for (int q0 = 0; q0 < n_pics;) {
    int q1 = q0 + 1;
    while (q1 < n_pics && count_cam_epipoles(c->epipoles, cur + q0, q1 + 1 - q0, refs) <= MAX_SLOTS) q1++;
    RCCHK(launch_pictures(c, pics + q0, q1 - q0, -1, 0, 3, true, c->dmvr, false, pu_base));
    if (q1 < n_pics) RCCHK(read_status(c, nullptr));
    for (int q = q0; q < q1; q++) pu_base += pics[q].n;
    q0 = q1;
  }
  return MM_OK;
}

int mm_set_dmvr(mm_ctx* c, int on) {
  if (!c) return MM_ERR_ARG;
  c->dmvr = on != 0;
  return MM_OK;
}

int mm_pred_status(mm_ctx* c, int* first_bad_pu) {
  if (!c) return MM_ERR_ARG;
  return read_status(c, first_bad_pu);
}

int mm_pred_prepare(mm_ctx* c, int cur_poc, const mm_pu_desc* pus, int n) {
  if (!c || n < 0 || (n > 0 && !pus)) return MM_ERR_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  c->prepared = false;
  HIPCHK(c, c->d_pu_in.ensure(c, n));
  if (n) HIPCHK(c, hipMemcpyAsync(c->d_pu_in.p, pus, (size_t)n * sizeof(mm_pu_desc), hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->prep_poc = cur_poc;
  c->prep_n = n;
  c->prepared = true;
  return MM_OK;
}

int mm_pred_run(mm_ctx* c, int16_t* dy, ptrdiff_t sdy, int16_t* dcb, int16_t* dcr, ptrdiff_t sdc) {
  if (!c || !dy || (c->geo.chroma && (!dcb || !dcr))) return MM_ERR_ARG;
  if (!c->prepared) return fail(c, MM_ERR_ARG, "mm_pred_run without a valid mm_pred_prepare");
  return mm_pred_device(c, c->prep_poc, c->d_pu_in.p, c->prep_n, dy, sdy, dcb, dcr, sdc);
}

int mm_pred(mm_ctx* c, int cur_poc, const mm_pu_desc* pus, int n, int16_t* dy, ptrdiff_t sdy, int16_t* dcb,
            int16_t* dcr, ptrdiff_t sdc) {
  RCCHK(mm_pred_prepare(c, cur_poc, pus, n));
  RCCHK(mm_pred_run(c, dy, sdy, dcb, dcr, sdc));
  return read_status(c, nullptr);
}

int mm_pred_list(mm_ctx* c, int cur_poc, const mm_pu_desc* pus, int n, int list, int hp, int16_t* dy, ptrdiff_t sdy,
                 int16_t* dcb, int16_t* dcr, ptrdiff_t sdc) {
  if (!c || n < 0 || (n > 0 && !pus) || (list != 0 && list != 1) || (hp != 0 && hp != 1)) return MM_ERR_ARG;
  const bool want_c = c->geo.chroma && dcb && dcr;
  if (!dy && !want_c) return MM_ERR_ARG;
  if ((dcb == nullptr) != (dcr == nullptr)) return MM_ERR_ARG;
  if (n == 0) return MM_OK;
  RCCHK(mm_pred_prepare(c, cur_poc, pus, n));
  c->prepared = false;  // the buffer now holds this list call's PUs, not a prepared picture
  RCCHK(launch_device_plan(c, cur_poc, c->d_pu_in.p, n, dy, sdy, dcb, dcr, sdc, list, hp,
                           (dy ? 1 : 0) | (want_c ? 2 : 0)));
  return read_status(c, nullptr);
}

int mm_last_timing(mm_ctx* c, float* ms) {
  if (!c || !ms) return MM_ERR_ARG;
  if (!c->timed) return fail(c, MM_ERR_ARG, "the last launch sequence was not timed (mm_set_call_timing)");
  HIPCHK(c, hipEventSynchronize(c->ev1));
  HIPCHK(c, hipEventElapsedTime(ms, c->ev0, c->ev1));
  return MM_OK;
}

int mm_upload_org(mm_ctx* c, int poc, const int16_t* y, ptrdiff_t sy, int src_dev) {
  if (!c || !y) return MM_ERR_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  RefHost& r = c->orgs[poc];
  if (!r.y) {
    r.stride_y = (c->geo.W + 63) & ~63;
    HIPCHK(c, dev_alloc(c, reinterpret_cast<void**>(&r.y), (size_t)r.stride_y * c->geo.H * sizeof(int16_t)));
  }
  HIPCHK(c, hipMemcpy2DAsync(r.y, r.stride_y * 2, y, sy * 2, c->geo.W * 2, c->geo.H,
                             src_dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return MM_OK;
}

// The candidates of every block (window or pattern, mm_me.h MeWindow) -> sads[n][w.C] on the device
static int me_run(mm_ctx* c, int cur_poc, const mm_me_block* blocks, int n, const MeWindow& w, uint32_t* sads) {
  HIPCHK(c, hipSetDevice(c->device));
  auto oit = c->orgs.find(cur_poc);
  if (oit == c->orgs.end()) return fail(c, MM_ERR_ARG, "no original picture uploaded for the current POC");
  std::vector<std::pair<int, RefDev>> refs;
  refs = ref_slots(c);
  PicTables t;
  std::string err;
  int rc = build_pic_tables(seq_info(c->prm), c->epipoles, cur_poc, refs, &t, &err);
  if (rc) return fail(c, rc, err);
  RCCHK(device_tables(c, &t));
  std::vector<MeBatch> batches;
  rc = plan_me_window(seq_info(c->prm), t, blocks, n, w, &batches, &err, false);
  if (rc) return fail(c, rc, err);
  c->timed = true;
  HIPCHK(c, hipEventRecord(c->ev0, c->stream));
  HIPCHK(c, hipMemsetAsync(sads, 0, (size_t)n * w.C * sizeof(uint32_t), c->stream));
  for (const MeBatch& bt : batches) {
    RCCHK(upload(c, c->d_me_blocks, bt.blocks));
    RCCHK(upload(c, c->d_me_off, bt.blk_off));
    const long n_chunks = (bt.n_elems + 63) / 64;
    HIPCHK(c, c->d_me_chunk.ensure(c, (size_t)std::max<long>(n_chunks, 1)));
    hipLaunchKernelGGL(k_me_chunks, dim3((unsigned)((n_chunks + 255) / 256)), dim3(256), 0, c->stream, c->d_me_off.p,
                       (int)bt.blocks.size(), bt.n_elems, c->d_me_chunk.p);
    HIPCHK(c, c->d_setup.ensure(c, bt.n_jobs));
    hipLaunchKernelGGL(k_me_setup, dim3((bt.n_jobs + 255) / 256), dim3(256), 0, c->stream, c->sc, w, c->d_me_blocks.p,
                       bt.n_jobs, t, c->d_setup.p);
    const int ne = (int)bt.n_elems;
    MeWindow wb = w;  // 16 sub-blocks per block: a block's window row is one aligned 16-lane group
    wb.seg16 = std::all_of(bt.blocks.begin(), bt.blocks.end(), [](const MeBlockDev& b) { return b.n == 16; }) ? 1 : 0;
    hipLaunchKernelGGL(k_me_sad, dim3(round_grid((ne + 255) / 256)), dim3(256), 0, c->stream, c->sc, c->geo, wb,
                       c->d_me_blocks.p, (int)bt.blocks.size(), c->d_me_off.p, c->d_me_chunk.p, ne, c->d_setup.p,
                       make_cache(c), t, oit->second.y, oit->second.stride_y, sads);
    HIPCHK(c, hipGetLastError());
    // no wait per batch: every batch's host vectors live until the synchronisation below, and the
    // next batch's uploads into the same device buffers are ordered after this batch's kernels on
    // the stream (a wait here cost ~0.3 ms per batch, 60 batches per C5 call)
  }
  HIPCHK(c, hipEventRecord(c->ev1, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return MM_OK;
}

int mm_sad_window(mm_ctx* c, int cur_poc, const mm_me_block* blocks, int n, int range, int step, uint32_t* sads) {
  if (!c || n < 0 || (n > 0 && (!blocks || !sads)) || range < 0 || range > 64 || step <= 0) return MM_ERR_ARG;
  if (n == 0) return MM_OK;
  MeWindow w;
  w.range = range;
  w.step = step;
  w.side = 2 * range + 1;
  w.C = w.side * w.side;
  return me_run(c, cur_poc, blocks, n, w, sads);
}

int mm_sad_pattern(mm_ctx* c, int cur_poc, const mm_me_block* blocks, int n, const int32_t* offsets, int k,
                   uint32_t* sads) {
  if (!c || n < 0 || (n > 0 && (!blocks || !sads)) || k < 1 || k > ME_MAX_PAT || !offsets) return MM_ERR_ARG;
  MeWindow w;
  w.range = 0;
  w.step = 16;
  w.side = w.C = w.npat = k;
  for (int i = 0; i < k; i++) {
    const int32_t ox = offsets[2 * i], oy = offsets[2 * i + 1];
    if (ox < -4096 || ox > 4096 || oy < -4096 || oy > 4096) return fail(c, MM_ERR_ARG, "pattern offset beyond +-256 pel");
    for (int q = 0; q < i; q++)
      if (offsets[2 * q] == ox && offsets[2 * q + 1] == oy) return fail(c, MM_ERR_ARG, "repeated pattern offset");
    w.pat[2 * i] = (int16_t)ox;
    w.pat[2 * i + 1] = (int16_t)oy;
  }
  // the staged box: k_me_sad takes it from the first and last candidates' windows; the pattern's
  // bounding box extends it by these (whole samples, rounded outwards)
  int lx = 0, hx = 0, ly = 0, hy = 0;
  const int ax0 = std::min(w.pat[0], w.pat[2 * k - 2]), ax1 = std::max(w.pat[0], w.pat[2 * k - 2]);
  const int ay0 = std::min(w.pat[1], w.pat[2 * k - 1]), ay1 = std::max(w.pat[1], w.pat[2 * k - 1]);
  for (int i = 0; i < k; i++) {
    lx = std::min(lx, (w.pat[2 * i] - ax0) >> 4);
    hx = std::max(hx, (w.pat[2 * i] - ax1 + 15) >> 4);
    ly = std::min(ly, (w.pat[2 * i + 1] - ay0) >> 4);
    hy = std::max(hy, (w.pat[2 * i + 1] - ay1 + 15) >> 4);
  }
  w.box_lx = lx;
  w.box_hx = hx;
  w.box_ly = ly;
  w.box_hy = hy;
  if (n == 0) return MM_OK;
  return me_run(c, cur_poc, blocks, n, w, sads);
}

// MM-DMVR of a PU list: every PU is flagged MM_PUF_DMVR and the list runs the device-planned
// picture path with DMVR on (search, decision, refined prediction); the deltas are read back.
int mm_pred_dmvr(mm_ctx* c, int cur_poc, const mm_pu_desc* pus, int n, int16_t* dy, ptrdiff_t sdy, int16_t* dcb,
                 int16_t* dcr, ptrdiff_t sdc, int32_t* mvd_out) {
  if (!c || n < 0 || (n > 0 && !pus) || !dy || (c->geo.chroma && (!dcb || !dcr))) return MM_ERR_ARG;
  if (n == 0) return MM_OK;
  HIPCHK(c, hipSetDevice(c->device));
  std::vector<mm_pu_desc> flagged(pus, pus + n);
  long n_sub = 0;
  for (auto& u : flagged) {
    u.flags |= MM_PUF_DMVR;
    if (u.w > 0 && u.h > 0) n_sub += (long)((u.w + 15) / 16) * ((u.h + 15) / 16);
  }
  RCCHK(mm_pred_prepare(c, cur_poc, flagged.data(), n));
  c->prepared = false;  // the buffer holds this call's PUs, not a prepared picture
  RCCHK(launch_device_plan(c, cur_poc, c->d_pu_in.p, n, dy, sdy, dcb, dcr, sdc, -1, 0, 3, false, true, true));
  const int rc = read_status(c, nullptr);
  if (rc) return rc;
  // the deltas of the sub-PUs in placement order: PUs in list order (DMVR bucket placement keeps
  // input order), sub-PUs in raster order -- in the plan slot the call used (slot 0 while this call
  // runs without plan-ahead and DMVR keeps one stripe, but read from where it actually went)
  if (mvd_out && n_sub)
    HIPCHK(c, hipMemcpy(mvd_out, c->slot[c->last_slot].dmvr_mvd.p, 2 * (size_t)n_sub * sizeof(int32_t),
                        hipMemcpyDeviceToHost));
  return MM_OK;
}

// Device copy of the context's epipole list, refreshed when the list changed since the last copy.
static int sync_epi_table(mm_ctx* c) {
  if (c->epipoles.version() == c->epi_version) return MM_OK;
  std::vector<mmmvp::EpiDev> e;
  epi_entries(c->epipoles, &e);
  HIPCHK(c, hipEventSynchronize(c->ev_epi));  // the staging buffer may still feed the previous copy
  const int nb = c->epi_buf ^ 1;                // the table the current version does not use
  // its last readers (conversions of two versions back, on the MVP stream) must be done before the
  // context stream rewrites it; conversions on the context stream itself are ordered anyway
  if (c->epi_used[nb]) {
    HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_epi_done[nb], 0));
    c->epi_used[nb] = false;
  }
  if (e.size() > c->h_epi_cap) {
    if (c->h_epi) (void)hipHostFree(c->h_epi);
    c->h_epi = nullptr;
    c->h_epi_cap = 0;
    const size_t cap = std::max<size_t>(64, 2 * e.size());
    HIPCHK(c, hipHostMalloc(reinterpret_cast<void**>(&c->h_epi), cap * sizeof(mmmvp::EpiDev), hipHostMallocDefault));
    c->h_epi_cap = cap;
  }
  HIPCHK(c, c->d_epi[nb].ensure(c, std::max<size_t>(64, 2 * e.size())));  // growth retires the old table
  if (!e.empty()) {
    std::copy(e.begin(), e.end(), c->h_epi);
    HIPCHK(c, hipMemcpyAsync(c->d_epi[nb].p, c->h_epi, e.size() * sizeof(mmmvp::EpiDev), hipMemcpyHostToDevice,
                             c->stream));
    HIPCHK(c, hipEventRecord(c->ev_epi, c->stream));
    c->epi_fresh = true;
  }
  // the previous version's table: its readers are the conversions issued on the MVP stream so far
  if (c->mvp_on_own) {
    HIPCHK(c, hipEventRecord(c->ev_epi_done[c->epi_buf], c->mvp_stream));
    c->epi_used[c->epi_buf] = true;
  }
  c->epi_buf = nb;
  c->epi_n = (int)e.size();
  c->epi_version = c->epipoles.version();
  return MM_OK;
}

static int read_mvp_status(mm_ctx* c, int* first_bad) {
  if (first_bad) *first_bad = -1;
  HIPCHK(c, hipStreamSynchronize(mvp_stream_of(c)));
  if (!c->mvp_pending) return MM_OK;
  c->mvp_pending = false;
  unsigned long long w = 0;
  HIPCHK(c, hipMemcpy(&w, c->d_mvp_status.p, sizeof(w), hipMemcpyDeviceToHost));
  if (w) {  // sticky word: cleared only here, after the conversions that may have set it are done
    HIPCHK(c, hipMemsetAsync(c->d_mvp_status.p, 0, sizeof(w), mvp_stream_of(c)));
    HIPCHK(c, hipStreamSynchronize(mvp_stream_of(c)));
  }
  return decode_status(c, w, first_bad, "MVP query");
}

int mm_mvp_convert_device(mm_ctx* c, const mm_mvp_query* d_q, int n, int32_t* d_mv_out) {
  if (!c || n < 0 || (n > 0 && (!d_q || !d_mv_out))) return MM_ERR_ARG;
  if (n == 0) return MM_OK;
  HIPCHK(c, hipSetDevice(c->device));
  RCCHK(sync_epi_table(c));
  const mmmvp::EpiTable et{c->d_epi[c->epi_buf].p, c->epi_n};
  unsigned long long* st = c->d_mvp_status.p;  // sticky (read_mvp_status clears it)
  const hipStream_t ms = mvp_stream_of(c);
  if (c->mvp_on_own && c->epi_fresh) HIPCHK(c, hipStreamWaitEvent(ms, c->ev_epi, 0));  // the table copy
  c->epi_fresh = false;
  c->timed = c->call_timing || !c->mvp_on_own;
  const int nb = (n + MVP_BLOCK - 1) / MVP_BLOCK;
  // Picture-sized batches are sorted by model pair first (k_mvp_bucket / k_mvp_place: C3's 156 K
  // queries 74 -> 68 us, MVP in the loop 0.2135 -> 0.208 ms per picture); below MVP_SORT_MIN the two
  // extra launches cost more than the coherence gains (a CTU's 136 queries: +8 us), and the
  // queries are converted in input order.
  const bool sort = n >= MVP_SORT_MIN;
  if (sort) {
    // the sort buffers are shared by the calls of the context: growing them frees the old ones in
    // stream order behind the queued work (DevBuf::ensure -> dev_free), so a conversion still running
    // on the MVP stream keeps its buffers
    HIPCHK(c, c->d_mvp_local.ensure(c, n));
    HIPCHK(c, c->d_mvp_perm.ensure(c, n));
  }
  if (c->timed) HIPCHK(c, hipEventRecord(c->ev0, ms));
  if (sort) {
    unsigned* bins = c->d_mvp_bins.p + MVP_COUNTERS * c->mvp_sort_par;
    hipLaunchKernelGGL(k_mvp_bucket, dim3(nb), dim3(MVP_BLOCK), 0, ms, d_q, n, bins,
                       c->d_mvp_bins.p + MVP_COUNTERS * (c->mvp_sort_par ^ 1), c->d_mvp_local.p);
    hipLaunchKernelGGL(k_mvp_place, dim3(nb), dim3(MVP_BLOCK), 0, ms, d_q, n, bins, c->d_mvp_local.p, c->d_mvp_perm.p);
    c->mvp_sort_par ^= 1;
  }
  hipLaunchKernelGGL(k_mvp_dev, dim3(nb), dim3(MVP_BLOCK), 0, ms, c->sc, d_q, n, sort ? c->d_mvp_perm.p : nullptr,
                     c->prm.active_models, et, d_mv_out, st);
  HIPCHK(c, hipGetLastError());
  if (c->timed) HIPCHK(c, hipEventRecord(c->ev1, ms));
  c->mvp_pending = true;
  return MM_OK;
}

// motionVectorInDesiredMotionModel one query at a time on the calling host thread, for the
// candidates VTM converts in decoding order (spatial merge / AMVP candidates: the neighbour's final
// MV, UnitTools.cpp:2930-2992, 3134-3167): the same csrc/mm_mvp.h bodies as k_mvp_dev, compiled
// for the host.  No device work and no context: the sequence parameters and an EpipoleList handle
// (a context's own list through mm_get_epipole_list, or a standalone one) are the inputs.
int mm_mvp_convert_host(const mm_seq_params* p, mm_epipole_list* e, const mm_mvp_query* q, int n, int32_t* mv_out,
                        int* first_bad) {
  if (first_bad) *first_bad = -1;
  if (!p || n < 0 || (n > 0 && (!q || !mv_out)) || p->width <= 0 || p->height <= 0) return MM_ERR_ARG;
  const SeqConst sc = seq_const(*p);
  mmmvp::EpiTable et{nullptr, 0};
  if (e) {
    if (e->host_version != e->l->version()) {
      epi_entries(*e->l, &e->host);
      e->host_version = e->l->version();
    }
    et = mmmvp::EpiTable{e->host.data(), (int)e->host.size()};
  }
  int rc = MM_OK;
  for (int i = 0; i < n; i++) {
    const int code = mmmvp::mvp_query(sc, q[i], p->active_models, et, mv_out + 2 * i);
    if (code && rc == MM_OK) {  // the lowest failing query, as mm_mvp_status reports it
      rc = code;
      if (first_bad) *first_bad = i;
    }
  }
  return rc;
}

int mm_set_mvp_stream(mm_ctx* c, void* s) {
  if (!c) return MM_ERR_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(mvp_stream_of(c)));  // conversions already issued finish where they were
  c->mvp_stream = (hipStream_t)s;
  c->mvp_on_own = s != nullptr;
  c->epi_fresh = c->mvp_on_own;  // order the next conversion after any table copy made so far
  return MM_OK;
}

int mm_mvp_status(mm_ctx* c, int* first_bad_query) {
  if (!c) return MM_ERR_ARG;
  return read_mvp_status(c, first_bad_query);
}

int mm_mvp_convert(mm_ctx* c, const mm_mvp_query* q, int n, int32_t* mv_out) {
  if (!c || n < 0 || (n > 0 && (!q || !mv_out))) return MM_ERR_ARG;
  if (n == 0) return MM_OK;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, c->d_mvp_q.ensure(c, n));
  HIPCHK(c, c->d_mvp_out.ensure(c, 2 * (size_t)n));
  HIPCHK(c, hipMemcpyAsync(c->d_mvp_q.p, q, (size_t)n * sizeof(mm_mvp_query), hipMemcpyHostToDevice, mvp_stream_of(c)));
  RCCHK(mm_mvp_convert_device(c, c->d_mvp_q.p, n, c->d_mvp_out.p));
  HIPCHK(c, hipMemcpyAsync(mv_out, c->d_mvp_out.p, 2 * (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost,
                           mvp_stream_of(c)));
  return read_mvp_status(c, nullptr);
}

int mm_set_stage_timing(mm_ctx* c, int on) {
  if (!c) return MM_ERR_ARG;
  c->stage_timing = on != 0;
  return MM_OK;
}

int mm_last_stage_timing(mm_ctx* c, float ms[4]) {
  if (!c || !ms) return MM_ERR_ARG;
  if (!c->stage_timing) return fail(c, MM_ERR_ARG, "stage timing is off (mm_set_stage_timing)");
  HIPCHK(c, hipEventSynchronize(c->ev1));
  hipEvent_t e[5] = {c->ev0, c->ev_stage[0], c->ev_stage[1], c->ev_stage[2], c->ev1};
  for (int i = 0; i < 4; i++) HIPCHK(c, hipEventElapsedTime(&ms[i], e[i], e[i + 1]));
  return MM_OK;
}

int mm_set_kernel_timing(mm_ctx* c, int on) {
  if (!c) return MM_ERR_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  if (on && !c->kt_ev[0][0]) {
    // timing events without the system-scope release (they publish nothing, like the slot gates)
    for (auto& pr : c->kt_ev)
      for (auto& e : pr) HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
  }
  if (!on && c->kt_on && c->plan_ahead) {
    // the gates may point into the ring: gate on the current position of the context stream again
    HIPCHK(c, hipEventRecord(c->ev_gate[0], c->stream));
    HIPCHK(c, hipEventRecord(c->ev_gate[1], c->stream));
    c->gate[0] = c->ev_gate[0];
    c->gate[1] = c->ev_gate[1];
  }
  c->kt_on = on != 0;
  c->kt_n = 0;
  return MM_OK;
}

int mm_kernel_times(mm_ctx* c, float* ms, int cap, int* n_out) {
  if (!c || !n_out || cap < 0 || (cap > 0 && !ms)) return MM_ERR_ARG;
  *n_out = 0;
  if (!c->kt_ev[0][0]) return fail(c, MM_ERR_ARG, "kernel timing was never on (mm_set_kernel_timing)");
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const int n = std::min(c->kt_n, mm_ctx::KT_RING);
  const int first = c->kt_n - n;  // the last n launches, oldest first
  int k = 0;
  for (int i = 0; i < n && k < cap; i++, k++) {
    hipEvent_t* pr = c->kt_ev[(first + i) % mm_ctx::KT_RING];
    HIPCHK(c, hipEventElapsedTime(&ms[k], pr[0], pr[1]));
  }
  *n_out = k;
  c->kt_n = 0;
  return MM_OK;
}

int mm_filter(mm_ctx* c, int comp, int vertical, const int16_t* src, ptrdiff_t src_stride, int16_t* dst,
              ptrdiff_t dst_stride, int w, int h, int frac, int is_first, int is_last) {
  if (!c || !src || !dst || w <= 0 || h <= 0) return MM_ERR_ARG;
  if (frac < 0 || frac >= (comp ? 32 : 16)) return fail(c, MM_ERR_ARG, "invalid fraction");
  if (!vertical && !is_first) return fail(c, MM_ERR_ARG, "filterHor is always isFirst");
  HIPCHK(c, hipSetDevice(c->device));
  // Window the filter reads (InterpolationFilter.cpp:540-644): (NT/2 - 1) samples before the block
  // and NT/2 after it along the filtered axis only (mm360.h states this margin to callers).
  const int NT = comp ? 4 : 8, before = NT / 2 - 1, after = NT / 2;
  const int mx0 = vertical ? 0 : before, mx1 = vertical ? 0 : after;
  const int my0 = vertical ? before : 0, my1 = vertical ? after : 0;
  const int ww = w + mx0 + mx1, hh = h + my0 + my1;
  std::vector<int16_t> win((size_t)ww * hh);
  for (int r = 0; r < hh; r++)
    for (int q = 0; q < ww; q++) win[(size_t)r * ww + q] = src[(long)(r - my0) * src_stride + (q - mx0)];
  int16_t *dsrc = nullptr, *ddst = nullptr;
  HIPCHK(c, dev_alloc(c, reinterpret_cast<void**>(&dsrc), win.size() * 2));
  hipError_t e = dev_alloc(c, reinterpret_cast<void**>(&ddst), (size_t)w * h * 2);
  if (e == hipSuccess) e = hipMemcpyAsync(dsrc, win.data(), win.size() * 2, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_filter, dim3((w * h + 255) / 256), dim3(256), 0, c->stream, comp, vertical,
                       dsrc + (size_t)my0 * ww + mx0, ww, ddst, w, w, h, frac, is_first, is_last, c->geo.bd);
    e = hipGetLastError();
  }
  std::vector<int16_t> out((size_t)w * h);
  if (e == hipSuccess) e = hipMemcpyAsync(out.data(), ddst, out.size() * 2, hipMemcpyDeviceToHost, c->stream);
  dev_free(c, dsrc);
  if (ddst) dev_free(c, ddst);
  const hipError_t es = hipStreamSynchronize(c->stream);  // the copies (pageable host memory) and the frees
  if (e == hipSuccess) e = es;
  if (e != hipSuccess) return fail(c, MM_ERR_HIP, hipGetErrorString(e));
  for (int r = 0; r < h; r++)
    for (int q = 0; q < w; q++) dst[(long)r * dst_stride + q] = out[(size_t)r * w + q];
  return MM_OK;
}

// ------------------------------------------------------------- bitstream side (mm_syntax.h)
int mm_sps_mm_write(const mm_sps_mm* sps, uint8_t* buf, int64_t cap_bytes, int64_t* bit_pos) {
  if (!sps || !buf || !bit_pos || cap_bytes < 0 || *bit_pos < 0 || !mmsyn::sps_valid(*sps)) return MM_ERR_ARG;
  mmsyn::BitWriter w{buf, cap_bytes * 8, *bit_pos};
  mmsyn::write_sps_mm(w, *sps);
  if (w.bad) return MM_ERR_ARG;
  *bit_pos = w.pos;
  return MM_OK;
}

int mm_sps_mm_read(const uint8_t* buf, int64_t nbits, int64_t* bit_pos, mm_sps_mm* sps) {
  if (!buf || !bit_pos || !sps || nbits < 0 || *bit_pos < 0) return MM_ERR_ARG;
  mmsyn::BitReader r{buf, nbits, *bit_pos};
  mm_sps_mm s;
  if (!mmsyn::read_sps_mm(r, s)) return MM_ERR_BITSTREAM;
  *sps = s;
  *bit_pos = r.pos;
  return MM_OK;
}

int mm_ph_epipole_write(const mm_sps_mm* sps, const int32_t delta[3], uint8_t* buf, int64_t cap_bytes,
                        int64_t* bit_pos) {
  if (!sps || !delta || !buf || !bit_pos || cap_bytes < 0 || *bit_pos < 0) return MM_ERR_ARG;
  mmsyn::BitWriter w{buf, cap_bytes * 8, *bit_pos};
  mmsyn::write_ph_epipole(w, *sps, delta);
  if (w.bad) return MM_ERR_ARG;
  *bit_pos = w.pos;
  return MM_OK;
}

int mm_ph_epipole_read(const mm_sps_mm* sps, const uint8_t* buf, int64_t nbits, int64_t* bit_pos, int32_t delta[3]) {
  if (!sps || !buf || !bit_pos || !delta || nbits < 0 || *bit_pos < 0) return MM_ERR_ARG;
  mmsyn::BitReader r{buf, nbits, *bit_pos};
  int32_t d[3];
  if (!mmsyn::read_ph_epipole(r, *sps, d)) return MM_ERR_BITSTREAM;
  std::memcpy(delta, d, sizeof d);
  *bit_pos = r.pos;
  return MM_OK;
}

int mm_motion_model_candidates(const mm_sps_mm* sps, int pred_type, const int8_t* col_models, int grid_w,
                               int grid_h, int pic_w, int pic_h, int col_list, int x, int y, int w, int h,
                               int32_t* cand, int32_t* n_cand) {
  if (!sps || !cand || !n_cand || pred_type < 0 || pred_type > 3) return MM_ERR_ARG;
  const mmsyn::ColField f{col_models, grid_w, grid_h};
  int n = 0;
  if (!mmsyn::order_candidates(*sps, pred_type, &f, pic_w, pic_h, col_list, x, y, w, h, cand, &n)) return MM_ERR_ARG;
  *n_cand = n;
  return MM_OK;
}

// the rows' candidate lists: a permutation of the active models, n_cand of them
static bool mm_cand_rows_ok(const mm_sps_mm& sps, const int32_t* cand, int n_pu, int* n_out) {
  int32_t act[mmsyn::NUM_MODELS];
  const int n = mmsyn::active_models(sps, act);
  for (int p = 0; p < n_pu; ++p) {
    const int32_t* row = cand + size_t(p) * MM_NUM_MODEL_IDS;
    uint32_t seen = 0;
    for (int i = 0; i < n; ++i) {
      if (row[i] < 0 || row[i] >= mmsyn::NUM_MODELS || (seen >> row[i]) & 1u) return false;
      if (std::find(act, act + n, row[i]) == act + n) return false;
      seen |= 1u << row[i];
    }
  }
  *n_out = n;
  return true;
}

int mm_motion_model_encode(const mm_sps_mm* sps, int slice_qp, int init_type, int coding_depth, int n_pu,
                           const int32_t* cand, const uint8_t* affine, const int32_t* models, uint8_t* out,
                           int64_t cap_bytes, int64_t* nbytes) {
  if (!sps || n_pu < 0 || (n_pu && (!cand || !models)) || !out || !nbytes || init_type < 0 || init_type > 2 ||
      coding_depth < 0 || cap_bytes < 0)
    return MM_ERR_ARG;
  int n = 0;
  if (!mm_cand_rows_ok(*sps, cand, n_pu, &n)) return MM_ERR_ARG;
  const bool mm_on = mmsyn::use_multi_model(*sps);
  mmsyn::MotionModelCtx ctx;
  ctx.init(slice_qp, init_type);
  mmsyn::CabacEncoder e;
  for (int p = 0; p < n_pu; ++p) {
    if (!mm_on || (affine && affine[p])) {  // CABACWriter.cpp:1860-1864
      if (models[p] != mmsyn::CLASSIC) return MM_ERR_ARG;
      continue;
    }
    if (!mmsyn::encode_motion_model(e, ctx, cand + size_t(p) * MM_NUM_MODEL_IDS, n, coding_depth, models[p]))
      return MM_ERR_ARG;
  }
  e.end_of_slice();
  if (int64_t(e.out.size()) > cap_bytes) return MM_ERR_ARG;
  std::memcpy(out, e.out.data(), e.out.size());
  *nbytes = int64_t(e.out.size());
  return MM_OK;
}

int mm_motion_model_decode(const mm_sps_mm* sps, int slice_qp, int init_type, int coding_depth, int n_pu,
                           const int32_t* cand, const uint8_t* affine, const uint8_t* in, int64_t nbytes,
                           int32_t* models_out) {
  if (!sps || n_pu < 0 || (n_pu && (!cand || !models_out)) || !in || nbytes < 0 || init_type < 0 ||
      init_type > 2 || coding_depth < 0)
    return MM_ERR_ARG;
  int n = 0;
  if (!mm_cand_rows_ok(*sps, cand, n_pu, &n)) return MM_ERR_ARG;
  const bool mm_on = mmsyn::use_multi_model(*sps);
  mmsyn::MotionModelCtx ctx;
  ctx.init(slice_qp, init_type);
  mmsyn::CabacDecoder d{in, nbytes};
  d.start();
  for (int p = 0; p < n_pu; ++p) {
    if (!mm_on || (affine && affine[p])) {  // CABACReader.cpp:2172-2176
      models_out[p] = mmsyn::CLASSIC;
      continue;
    }
    models_out[p] = mmsyn::decode_motion_model(d, ctx, cand + size_t(p) * MM_NUM_MODEL_IDS, n, coding_depth);
    if (d.bad || models_out[p] == mmsyn::INVALID) return MM_ERR_BITSTREAM;
  }
  if (!d.bin_trm() || !d.finish()) return MM_ERR_BITSTREAM;
  return MM_OK;
}

}  // extern "C"
