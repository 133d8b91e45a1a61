// mm_kernels.hip -- gfx950 kernels and the C-ABI (include/mm360.h) of the 360-degree
// multi-model motion-compensation path.
//
// Pipeline of one mm_pred_run (one picture's PU list, all device work, one stream):
//   k_setup    thread per reprojection job (PU x list x {luma, chroma}): the per-block part of
//              reprojectMotionVectorSubblocks (centre transforms, rotation matrices, k, ...).
//   k_reproj   thread per sub-block element of every job: <Model>::modelMotion[Cached] + NaN
//              fallback + fixed-point rounding -> int32 (X, Y) per element.
//   k_mc       thread per luma 4x4 sub-block of every PU: for each used list, the 8-tap luma and
//              4-tap 4:2:0 chroma sub-block predictions (xPredInterBlkMM :776-828) and the
//              addAvg / uni output (xWeightedAverage), written straight into the picture planes.
// Reference planes stay resident in HBM, unpadded; the edge-replication margin of the reference
// is realised by address clamping (identical results, no padded copies).
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
#include "mm_pipeline.h"
#include "mm_plan.h"

using namespace mmpipe;

#define MM_VERSION 100

namespace {

__constant__ int8_t c_luma_taps[16][8] = MM_LUMA_TAPS_INIT;
__constant__ int8_t c_chroma_taps[32][4] = MM_CHROMA_TAPS_INIT;

__global__ void k_mpa_cache(SeqConst sc, int plane, int cols, int rows, float* px, float* py, uint8_t* vip) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= cols * rows) return;
  mpa_cache_thread(t, sc, plane, cols, rows, px, py, vip);
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
  int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_elems) return;
  reproj_thread(g, sc, jobs, n_jobs, job_offsets, chunk_start, setups, cache, out);
}

__global__ void __launch_bounds__(256) k_mc(Geometry geo, const PuDev* __restrict__ pus, int n_pus,
                                            const int* __restrict__ pu_offsets, const int* __restrict__ chunk_start,
                                            int n_sb, const JobDev* __restrict__ jobs, const int32_t* __restrict__ reproj,
                                            const RefDev* __restrict__ refs, int16_t* __restrict__ dst_y, int dsy,
                                            int16_t* __restrict__ dst_cb, int16_t* __restrict__ dst_cr, int dsc) {
  int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_sb) return;
  const Taps taps{c_luma_taps, c_chroma_taps};
  mc_thread(g, geo, taps, pus, n_pus, pu_offsets, chunk_start, jobs, reproj, refs, dst_y, dsy, dst_cb, dst_cr, dsc);
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
};

template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t n) {
    if (n <= cap && p) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(n, 1);
    hipError_t e = hipMalloc(&p, want * sizeof(T));
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

struct mm_ctx {
  mm_seq_params prm{};
  SeqConst sc{};
  Geometry geo{};
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  std::map<int, RefHost> refs;
  EpipoleMap epipoles;
  float* mpa_px[3] = {nullptr, nullptr, nullptr};
  float* mpa_py[3] = {nullptr, nullptr, nullptr};
  uint8_t* mpa_vip[3] = {nullptr, nullptr, nullptr};
  Plan plan;
  DevBuf<JobDev> d_jobs;
  DevBuf<int> d_job_off, d_job_chunk, d_pu_off, d_pu_chunk;
  DevBuf<BlockSetup> d_setup;
  DevBuf<int32_t> d_reproj;
  DevBuf<PuDev> d_pus;
  DevBuf<RefDev> d_refs;
  DevBuf<M3> d_ged;
  bool prepared = false;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
};

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
  HIPCHK(c, d.ensure(h.size()));
  if (!h.empty()) HIPCHK(c, hipMemcpyAsync(d.p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice, c->stream));
  return MM_OK;
}

static MpaCache make_cache(mm_ctx* c) {
  MpaCache mc{};
  for (int pl = 0; pl < 3; pl++) {
    mc.px[pl] = c->mpa_px[pl];
    mc.py[pl] = c->mpa_py[pl];
    mc.vip[pl] = c->mpa_vip[pl];
  }
  mc.cols = c->geo.W / 4;
  mc.rows = c->geo.H / 4;
  return mc;
}

static int upload_jobs(mm_ctx* c) {
  RCCHK(upload(c, c->d_jobs, c->plan.jobs));
  RCCHK(upload(c, c->d_job_off, c->plan.job_off));
  RCCHK(upload(c, c->d_job_chunk, c->plan.job_chunk));
  RCCHK(upload(c, c->d_ged, c->plan.ged));
  HIPCHK(c, c->d_setup.ensure(c->plan.jobs.size()));
  HIPCHK(c, c->d_reproj.ensure(2 * (size_t)c->plan.n_elems));
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

const char* mm_last_error(mm_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int mm_create(const mm_seq_params* p, int device, mm_ctx** out_ctx) {
  if (!p || !out_ctx) return MM_ERR_ARG;
  *out_ctx = nullptr;
  if (p->width <= 0 || p->height <= 0 || (p->width & 7) || (p->height & 7)) return MM_ERR_ARG;
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
  c->sc.Wf = (float)p->width;
  c->sc.Hf = (float)p->height;
  c->sc.off = p->mm_offset4x4 == 4 ? 1.5f : (float)p->mm_offset4x4;
  c->sc.focal = (float)(1. / std::tan(M_PI / p->height));  // Projection.h:127-130
  c->sc.res = (float)(M_PI / p->height);                    // MVReprojection.cpp:27,33,39
  c->sc.ged_flavor = p->ged_flavor;
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
  if (hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess) {
    mm_destroy(c);
    return MM_ERR_HIP;
  }
  // MPA frame caches (MVReprojection::init -> MotionPlaneAdaptiveMotionModel::fillCache)
  const int cols = p->width / 4, rows = p->height / 4, n = cols * rows;
  for (int pl = 0; pl < 3; pl++) {
    if (!(p->active_models & (1u << (MPA_FRONT_BACK + pl)))) continue;
    if (hipMalloc(&c->mpa_px[pl], n * sizeof(float)) != hipSuccess ||
        hipMalloc(&c->mpa_py[pl], n * sizeof(float)) != hipSuccess || hipMalloc(&c->mpa_vip[pl], n) != hipSuccess) {
      mm_destroy(c);
      return MM_ERR_HIP;
    }
    hipLaunchKernelGGL(k_mpa_cache, dim3((n + 255) / 256), dim3(256), 0, c->stream, c->sc, MPA_FRONT_BACK + pl, cols,
                       rows, c->mpa_px[pl], c->mpa_py[pl], c->mpa_vip[pl]);
  }
  if (hipGetLastError() != hipSuccess || hipStreamSynchronize(c->stream) != hipSuccess) {
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
  for (auto& kv : c->refs) {
    (void)hipFree(kv.second.y);
    (void)hipFree(kv.second.cb);
    (void)hipFree(kv.second.cr);
  }
  for (int pl = 0; pl < 3; pl++) {
    if (c->mpa_px[pl]) (void)hipFree(c->mpa_px[pl]);
    if (c->mpa_py[pl]) (void)hipFree(c->mpa_py[pl]);
    if (c->mpa_vip[pl]) (void)hipFree(c->mpa_vip[pl]);
  }
  c->d_jobs.release();
  c->d_job_off.release();
  c->d_job_chunk.release();
  c->d_pu_off.release();
  c->d_pu_chunk.release();
  c->d_setup.release();
  c->d_reproj.release();
  c->d_pus.release();
  c->d_refs.release();
  c->d_ged.release();
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  delete c;
  return MM_OK;
}

int mm_set_stream(mm_ctx* c, void* s) {
  if (!c) return MM_ERR_ARG;
  c->stream = (hipStream_t)s;
  return MM_OK;
}

int mm_synchronize(mm_ctx* c) {
  if (!c) return MM_ERR_ARG;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return MM_OK;
}

int mm_set_epipole(mm_ctx* c, int cur, int ref, const int32_t q24[3]) {
  if (!c || !q24) return MM_ERR_ARG;
  c->epipoles[{cur, ref}] = {q24[0], q24[1], q24[2]};
  return MM_OK;
}

int mm_upload_ref(mm_ctx* c, int poc, const int16_t* y, ptrdiff_t sy, const int16_t* cb, const int16_t* cr,
                  ptrdiff_t sc_, int src_dev) {
  if (!c || !y) return MM_ERR_ARG;
  if (c->geo.chroma && (!cb || !cr)) return fail(c, MM_ERR_ARG, "chroma planes required for 4:2:0");
  HIPCHK(c, hipSetDevice(c->device));
  RefHost& r = c->refs[poc];
  const int W = c->geo.W, H = c->geo.H, Wc = c->geo.Wc, Hc = c->geo.Hc;
  if (!r.y) {
    r.stride_y = (W + 63) & ~63;
    r.stride_c = (Wc + 63) & ~63;
    HIPCHK(c, hipMalloc(&r.y, (size_t)r.stride_y * H * sizeof(int16_t)));
    if (c->geo.chroma) {
      HIPCHK(c, hipMalloc(&r.cb, (size_t)r.stride_c * Hc * sizeof(int16_t)));
      HIPCHK(c, hipMalloc(&r.cr, (size_t)r.stride_c * Hc * sizeof(int16_t)));
    }
  }
  hipMemcpyKind k = src_dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
  HIPCHK(c, hipMemcpy2DAsync(r.y, r.stride_y * 2, y, sy * 2, W * 2, H, k, c->stream));
  if (c->geo.chroma) {
    HIPCHK(c, hipMemcpy2DAsync(r.cb, r.stride_c * 2, cb, sc_ * 2, Wc * 2, Hc, k, c->stream));
    HIPCHK(c, hipMemcpy2DAsync(r.cr, r.stride_c * 2, cr, sc_ * 2, Wc * 2, Hc, k, c->stream));
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->prepared = false;  // slot pointers may have changed
  return MM_OK;
}

int mm_release_ref(mm_ctx* c, int poc) {
  if (!c) return MM_ERR_ARG;
  auto it = c->refs.find(poc);
  if (it == c->refs.end()) return fail(c, MM_ERR_NOREF, "reference POC not uploaded");
  (void)hipStreamSynchronize(c->stream);
  (void)hipFree(it->second.y);
  (void)hipFree(it->second.cb);
  (void)hipFree(it->second.cr);
  c->refs.erase(it);
  c->prepared = false;
  return MM_OK;
}

int mm_reproject(mm_ctx* c, const mm_block_desc* blocks, int n, int32_t* out_xy) {
  if (!c || n < 0 || (n > 0 && (!blocks || !out_xy))) return MM_ERR_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  c->prepared = false;
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

int mm_pred_prepare(mm_ctx* c, int cur_poc, const mm_pu_desc* pus, int n) {
  if (!c || n < 0 || (n > 0 && !pus)) return MM_ERR_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  c->prepared = false;
  Planner pl(seq_info(c->prm), c->epipoles, &c->plan);
  int rc = pl.plan_pus(cur_poc, pus, n, [c](int poc) { return c->refs.count(poc) != 0; });
  if (rc) return fail(c, rc, c->plan.err);
  std::vector<RefDev> refs;
  for (int poc : c->plan.ref_pocs) {
    const RefHost& r = c->refs[poc];
    refs.push_back(RefDev{r.y, r.cb, r.cr, r.stride_y, r.stride_c});
  }
  RCCHK(upload_jobs(c));
  RCCHK(upload(c, c->d_pus, c->plan.pus));
  RCCHK(upload(c, c->d_pu_off, c->plan.pu_off));
  RCCHK(upload(c, c->d_pu_chunk, c->plan.pu_chunk));
  RCCHK(upload(c, c->d_refs, refs));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->prepared = true;
  return MM_OK;
}

int mm_pred_run(mm_ctx* c, int16_t* dy, ptrdiff_t sdy, int16_t* dcb, int16_t* dcr, ptrdiff_t sdc) {
  if (!c || !dy || (c->geo.chroma && (!dcb || !dcr))) return MM_ERR_ARG;
  if (!c->prepared) return fail(c, MM_ERR_ARG, "mm_pred_run without a valid mm_pred_prepare");
  const int n_pus = (int)c->plan.pus.size(), n_sb = c->plan.n_sb;
  if (n_pus == 0) return MM_OK;
  HIPCHK(c, hipEventRecord(c->ev0, c->stream));
  RCCHK(run_reproj_kernels(c));
  hipLaunchKernelGGL(k_mc, dim3((n_sb + 255) / 256), dim3(256), 0, c->stream, c->geo, c->d_pus.p, n_pus, c->d_pu_off.p,
                     c->d_pu_chunk.p, n_sb, c->d_jobs.p, c->d_reproj.p, c->d_refs.p, dy, (int)sdy, dcb, dcr, (int)sdc);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipEventRecord(c->ev1, c->stream));
  return MM_OK;
}

int mm_pred(mm_ctx* c, int cur_poc, const mm_pu_desc* pus, int n, int16_t* dy, ptrdiff_t sdy, int16_t* dcb,
            int16_t* dcr, ptrdiff_t sdc) {
  RCCHK(mm_pred_prepare(c, cur_poc, pus, n));
  RCCHK(mm_pred_run(c, dy, sdy, dcb, dcr, sdc));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return MM_OK;
}

int mm_last_timing(mm_ctx* c, float* ms) {
  if (!c || !ms) return MM_ERR_ARG;
  HIPCHK(c, hipEventSynchronize(c->ev1));
  HIPCHK(c, hipEventElapsedTime(ms, c->ev0, c->ev1));
  return MM_OK;
}

int mm_filter(mm_ctx* c, int comp, int vertical, const int16_t* src, ptrdiff_t src_stride, int16_t* dst,
              ptrdiff_t dst_stride, int w, int h, int frac, int is_first, int is_last) {
  if (!c || !src || !dst || w <= 0 || h <= 0) return MM_ERR_ARG;
  if (frac < 0 || frac >= (comp ? 32 : 16)) return fail(c, MM_ERR_ARG, "invalid fraction");
  if (!vertical && !is_first) return fail(c, MM_ERR_ARG, "filterHor is always isFirst");
  HIPCHK(c, hipSetDevice(c->device));
  const int NT = comp ? 4 : 8, m = NT / 2;
  const int ww = w + 2 * m, hh = h + 2 * m;
  std::vector<int16_t> win((size_t)ww * hh);
  for (int r = 0; r < hh; r++)
    for (int q = 0; q < ww; q++) win[(size_t)r * ww + q] = src[(long)(r - m) * src_stride + (q - m)];
  int16_t *dsrc = nullptr, *ddst = nullptr;
  HIPCHK(c, hipMalloc(&dsrc, win.size() * 2));
  hipError_t e = hipMalloc(&ddst, (size_t)w * h * 2);
  if (e == hipSuccess) e = hipMemcpy(dsrc, win.data(), win.size() * 2, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_filter, dim3((w * h + 255) / 256), dim3(256), 0, c->stream, comp, vertical,
                       dsrc + (size_t)m * ww + m, ww, ddst, w, w, h, frac, is_first, is_last, c->geo.bd);
    e = hipGetLastError();
  }
  std::vector<int16_t> out((size_t)w * h);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e == hipSuccess) e = hipMemcpy(out.data(), ddst, out.size() * 2, hipMemcpyDeviceToHost);
  (void)hipFree(dsrc);
  if (ddst) (void)hipFree(ddst);
  if (e != hipSuccess) return fail(c, MM_ERR_HIP, hipGetErrorString(e));
  for (int r = 0; r < h; r++)
    for (int q = 0; q < w; q++) dst[(long)r * dst_stride + q] = out[(size_t)r * w + q];
  return MM_OK;
}

}  // extern "C"
