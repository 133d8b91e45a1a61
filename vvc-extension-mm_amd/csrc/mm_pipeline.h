// mm_pipeline.h -- work descriptors and per-thread bodies of the MC pipeline (host + device).
//
// The HIP kernels in mm_kernels.hip are one-line wrappers around these bodies; the CPU twin
// used by the CPU test suite (tests/native/host_twin.cpp) loops over the same bodies, so the
// device logic is exercised bit-for-bit on the host before it ever reaches a GPU.
#pragma once
#include "mm_filter.h"
#include "mm_models.h"

namespace mmpipe {
using namespace mmmod;
using namespace mmflt;

struct RefDev {
  const int16_t* y;
  const int16_t* cb;
  const int16_t* cr;
  int stride_y, stride_c;
};

// One reprojection job == one reprojectMotionVectorSubblocks call
// 64 bytes, 16-byte aligned: written and read as four 16-byte words (k_plan_place, k_reproj*)
struct alignas(16) JobDev {
  int x, y;    // block position in LUMA units (grid origin)
  int cw, ch;  // block size in component units
  int mv_hor, mv_ver;
  int n;        // elements = (cw/sbw)*(ch/sbh)
  int rows;     // ch/sbh (Eigen column-major rows)
  int offset;   // first element in the result array
  // device-planned prediction: where k_mc finds this job's results (McIn, one record per luma
  // 4x4 sub-block of the PU, row-major from sb_base)
  int sb_base, pu_cols;
  int16_t model;
  int16_t ged_idx;  // index into the GED rotation table (-1 if not GED)
  int8_t comp;      // 0 luma, 1 chroma (4:2:0)
  int8_t list, slot;
  int8_t alias;     // MPA chroma == luma, fill both records
};
static_assert(sizeof(JobDev) == 64, "JobDev is four 16-byte words");

// Per-luma-sub-block inputs of k_mc, written by the reprojection of a device-planned picture so
// that k_mc reads them with one coalesced load per list instead of chasing PU -> job -> result:
// lum[l][g] = (xPos/xFrac fixed point X, Y, PU id << 5 | reference slot, oy << 16 | ox) and chr[l][g] = the
// chroma X, Y (1/32 pel) of list l for luma sub-block g.
struct alignas(16) mm_int4 {
  int x, y, z, w;
};
struct alignas(8) mm_int2 {
  int x, y;
};
struct McIn {
  mm_int4* lum[2];
  mm_int2* chr[2];
};

struct alignas(16) PuDev {  // 48 bytes: three 16-byte words
  int x, y, w, h;
  int ref_slot[2];  // -1 = list unused
  int job[2][2];    // [list][comp] -> job index
  int sb_offset;    // first luma sub-block of this PU in the k_mc enumeration
};

// Frame-grid caches, row-major [j][i] over the (W/4) x (H/4) grid x = 4i + off, y = 4j + off:
//  * MPA perspective coordinates per plane (MotionPlaneAdaptiveMotionModel::fillCache);
//  * the sphere point of every grid position and TAN's per-point terms (GridTerms), packet math,
//    used by packet lanes of TAN / 3DT / ROT / GED blocks (null when no such model is active).
struct MpaCache {
  const float* px[3];
  const float* py[3];
  const uint8_t* vip[3];
  int cols, rows;  // W/4, H/4
  const float* sx;
  const float* sy;
  const float* sz;
  const float* ta;   // TAN alpha
  const float* tse;  // TAN psin(eps)
  const float* tce;  // TAN pcos(eps)
};

// k_sph_cache: GridTerms of grid point t (packet math, as every element of an N % 4 == 0 block)
MM_HD void sph_cache_thread(int t, const SeqConst& sc, int cols, float* sx, float* sy, float* sz, float* ta, float* tse,
                            float* tce) {
  const int j = t / cols, i = t - j * cols;
  const Math m{1};
  const V3 p = erp_to_sphere(4.0f * (float)i + sc.off, 4.0f * (float)j + sc.off, sc, m);
  sx[t] = p.x;
  sy[t] = p.y;
  sz[t] = p.z;
  if (ta) {
    const V3 sp = cart_to_sph(p, m, true);
    const float eps = PI_2_F - sp.y;
    ta[t] = sp.z;
    tse[t] = m.sin(eps);
    tce[t] = m.cos(eps);
  }
}

// Grid terms of element (row, col) of job j when it is a packet lane and the caches hold them.
MM_HD void load_grid_terms(const MpaCache& cache, const JobDev& j, int row, int col, bool packet, GridTerms* gt) {
  gt->have_p = gt->have_tan = 0;
  if (!packet || !cache.sx) return;
  const int ci = ((j.y >> 2) + row) * cache.cols + (j.x >> 2) + col;
  if (j.model == TANGENTIAL) {
    if (!cache.ta) return;
    gt->have_tan = 1;
    gt->alpha = cache.ta[ci];
    gt->se = cache.tse[ci];
    gt->ce = cache.tce[ci];
  } else if (j.model >= THREE_D_TRANSLATIONAL && j.model <= GEODESIC_CAMPOSE) {
    gt->have_p = 1;
    gt->p = {cache.sx[ci], cache.sy[ci], cache.sz[ci]};
  }
}

struct Geometry {
  int W, H, Wc, Hc;
  int maxCUw, maxCUh, maxCUwc, maxCUhc;
  int bd;
  int chroma;     // 1 = 4:2:0
  int vec_store;  // destination planes allow 8-byte luma / 4-byte chroma row stores
};

struct Taps {
  const int8_t (*luma)[8];
  const int8_t (*chroma)[4];
  const PackedTaps* packed;  // tap pairs of the device interior filter
};

// item containing flat index g: chunk_start[g/64] is the item holding g rounded down to 64
MM_HD int find_item(const int* offsets, const int* chunk_start, int g, int n_items) {
  int j = chunk_start[g >> 6];
  while (j + 1 < n_items && offsets[j + 1] <= g) j++;
  return j;
}

#if defined(__HIP__)
// The same lookup for a whole wavefront whose lanes hold g = g0 + lane (g0 % 64 == 0): one
// uniform chunk_start load, one coalesced load of the next 64 item offsets, and a 6-step binary
// search over them with cross-lane reads -- instead of a chain of dependent loads per lane.
// Items are non-empty, so the offsets relative to g0 are strictly increasing.
__device__ __forceinline__ int wave_find_item(const int* offsets, const int* chunk_start, int g, int n_items) {
  const int lane = __lane_id();
  const int g0 = g - lane;
  const int j0 = __builtin_amdgcn_readfirstlane(chunk_start[g0 >> 6]);
  const int i = j0 + lane;
  int s = 64;
  if (i < n_items) {
    s = offsets[i] - g0;
    s = s < 0 ? 0 : s;
  }
  int lo = 0;
#pragma unroll
  for (int step = 32; step > 0; step >>= 1) {
    const int cand = __shfl(s, lo + step);  // lo + step <= 63
    if (cand <= lane) lo += step;
  }
  return j0 + lo;
}
#endif

// MotionPlaneAdaptiveMotionModel::fillCache on MVReprojection::fillCache's frame grid; storage
// row-major [j][i], Eigen column-major index i*rows + j decides packet vs tail.
MM_HD void mpa_cache_thread(int t, const SeqConst& sc, int plane, int cols, int rows, float* px, float* py,
                            uint8_t* vip) {
  const int n = cols * rows;
  int j = t / cols, i = t % cols;
  int eig = i * rows + j;
  float gx = 4.0f * (float)i + sc.off, gy = 4.0f * (float)j + sc.off;
  float x, y;
  bool v;
  mpa_to_perspective(plane, gx, gy, sc, Math{packet_lane(eig, n)}, &x, &y, &v);
  px[t] = x;
  py[t] = y;
  vip[t] = v ? 1 : 0;
}

#ifndef MM_REPROJ_ROWMAJOR
#define MM_REPROJ_ROWMAJOR 1
#endif
// The reprojection of one element of a device-planned job, stored in k_mc's record layout.
MM_HD void reproj_thread_mc(int g, int ji, const SeqConst& sc, const JobDev* jobs, const int* job_offsets,
                            const BlockSetup* setups, const MpaCache& cache, const McIn& mc) {
  const JobDev& j = jobs[ji];
  // Elements are enumerated row-major over the block (the records k_mc reads and the frame-cache
  // entries are then contiguous across lanes); Eigen's column-major index still decides packet
  // vs tail.  pu_cols = cw / sbw for luma and for 4:2:0 chroma alike.
  const int local = g - job_offsets[ji];
#if MM_REPROJ_ROWMAJOR
  // VVC block widths are powers of two: a shift instead of the ~20-instruction integer division
  const int pc = j.pu_cols;
  int row;
  if ((pc & (pc - 1)) == 0)
    row = local >> __builtin_ctz((unsigned)pc);
  else
    row = local / pc;
  const int col = local - row * pc;
  const int eig = col * j.rows + row;
#else
  const int col = local / j.rows, row = local - col * j.rows;
  const int eig = local;
#endif
  const float gx = (float)(j.x + 4 * col) + sc.off;
  const float gy = (float)(j.y + 4 * row) + sc.off;
  const bool mpa_cached = (j.comp == 0) && (j.model >= MPA_FRONT_BACK && j.model <= MPA_TOP_BOTTOM);
  float px = 0.0f, py = 0.0f;
  bool vip = false;
  if (mpa_cached) {
    const int ci = ((j.y >> 2) + row) * cache.cols + (j.x >> 2) + col;
    const int pl = j.model - MPA_FRONT_BACK;
    px = cache.px[pl][ci];
    py = cache.py[pl][ci];
    vip = cache.vip[pl][ci] != 0;
  }
  const bool packet = packet_lane(eig, j.n);
  GridTerms gt;
  load_grid_terms(cache, j, row, col, packet, &gt);
  int32_t fx, fy;
  reproject_element(sc, setups[ji], gx, gy, packet, mpa_cached, px, py, vip, j.comp ? 1 : 0, &fx, &fy, &gt);
  // chroma 2x2 sub-block (row, col) belongs to luma 4x4 sub-block (row, col) of the same PU
  const int sb = j.sb_base + row * j.pu_cols + col;
  mm_int2 xy;
  xy.x = fx;
  xy.y = fy;
  if (j.comp == 0) {
    mm_int4 r;
    r.x = fx;
    r.y = fy;
    r.z = (j.sb_base << 5) | j.slot;  // reference slot (< 32) and the PU's id (its first sub-block)
    r.w = ((j.y + 4 * row) << 16) | (j.x + 4 * col);
    mc.lum[j.list][sb] = r;
    if (j.alias) mc.chr[j.list][sb] = xy;
  } else {
    mc.chr[j.list][sb] = xy;
  }
}

MM_HD void setup_job(const JobDev& j, const SeqConst& sc, const M3* ged, BlockSetup* out) {
  const int cs = j.comp ? 1 : 0;
  block_setup(out, sc, j.model, j.comp == 0, j.x >> cs, j.y >> cs, j.cw, j.ch, j.mv_hor, j.mv_ver,
              j.ged_idx >= 0 ? &ged[j.ged_idx] : nullptr);
}
MM_HD void setup_thread(int t, const SeqConst& sc, const JobDev* jobs, const M3* ged, BlockSetup* out) {
  setup_job(jobs[t], sc, ged, &out[t]);
}

// ji = the job holding flat element g (find_item / wave_find_item)
MM_HD void reproj_thread(int g, int ji, const SeqConst& sc, const JobDev* jobs, const int* job_offsets,
                         const BlockSetup* setups, const MpaCache& cache, int32_t* out_xy) {
  const JobDev& j = jobs[ji];
  const int local = g - job_offsets[ji];  // enumeration order; results go to j.offset + local
  const int col = local / j.rows, row = local - col * j.rows;
  // grid: luma frame grid (4i + off) or chroma LinSpaced (2*xc + off + 4i) -- the same values
  const float gx = (float)(j.x + 4 * col) + sc.off;
  const float gy = (float)(j.y + 4 * row) + sc.off;
  const bool mpa_cached = (j.comp == 0) && (j.model >= MPA_FRONT_BACK && j.model <= MPA_TOP_BOTTOM);
  float px = 0.0f, py = 0.0f;
  bool vip = false;
  if (mpa_cached) {
    const int ci = ((j.y >> 2) + row) * cache.cols + (j.x >> 2) + col;
    const int pl = j.model - MPA_FRONT_BACK;
    px = cache.px[pl][ci];
    py = cache.py[pl][ci];
    vip = cache.vip[pl][ci] != 0;
  }
  int32_t fx, fy;
  reproject_element(sc, setups[ji], gx, gy, packet_lane(local, j.n), mpa_cached, px, py, vip, j.comp ? 1 : 0, &fx,
                    &fy);
  out_xy[2 * (j.offset + local)] = fx;
  out_xy[2 * (j.offset + local) + 1] = fy;
}

// N output samples of one row: one 8-byte (N = 4) or 4-byte (N = 2) store when the destination
// allows it (Geometry::vec_store), else per-sample stores
template <int N>
MM_HD void store_row(int16_t* d, const int16_t* v, int vec) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (vec) {
    if constexpr (N == 4) {
      typedef uint32_t u32x2_a8 __attribute__((ext_vector_type(2), aligned(8)));
      u32x2_a8 w;
      w.x = ((uint32_t)(uint16_t)v[0]) | ((uint32_t)(uint16_t)v[1] << 16);
      w.y = ((uint32_t)(uint16_t)v[2]) | ((uint32_t)(uint16_t)v[3] << 16);
      *reinterpret_cast<u32x2_a8*>(d) = w;
    } else {
      *reinterpret_cast<uint32_t*>(d) = ((uint32_t)(uint16_t)v[0]) | ((uint32_t)(uint16_t)v[1] << 16);
    }
    return;
  }
#endif
  (void)vec;
  for (int c = 0; c < N; c++) d[c] = v[c];
}

// One luma 4x4 sub-block and its two 4:2:0 chroma 2x2 sub-blocks from the McIn records (device-
// planned pictures); cls = 0 bi, 1 uni L0, 2 uni L1 (sb_class of g's PU bucket).
MM_HD void mc_thread_rec(int g, int cls, const Geometry& geo, const Taps& taps, const McIn& mc, const RefDev* refs,
                         int16_t* dst_y, int dsy, int16_t* dst_cb, int16_t* dst_cr, int dsc) {
  const bool bi = cls == 0;
  const int uni_list = cls == 2 ? 1 : 0;
  const bool used[2] = {bi || uni_list == 0, bi || uni_list == 1};
  mm_int4 L[2];
  mm_int2 C[2];
#pragma unroll
  for (int l = 0; l < 2; l++) {
    if (!used[l]) continue;
    L[l] = mc.lum[l][g];
    if (geo.chroma) C[l] = mc.chr[l][g];
  }
  const int pos = used[0] ? L[0].w : L[1].w;
  const int ox = pos & 0xffff, oy = pos >> 16;
  int16_t pl[2][16];
#pragma unroll
  for (int l = 0; l < 2; l++) {
    if (!used[l]) continue;
    const int32_t fx = L[l].x, fy = L[l].y;
    const int xPos = fx >> 4, yPos = fy >> 4, xFrac = fx & 15, yFrac = fy & 15;
    const RefDev r = refs[L[l].z & 31];
    if (sb_out_of_range(xPos, yPos, geo.W, geo.H, geo.maxCUw, geo.maxCUh, 4, 4)) {
      for (int i = 0; i < 16; i++) pl[l][i] = 0;
    } else if (window_interior<8, 4, 4>(xPos, yPos, geo.W, geo.H)) {
#if defined(__HIP_DEVICE_COMPILE__)
      predict_subblock_interior<8, 4, 4>(r.y, r.stride_y, xPos, yPos, taps.packed->lh[xFrac][(xPos - 3) & 1],
                                         taps.packed->lv[yFrac], bi, geo.bd, pl[l]);
#else
      predict_subblock_interior<8, 4, 4>(r.y, r.stride_y, xPos, yPos, taps.luma[xFrac], taps.luma[yFrac], bi, geo.bd,
                                         pl[l]);
#endif
    } else {
      predict_subblock<8, 4, 4>(r.y, r.stride_y, geo.W, geo.H, xPos, yPos, taps.luma[xFrac], taps.luma[yFrac], bi,
                                geo.bd, pl[l]);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; r++) {
    int16_t o[4];
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const int i = r * 4 + c;
      o[c] = bi ? add_avg(pl[0][i], pl[1][i], geo.bd) : (uni_list == 0 ? pl[0][i] : pl[1][i]);
    }
    store_row<4>(dst_y + (long)(oy + r) * dsy + ox, o, geo.vec_store);
  }
  if (!geo.chroma) return;
  int16_t pcb[2][4], pcr[2][4];
#pragma unroll
  for (int l = 0; l < 2; l++) {
    if (!used[l]) continue;
    const int32_t fx = C[l].x, fy = C[l].y;
    const int xPos = fx >> 5, yPos = fy >> 5, xFrac = fx & 31, yFrac = fy & 31;
    const RefDev r = refs[L[l].z & 31];
    if (sb_out_of_range(xPos, yPos, geo.Wc, geo.Hc, geo.maxCUwc, geo.maxCUhc, 2, 2)) {
      for (int i = 0; i < 4; i++) pcb[l][i] = pcr[l][i] = 0;
    } else if (window_interior<4, 2, 2>(xPos, yPos, geo.Wc, geo.Hc)) {
#if defined(__HIP_DEVICE_COMPILE__)
      const uint32_t* ht = taps.packed->ch[xFrac][(xPos - 1) & 1];
      const uint32_t* vt = taps.packed->cv[yFrac];
      predict_subblock_interior<4, 2, 2>(r.cb, r.stride_c, xPos, yPos, ht, vt, bi, geo.bd, pcb[l]);
      predict_subblock_interior<4, 2, 2>(r.cr, r.stride_c, xPos, yPos, ht, vt, bi, geo.bd, pcr[l]);
#else
      predict_subblock_interior<4, 2, 2>(r.cb, r.stride_c, xPos, yPos, taps.chroma[xFrac], taps.chroma[yFrac], bi,
                                         geo.bd, pcb[l]);
      predict_subblock_interior<4, 2, 2>(r.cr, r.stride_c, xPos, yPos, taps.chroma[xFrac], taps.chroma[yFrac], bi,
                                         geo.bd, pcr[l]);
#endif
    } else {
      predict_subblock<4, 2, 2>(r.cb, r.stride_c, geo.Wc, geo.Hc, xPos, yPos, taps.chroma[xFrac], taps.chroma[yFrac],
                                bi, geo.bd, pcb[l]);
      predict_subblock<4, 2, 2>(r.cr, r.stride_c, geo.Wc, geo.Hc, xPos, yPos, taps.chroma[xFrac], taps.chroma[yFrac],
                                bi, geo.bd, pcr[l]);
    }
  }
  const int cx = ox >> 1, cy = oy >> 1;
#pragma unroll
  for (int r = 0; r < 2; r++) {
    int16_t ob[2], orr[2];
#pragma unroll
    for (int c = 0; c < 2; c++) {
      const int i = r * 2 + c;
      ob[c] = bi ? add_avg(pcb[0][i], pcb[1][i], geo.bd) : (uni_list == 0 ? pcb[0][i] : pcb[1][i]);
      orr[c] = bi ? add_avg(pcr[0][i], pcr[1][i], geo.bd) : (uni_list == 0 ? pcr[0][i] : pcr[1][i]);
    }
    store_row<2>(dst_cb + (long)(cy + r) * dsc + cx, ob, geo.vec_store);
    store_row<2>(dst_cr + (long)(cy + r) * dsc + cx, orr, geo.vec_store);
  }
}

// One luma 4x4 sub-block (and its two 4:2:0 chroma 2x2 sub-blocks) of one PU: both lists,
// xPredInterBlkMM's per-sub-block dispatch (InterPrediction.cpp:776-828), then addAvg (bi) or the
// rndRes uni prediction (xWeightedAverage, InterPrediction.cpp:1584-1679).
// pi = the PU holding luma sub-block g (find_item / wave_find_item)
MM_HD void mc_thread(int g, int pi, const Geometry& geo, const Taps& taps, const PuDev* pus, const JobDev* jobs,
                     const int32_t* reproj, const RefDev* refs, int16_t* dst_y, int dsy, int16_t* dst_cb,
                     int16_t* dst_cr, int dsc) {
  const PuDev pu = pus[pi];
  // lanes walk the PU row-major (horizontally adjacent sub-blocks in adjacent lanes share the
  // reference cache lines of each window row); reprojection results are Eigen column-major
  const int lin = g - pu.sb_offset;
  const int rows = pu.h >> 2, cols = pu.w >> 2;
  const int row = lin / cols, col = lin - row * cols;
  const int local = col * rows + row;
  const bool bi = pu.ref_slot[0] >= 0 && pu.ref_slot[1] >= 0;
  const int uni_list = pu.ref_slot[0] >= 0 ? 0 : 1;

  // ---- luma 4x4 ----
  int16_t pl[2][16];
#pragma unroll
  for (int l = 0; l < 2; l++) {
    if (pu.ref_slot[l] < 0) continue;
    const JobDev& j = jobs[pu.job[l][0]];
    const int32_t fx = reproj[2 * (j.offset + local)], fy = reproj[2 * (j.offset + local) + 1];
    const int xPos = fx >> 4, yPos = fy >> 4, xFrac = fx & 15, yFrac = fy & 15;
    const RefDev r = refs[pu.ref_slot[l]];
    if (sb_out_of_range(xPos, yPos, geo.W, geo.H, geo.maxCUw, geo.maxCUh, 4, 4)) {
      for (int i = 0; i < 16; i++) pl[l][i] = 0;
    } else if (window_interior<8, 4, 4>(xPos, yPos, geo.W, geo.H)) {
#if defined(__HIP_DEVICE_COMPILE__)
      predict_subblock_interior<8, 4, 4>(r.y, r.stride_y, xPos, yPos, taps.packed->lh[xFrac][(xPos - 3) & 1],
                                         taps.packed->lv[yFrac], bi, geo.bd, pl[l]);
#else
      predict_subblock_interior<8, 4, 4>(r.y, r.stride_y, xPos, yPos, taps.luma[xFrac], taps.luma[yFrac], bi, geo.bd,
                                         pl[l]);
#endif
    } else {
      predict_subblock<8, 4, 4>(r.y, r.stride_y, geo.W, geo.H, xPos, yPos, taps.luma[xFrac],
                                taps.luma[yFrac], bi, geo.bd, pl[l]);
    }
  }
  {
    const int ox = pu.x + 4 * col, oy = pu.y + 4 * row;
#pragma unroll
    for (int r = 0; r < 4; r++) {
      int16_t o[4];
#pragma unroll
      for (int c = 0; c < 4; c++) {
        const int i = r * 4 + c;
        o[c] = bi ? add_avg(pl[0][i], pl[1][i], geo.bd) : (uni_list == 0 ? pl[0][i] : pl[1][i]);
      }
      store_row<4>(dst_y + (long)(oy + r) * dsy + ox, o, geo.vec_store);
    }
  }
  if (!geo.chroma) return;
  // ---- chroma 2x2 (Cb and Cr share one reprojection) ----
  int16_t pcb[2][4], pcr[2][4];
#pragma unroll
  for (int l = 0; l < 2; l++) {
    if (pu.ref_slot[l] < 0) continue;
    const JobDev& j = jobs[pu.job[l][1]];
    const int32_t fx = reproj[2 * (j.offset + local)], fy = reproj[2 * (j.offset + local) + 1];
    const int xPos = fx >> 5, yPos = fy >> 5, xFrac = fx & 31, yFrac = fy & 31;
    const RefDev r = refs[pu.ref_slot[l]];
    if (sb_out_of_range(xPos, yPos, geo.Wc, geo.Hc, geo.maxCUwc, geo.maxCUhc, 2, 2)) {
      for (int i = 0; i < 4; i++) pcb[l][i] = pcr[l][i] = 0;
    } else if (window_interior<4, 2, 2>(xPos, yPos, geo.Wc, geo.Hc)) {
#if defined(__HIP_DEVICE_COMPILE__)
      const uint32_t* ht = taps.packed->ch[xFrac][(xPos - 1) & 1];
      const uint32_t* vt = taps.packed->cv[yFrac];
      predict_subblock_interior<4, 2, 2>(r.cb, r.stride_c, xPos, yPos, ht, vt, bi, geo.bd, pcb[l]);
      predict_subblock_interior<4, 2, 2>(r.cr, r.stride_c, xPos, yPos, ht, vt, bi, geo.bd, pcr[l]);
#else
      predict_subblock_interior<4, 2, 2>(r.cb, r.stride_c, xPos, yPos, taps.chroma[xFrac], taps.chroma[yFrac], bi,
                                         geo.bd, pcb[l]);
      predict_subblock_interior<4, 2, 2>(r.cr, r.stride_c, xPos, yPos, taps.chroma[xFrac], taps.chroma[yFrac], bi,
                                         geo.bd, pcr[l]);
#endif
    } else {
      predict_subblock<4, 2, 2>(r.cb, r.stride_c, geo.Wc, geo.Hc, xPos, yPos, taps.chroma[xFrac],
                                taps.chroma[yFrac], bi, geo.bd, pcb[l]);
      predict_subblock<4, 2, 2>(r.cr, r.stride_c, geo.Wc, geo.Hc, xPos, yPos, taps.chroma[xFrac],
                                taps.chroma[yFrac], bi, geo.bd, pcr[l]);
    }
  }
  {
    const int ox = (pu.x >> 1) + 2 * col, oy = (pu.y >> 1) + 2 * row;
#pragma unroll
    for (int r = 0; r < 2; r++) {
      int16_t ob[2], orr[2];
#pragma unroll
      for (int c = 0; c < 2; c++) {
        const int i = r * 2 + c;
        ob[c] = bi ? add_avg(pcb[0][i], pcb[1][i], geo.bd) : (uni_list == 0 ? pcb[0][i] : pcb[1][i]);
        orr[c] = bi ? add_avg(pcr[0][i], pcr[1][i], geo.bd) : (uni_list == 0 ? pcr[0][i] : pcr[1][i]);
      }
      store_row<2>(dst_cb + (long)(oy + r) * dsc + ox, ob, geo.vec_store);
      store_row<2>(dst_cr + (long)(oy + r) * dsc + ox, orr, geo.vec_store);
    }
  }
}

}  // namespace mmpipe
