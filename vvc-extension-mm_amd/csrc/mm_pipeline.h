// mm_pipeline.h -- work descriptors and per-thread bodies of the MC pipeline (host + device).
//
// The HIP kernels in mm_kernels.hip are one-line wrappers around these bodies; the CPU twin
// used by the CPU test suite (tests/native/host_twin.cpp) loops over the same bodies, so the
// device logic is exercised bit-for-bit on the host before it ever reaches a GPU.
#pragma once
#include <cstddef>
#include "mm_filter.h"
#include "mm_models.h"
#include "mm_probe.h"

namespace mmpipe {
using namespace mmmod;
using namespace mmflt;

struct RefDev {
  const int16_t* y;
  const int16_t* cb;
  const int16_t* cr;
  int stride_y, stride_c;
  uint32_t off_y, off_cb;  // byte offsets of the Y and interleaved chroma planes in the context's RefPool
};

// One reprojection job == one reprojectMotionVectorSubblocks call
// 32 bytes, 16-byte aligned: written and read as two 16-byte words (k_plan_place, k_setup*,
// k_reproj*).  The scattered record stores are a third of k_plan_place's time, so the fields are
// as narrow as their ranges allow: positions < 2^15 (mm_create limits pictures to 16384 samples),
// block sizes <= 128, <= 1024 elements, models < 16, GED table index < 19.
struct alignas(16) JobDev {
  int16_t x, y;        // block position in LUMA units (grid origin)
  uint8_t cw, ch;      // block size in component units
  uint8_t rows;        // ch/sbh (Eigen column-major rows)
  uint8_t pu_cols;     // device plan: sub-block columns of the PU (cw / sbw)
  int32_t mv_hor, mv_ver;
  int32_t offset;      // first element in the result array
  // device-planned prediction: where k_mc finds this job's results (McRec, one record per luma
  // 4x4 sub-block of the PU from sb_base)
  int32_t sb_base;
  uint16_t n;          // elements = (cw/sbw)*(ch/sbh)
  int8_t model;
  uint8_t comp : 1;    // 0 luma, 1 chroma (4:2:0)
  uint8_t list : 1;
  uint8_t alias : 1;   // MPA chroma == luma, fill both records
  uint8_t slot : 4;
  int32_t meta_hi : 24;  // McRec meta word .y of the PU (slots, BCW) | MM_META_PRIMARY if this job writes it
  int32_t ged_idx : 8;   // index into the GED rotation table (-1 if not GED)
};
static_assert(sizeof(JobDev) == 32, "JobDev is two 16-byte words");

struct alignas(16) mm_int4 {
  int x, y, z, w;
};
struct alignas(8) mm_int2 {
  int x, y;
};
// Per-luma-sub-block inputs of k_mc, written by the reprojection of a device-planned picture in
// the order k_mc reads them (sub-block g of the enumeration):
//   meta[g]    = (ox | oy << 16, slot0 | slot1 << 4 | bcw << 8 | use0 << 12 | use1 << 13 | pic << 14):
//                output position of the luma 4x4 sub-block, reference slot per list, BCW index, the
//                lists the sub-block uses, the picture of a multi-picture call -- written by the PU's
//                primary job;
//   lpos[l][g] = the list-l luma position in 1/16 pel relative to the sub-block origin
//                (16 ox, 16 oy), as two int16 (x lo, y hi) -- written by the luma job;
//   cpos[l][g] = the 4:2:0 chroma position in 1/32 pel relative to (32 (ox / 2), 32 (oy / 2)),
//                likewise -- written by the chroma job, or by the aliasing MPA luma job.
// A relative position that does not fit 16 bits (a wrap across the ERP seam, motion of more than
// 2047 samples) is stored as MM_POS_FAR and its absolute (x, y) in far[l][comp][g], which only those
// sub-blocks touch.  So a bi sub-block is 24 bytes (8 + 4 x 4), each array written by one job kind
// in whole lines, against 40 bytes of interleaved luma / chroma halves before (round 2).
struct McRec {
  mm_int2* meta;
  uint32_t* lpos[2];
  uint32_t* cpos[2];
  mm_int2* far[2][2];  // [list][comp]
};
#define MM_POS_FAR 0x8000u  // low half of a relative position word: look up far[][][]

// A position relative to base as one word, or MM_POS_FAR
MM_HD uint32_t pack_rel(int32_t fx, int32_t fy, int32_t bx, int32_t by) {
  const long dx = (long)fx - bx, dy = (long)fy - by;
  if (dx < -32767 || dx > 32767 || dy < -32768 || dy > 32767) return MM_POS_FAR;
  return ((uint32_t)(uint16_t)(int16_t)dx) | ((uint32_t)(uint16_t)(int16_t)dy << 16);
}
#define MM_META_PRIMARY (1 << 16)
#define MM_META_USE0 (1 << 12)
#define MM_META_USE1 (1 << 13)
#define MM_META_SEG_SHIFT 14  // bits 14-15: the picture of a multi-picture call (mm_pred_device_multi)
#ifndef MM_MAX_PICS
#define MM_MAX_PICS 4  // include/mm360.h
#endif

// The destination planes of a call's pictures (device pointers; picture q of mm_pred_device_multi,
// q = 0 for a single picture), picked by the sub-block's picture index with selects.
struct DstPlanes {
  int16_t* y[MM_MAX_PICS];
  int16_t* cb[MM_MAX_PICS];
  int16_t* cr[MM_MAX_PICS];
  int sy[MM_MAX_PICS], sc[MM_MAX_PICS];
};

// w1 = g_BcwWeights[bcw] (Rom.cpp:203 {-2, 3, 4, 5, 10}) as nibbles of w1 + 2; w0 = 8 - w1
MM_HD int bcw_w1(int bcw) { return (int)((0xC7650u >> (4 * bcw)) & 15u) - 2; }

// MVReprojection::fillCache's frame grid, MPA perspective coordinates per plane
// (MotionPlaneAdaptiveMotionModel::fillCache), row-major [j][i] over the (W/4) x (H/4) grid
// x = 4i + off, y = 4j + off.
//
// trig_col / trig_row (optional, may be null): EquirectangularProjection::toSphere on the same grid
// is separable (Projection.cpp:213-228 -> Coordinate.cpp:57-59): phi depends only on the grid column
// i, theta only on the grid row j, and sphericalToCartesian with R = 1 is
// (sin th cos ph, sin th sin ph, cos th).  One (sin, cos) pair per column and per row, in both
// flavours an element can need (Eigen packet psin/pcos, v = 1; glibc scalar sinf/cosf, v = 0), gives
// every grid element's sphere point bit-identically -- the same functions of the same arguments,
// computed once per sequence instead of twice per element (the north star's shared spherical trig).
// Layout: trig_col[(v * cols + i) * 2 + {0: sin, 1: cos}] of phi, trig_row likewise of theta.
// px / py / vip hold the three MPA planes back to back (plane pl at pl * cols * rows): the plane is
// picked by address arithmetic, never by indexing a pointer array with a per-lane model (which
// would copy the kernel-argument struct to scratch memory).
// tan_grid (optional, may be null): TAN's first step per grid point and flavour (mm_models.h
// GridSphere), [packet][gj][gi], built by k_tan_grid when TANGENTIAL is active.
struct alignas(16) TanEntry {
  float alpha, se, ce, pad;
};
struct MpaCache {
  const float* px;
  const float* py;
  const uint8_t* vip;
  int cols, rows;  // W/4, H/4
  const float* trig_col;
  const float* trig_row;
  const TanEntry* tan_grid;
};

// One entry of the separable toSphere table (t over 2 * cols column entries, then 2 * rows rows)
MM_HD void erp_trig_thread(int t, const SeqConst& sc, int cols, int rows, float* col, float* row) {
  if (t < 2 * cols) {
    const int v = t >= cols ? 1 : 0, i = t - v * cols;
    const float ph = erp_phi(4.0f * (float)i + sc.off, sc);
    const Math m{v};
    col[2 * t] = m.sin(ph);
    col[2 * t + 1] = m.cos(ph);
    return;
  }
  t -= 2 * cols;
  if (t >= 2 * rows) return;
  const int v = t >= rows ? 1 : 0, j = t - v * rows;
  const float th = erp_theta(4.0f * (float)j + sc.off, sc);
  const Math m{v};
  row[2 * t] = m.sin(th);
  row[2 * t + 1] = m.cos(th);
}

// toSphere of frame-grid element (column gi, row gj) from the table
MM_HD V3 grid_sphere(const MpaCache& c, int gi, int gj, bool packet) {
  const int v = packet ? 1 : 0;
  const float* pc = c.trig_col + 2 * (v * c.cols + gi);
  const float* pr = c.trig_row + 2 * (v * c.rows + gj);
  return sph_from_trig(pr[0], pr[1], pc[0], pc[1]);
}
MM_HD bool is_mpa_model(int m) { return m >= MPA_FRONT_BACK && m <= MPA_TOP_BOTTOM; }

// The frame-cache entry of an MPA model at grid (gi, gj)
MM_HD void mpa_lookup(const MpaCache& c, int model, int gi, int gj, float* px, float* py, bool* vip) {
  const long k = (long)(model - MPA_FRONT_BACK) * c.cols * c.rows + (long)gj * c.cols + gi;
  *px = c.px[k];
  *py = c.py[k];
  *vip = c.vip[k] != 0;
}
// What a non-MPA element needs of its grid point from the tables, when they exist: TAN's first
// step from tan_grid, the other models' sphere point from the trig table
MM_HD GridSphere grid_point(const MpaCache& c, int model, int gi, int gj, bool packet) {
  GridSphere g = no_grid();
  if (is_mpa_model(model)) return g;
  if (model == TANGENTIAL && c.tan_grid) {
    const TanEntry e = c.tan_grid[(packet ? (long)c.cols * c.rows : 0L) + (long)gj * c.cols + gi];
    g.tan_valid = 1;
    g.alpha = e.alpha;
    g.se = e.se;
    g.ce = e.ce;
    return g;
  }
  if (!c.trig_col) return g;
  g.p = grid_sphere(c, gi, gj, packet);
  g.valid = 1;
  return g;
}
// One entry of tan_grid (t over 2 * cols * rows: flavour, row, column)
MM_HD void tan_grid_thread(long t, const SeqConst& sc, const MpaCache& c, TanEntry* out) {
  const long n = (long)c.cols * c.rows;
  if (t >= 2 * n) return;
  const bool packet = t >= n;
  const long k = t - (packet ? n : 0);
  const int gj = (int)(k / c.cols), gi = (int)(k - (long)gj * c.cols);
  TanEntry e;
  tan_grid_entry(grid_sphere(c, gi, gj, packet), Math{packet}, &e.alpha, &e.se, &e.ce);
  e.pad = 0.0f;
  out[t] = e;
}

struct Geometry {
  int W, H, Wc, Hc;
  int maxCUw, maxCUh, maxCUwc, maxCUhc;
  int bd;
  int chroma;     // 1 = 4:2:0
  int vec_store;  // destination planes allow 8-byte luma / 4-byte chroma row stores
  int hp;         // mm_pred_list hp: every list keeps the 14-bit intermediate (bi = true)
  int store;      // components written: bit 0 luma, bit 1 chroma
  int padded;     // device: the reference planes carry edge-replicated margins wide enough for every
                  // in-range window (mm_kernels.hip place_ref), so no window needs clamped reads
};

struct Taps {
  const int8_t (*luma)[8];
  const int8_t (*chroma)[4];
  const PackedTaps* packed;  // tap pairs of the device interior filter
  RefPool pool;              // the reference pool the device interior filter reads through
};

// item containing flat index g: chunk_start[g/64] is the item holding g rounded down to 64
MM_HD int find_item(const int* offsets, const int* chunk_start, int g, int n_items) {
  int j = chunk_start[g >> 6];
  while (j + 1 < n_items && offsets[j + 1] <= g) j++;
  return j;
}

#if defined(__HIP__)
// Tables that a kernel indexes per lane (the GED rotations, the reference table) are copied from
// the kernel arguments into LDS by the first threads of the workgroup; every caller then
// synchronises the workgroup (__syncthreads) before any thread reads `lds`.  The round-4 MM-DMVR
// search faulted because its threads read a staged reference table before that barrier
// (profiles/r04_kernarg_fault.txt, correction); DESIGN.md 4.6 audits every staging kernel and the
// MM_RACE_PROBE build (mm_probe.h) checks them.  Round 4's replacement -- scalar loads of the words
// with a per-lane select -- measured equal for k_mc and 1-3 us slower for k_setup_dev
// (profiles/r05_ab_staging_and_mc_split.txt), so the plain per-lane copy stays.
template <int NW>
__device__ __forceinline__ void stage_arg_words(const uint32_t* arg, uint32_t* lds) {
  for (int k = threadIdx.x; k < NW; k += blockDim.x) lds_put(lds[k], arg[k], 0x7fc00000u);  // poison: NaN
}
// The device fields of a picture's reference table (RefDev stride_y, stride_c, off_y, off_cb; the
// host plane pointers are not used on the device) for NS slots, from the packed pool-slot numbers
// and the pool's uniform layout (lanes 0..NS-1).
template <int NS>
__device__ __forceinline__ void stage_ref_table(const uint32_t* pool_slot4, const RefPool& pool, RefDev* lds) {
  static_assert(NS % 4 == 0 && NS <= 64, "four slots per packed word");
  if (threadIdx.x >= NS) return;
  const int lane = threadIdx.x;
  const uint32_t ps = (pool_slot4[lane >> 2] >> (8 * (lane & 3))) & 255u;
  RefDev& r = lds[lane];
  r.stride_y = pool.stride_y;
  r.stride_c = pool.stride_c;
  // probe poison: the pool's last picture slot (inside the pool, the wrong picture)
  const uint32_t last = pool.bytes - pool.pic_bytes;
  lds_put(r.off_y, ps * pool.pic_bytes + pool.y0, last + pool.y0);
  lds_put(r.off_cb, ps * pool.pic_bytes + pool.cb0, last + pool.cb0);
}

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

// The reprojection of one element of a device-planned job, stored in k_mc's record layout.
#ifndef MM_REPROJ_BYVAL
#define MM_REPROJ_BYVAL 1  // k_reproj_dev copies its job record and setup by value (loads issued together)
#endif
MM_HD void reproj_thread_mc(int g, int ji, const SeqConst& sc, const JobDev* jobs, const int* job_offsets,
                            const BlockSetup& setup, const MpaCache& cache, const McRec& mc) {
#if MM_REPROJ_BYVAL
  const JobDev j = jobs[ji];
#else
  const JobDev& j = jobs[ji];
#endif
  // Elements are enumerated row-major over the block (the records k_mc reads and the frame-cache
  // entries are then contiguous across lanes); Eigen's column-major index still decides packet
  // vs tail.  pu_cols = cw / sbw for luma and for 4:2:0 chroma alike.
  const int local = g - job_offsets[ji];
  // VVC block widths are powers of two: a shift instead of the ~20-instruction integer division
  const int pc = j.pu_cols;
  int row;
  if ((pc & (pc - 1)) == 0)
    row = local >> __builtin_ctz((unsigned)pc);
  else
    row = local / pc;
  const int col = local - row * pc;
  const int eig = col * j.rows + row;
  const float gx = (float)(j.x + 4 * col) + sc.off;
  const float gy = (float)(j.y + 4 * row) + sc.off;
  const bool mpa_cached = (j.comp == 0) && (j.model >= MPA_FRONT_BACK && j.model <= MPA_TOP_BOTTOM);
  float px = 0.0f, py = 0.0f;
  bool vip = false;
  if (mpa_cached) {
    mpa_lookup(cache, j.model, (j.x >> 2) + col, (j.y >> 2) + row, &px, &py, &vip);
  }
  const bool packet = packet_lane(eig, j.n);
  const GridSphere pg = grid_point(cache, j.model, (j.x >> 2) + col, (j.y >> 2) + row, packet);
  int32_t fx, fy;
  reproject_element(sc, setup, gx, gy, packet, mpa_cached, px, py, vip, j.comp ? 1 : 0, &fx, &fy, pg);
  // chroma 2x2 sub-block (row, col) belongs to luma 4x4 sub-block (row, col) of the same PU
  const int sb = j.sb_base + row * j.pu_cols + col;
  const int ox = j.x + 4 * col, oy = j.y + 4 * row;  // luma sub-block origin; 32 (ox / 2) == 16 ox
  const uint32_t rel = pack_rel(fx, fy, 16 * ox, 16 * oy);
  mm_int2 xy;
  xy.x = fx;
  xy.y = fy;
  // the list's arrays by selects: indexing the kernel-argument arrays with j.list would copy the
  // whole McRec into a per-lane private array (promoted to 72 B of LDS per lane)
  const bool l1 = j.list != 0;
  uint32_t* const lpos = l1 ? mc.lpos[1] : mc.lpos[0];
  uint32_t* const cpos = l1 ? mc.cpos[1] : mc.cpos[0];
  mm_int2* const lfar = l1 ? mc.far[1][0] : mc.far[0][0];
  mm_int2* const cfar = l1 ? mc.far[1][1] : mc.far[0][1];
  if (j.comp == 0) {
    lpos[sb] = rel;
    if (rel == MM_POS_FAR) lfar[sb] = xy;
    if (j.alias) {  // MPA chroma == luma (mm_devplan.h mpa_chroma_aliases)
      cpos[sb] = rel;
      if (rel == MM_POS_FAR) cfar[sb] = xy;
    }
    if (j.meta_hi & MM_META_PRIMARY) {
      mm_int2 m;
      m.x = (oy << 16) | ox;
      m.y = j.meta_hi & 0xffff;
      mc.meta[sb] = m;
    }
  } else {
    cpos[sb] = rel;
    if (rel == MM_POS_FAR) cfar[sb] = xy;
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
    mpa_lookup(cache, j.model, (j.x >> 2) + col, (j.y >> 2) + row, &px, &py, &vip);
  }
  const bool packet = packet_lane(local, j.n);
  const GridSphere pg = grid_point(cache, j.model, (j.x >> 2) + col, (j.y >> 2) + row, packet);
  int32_t fx, fy;
  reproject_element(sc, setups[ji], gx, gy, packet, mpa_cached, px, py, vip, j.comp ? 1 : 0, &fx, &fy, pg);
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

// AreaBuf<Pel>::addWeightedAvg (Buffer.cpp:398-424): clip((p0 w0 + p1 w1 + offset) >> shiftNum),
// shiftNum = IF_INTERNAL_FRAC_BITS + 3, offset = (1 << (shiftNum - 1)) + (IF_INTERNAL_OFFS << 3).
// With BCW_DEFAULT (w0 = w1 = 4) numerator and shift are exactly 4x those of AreaBuf<Pel>::addAvg
// (Buffer.cpp:551-582), so this one form is xWeightedAverage's bi output for every bcwIdx
// (InterPrediction.cpp:1596-1600); tests/test_filter_identity.py checks the identity.
MM_HD int16_t weighted_avg(int p0, int p1, int w0, int w1, int bd) {
  const int shiftNum = if_internal_frac_bits(bd) + 3;
  const int offset = (1 << (shiftNum - 1)) + (IF_INTERNAL_OFFS << 3);
  return clip_pel((p0 * w0 + p1 * w1 + offset) >> shiftNum, (1 << bd) - 1);
}

// One luma 4x4 sub-block and its two 4:2:0 chroma 2x2 sub-blocks from the McRec records (device-
// planned pictures): for each list the sub-block uses, xPredInterBlkMM's per-sub-block dispatch
// (InterPrediction.cpp:776-828) at the 14-bit intermediate (bi = true), then xWeightedAverage
// (InterPrediction.cpp:1584-1679): addAvg / addWeightedAvg of the two lists for bi, and for uni the
// rndRes prediction -- which equals weighted_avg(p, *, 8, 0) of the list's 14-bit prediction p
// exactly (both are floor((p + 2^(h-1) + 2^13) / 2^h) clipped, h = IF_INTERNAL_FRAC_BITS: the uni
// V pass's offset is a multiple of 2^6, so its single shift equals the 14-bit shift followed by
// this one; tests/test_filter_identity.py).  So bi and uni sub-blocks share one body and a wave may
// hold both (k_mc's waves follow the picture's spatial order, not PU classes); a list no lane of
// the wave uses is skipped as a whole.  A sub-block whose window lies out of range is zero in the
// reference at the precision the list is predicted at (InterPrediction.cpp:780-783): the 14-bit
// intermediate for bi and HP, the final samples for uni -- so a uni one is filled with
// -IF_INTERNAL_OFFS, which weighted_avg(., *, 8, 0) maps to 0 (tests/test_twin.py).
// HP (mm_pred_list hp = 1): every sub-block uses one list and keeps its 14-bit prediction.
// The 24 bytes of one sub-block's record, loaded by mc_rec_load (the positions of both lists
// unconditionally: the arrays are zeroed at allocation, and a wave of the class-agnostic
// enumeration mixes bi and uni sub-blocks, so it loads both lists anyway).  k_mc_dev loads the next
// iteration's record before predicting the current one.
struct McIn {
  mm_int2 meta;
  uint32_t lp[2], cp[2];
};
MM_HD McIn mc_rec_load(const McRec& mc, int g) {
  McIn r;
  r.meta = mc.meta[g];
#pragma unroll
  for (int l = 0; l < 2; l++) {
    r.lp[l] = mc.lpos[l][g];
    r.cp[l] = mc.cpos[l][g];
  }
  return r;
}

template <bool HP>
MM_HD void mc_rec_impl(int g, const McIn& in, const Geometry& geo, const Taps& taps, const McRec& mc,
                       const RefDev* refs, const DstPlanes& dst) {
  const mm_int2 meta = in.meta;
  // the picture's planes: `dst` is an LDS copy on the device (k_mc_dev), so a per-lane index reads LDS
  // at the store, and no plane pointer is held in registers through the filter
  const int pic = (meta.y >> MM_META_SEG_SHIFT) & (MM_MAX_PICS - 1);
  const bool used[2] = {(meta.y & MM_META_USE0) != 0, (meta.y & MM_META_USE1) != 0};
  const int ox = meta.x & 0xffff, oy = meta.x >> 16;
  mm_int4 P[2];  // (luma x, y in 1/16 pel, chroma x, y in 1/32 pel) per list
#pragma unroll
  for (int l = 0; l < 2; l++) {
    if (!used[l]) continue;
    const uint32_t lp = in.lp[l], cp = in.cp[l];
    P[l].x = 16 * ox + (int16_t)(lp & 0xffffu);
    P[l].y = 16 * oy + (int16_t)(lp >> 16);
    P[l].z = 16 * ox + (int16_t)(cp & 0xffffu);
    P[l].w = 16 * oy + (int16_t)(cp >> 16);
    if (lp == MM_POS_FAR) {
      const mm_int2 f = mc.far[l][0][g];
      P[l].x = f.x;
      P[l].y = f.y;
    }
    if (cp == MM_POS_FAR) {
      const mm_int2 f = mc.far[l][1][g];
      P[l].z = f.x;
      P[l].w = f.y;
    }
  }
  const int slot[2] = {meta.y & 15, (meta.y >> 4) & 15};
  const bool bi = used[0] && used[1];
  // bi: (w0, w1) of the BCW index; uni: the list's prediction with weight 8 (see above)
  const int w1b = bcw_w1((meta.y >> 8) & 7);
  const int wa = bi ? 8 - w1b : 8, wb = bi ? w1b : 0;
  const int16_t oor = (HP || bi) ? 0 : (int16_t)-IF_INTERNAL_OFFS;  // out-of-range fill (see above)
  if (geo.store & 1) {
    int16_t pl[2][16];
#pragma unroll
    for (int l = 0; l < 2; l++) {
      for (int i = 0; i < 16; i++) pl[l][i] = 0;
      if (!used[l]) continue;
      const int32_t fx = P[l].x, fy = P[l].y;
      const int xPos = fx >> 4, yPos = fy >> 4, xFrac = fx & 15, yFrac = fy & 15;
      const RefDev r = refs[slot[l]];
      if (sb_out_of_range(xPos, yPos, geo.W, geo.H, geo.maxCUw, geo.maxCUh, 4, 4)) {
        for (int i = 0; i < 16; i++) pl[l][i] = oor;
#if defined(__HIP_DEVICE_COMPILE__)
      } else if (geo.padded || window_interior<8, 4, 4>(xPos, yPos, geo.W, geo.H)) {
        predict_subblock_pool<8, 4, 4>(taps.pool, r.off_y, 0, r.stride_y, xPos, yPos, taps.packed->lh[xFrac][(xPos - 3) & 1],
                                       taps.packed->lv[yFrac], true, geo.bd, pl[l]);
#else
      } else if (window_interior<8, 4, 4>(xPos, yPos, geo.W, geo.H)) {
        predict_subblock_interior<8, 4, 4>(r.y, r.stride_y, xPos, yPos, taps.luma[xFrac], taps.luma[yFrac], true,
                                           geo.bd, pl[l]);
#endif
      } else {
        predict_subblock<8, 4, 4>(r.y, r.stride_y, geo.W, geo.H, xPos, yPos, taps.luma[xFrac], taps.luma[yFrac], true,
                                  geo.bd, pl[l]);
      }
    }
    const int pa = used[0] ? 0 : 1;  // uni L1: the list-1 prediction takes the first weight
#pragma unroll
    for (int r = 0; r < 4; r++) {
      int16_t o[4];
#pragma unroll
      for (int c = 0; c < 4; c++) {
        const int i = r * 4 + c;
        const int a = pa ? pl[1][i] : pl[0][i];
        o[c] = HP ? (int16_t)a : weighted_avg(a, pl[1][i], wa, wb, geo.bd);
      }
      store_row<4>(dst.y[pic] + (long)(oy + r) * dst.sy[pic] + ox, o, geo.vec_store);
    }
  }
  if (!geo.chroma || !(geo.store & 2)) return;
  int16_t pcb[2][4], pcr[2][4];
#pragma unroll
  for (int l = 0; l < 2; l++) {
    for (int i = 0; i < 4; i++) pcb[l][i] = pcr[l][i] = 0;
    if (!used[l]) continue;
    const int32_t fx = P[l].z, fy = P[l].w;
    const int xPos = fx >> 5, yPos = fy >> 5, xFrac = fx & 31, yFrac = fy & 31;
    const RefDev r = refs[slot[l]];
    if (sb_out_of_range(xPos, yPos, geo.Wc, geo.Hc, geo.maxCUwc, geo.maxCUhc, 2, 2)) {
      for (int i = 0; i < 4; i++) pcb[l][i] = pcr[l][i] = oor;
#if defined(__HIP_DEVICE_COMPILE__)
    } else {  // device contexts always hold padded pool planes (geo.padded), chroma interleaved
      predict_chroma_pool_il(taps.pool, r.off_cb, r.stride_c, xPos, yPos, taps.packed->ch[xFrac][0],
                             taps.packed->cv[yFrac], true, geo.bd, pcb[l], pcr[l]);
    }
#else
    } else if (window_interior<4, 2, 2>(xPos, yPos, geo.Wc, geo.Hc)) {
      predict_subblock_interior<4, 2, 2>(r.cb, r.stride_c, xPos, yPos, taps.chroma[xFrac], taps.chroma[yFrac], true,
                                         geo.bd, pcb[l]);
      predict_subblock_interior<4, 2, 2>(r.cr, r.stride_c, xPos, yPos, taps.chroma[xFrac], taps.chroma[yFrac], true,
                                         geo.bd, pcr[l]);
    } else {
      predict_subblock<4, 2, 2>(r.cb, r.stride_c, geo.Wc, geo.Hc, xPos, yPos, taps.chroma[xFrac], taps.chroma[yFrac],
                                true, geo.bd, pcb[l]);
      predict_subblock<4, 2, 2>(r.cr, r.stride_c, geo.Wc, geo.Hc, xPos, yPos, taps.chroma[xFrac], taps.chroma[yFrac],
                                true, geo.bd, pcr[l]);
    }
#endif
  }
  const int pa = used[0] ? 0 : 1;
  const int cx = ox >> 1, cy = oy >> 1;
#pragma unroll
  for (int r = 0; r < 2; r++) {
    int16_t ob[2], orr[2];
#pragma unroll
    for (int c = 0; c < 2; c++) {
      const int i = r * 2 + c;
      const int ab = pa ? pcb[1][i] : pcb[0][i], ar = pa ? pcr[1][i] : pcr[0][i];
      ob[c] = HP ? (int16_t)ab : weighted_avg(ab, pcb[1][i], wa, wb, geo.bd);
      orr[c] = HP ? (int16_t)ar : weighted_avg(ar, pcr[1][i], wa, wb, geo.bd);
    }
    store_row<2>(dst.cb[pic] + (long)(cy + r) * dst.sc[pic] + cx, ob, geo.vec_store);
    store_row<2>(dst.cr[pic] + (long)(cy + r) * dst.sc[pic] + cx, orr, geo.vec_store);
  }
}

// UNI_HP: mm_pred_list with hp = 1 (every sub-block is uni and keeps the 14-bit intermediate);
// a separate kernel instance, so the picture path's register allocation does not carry it.
template <bool UNI_HP = false>
MM_HD void mc_thread_rec(int g, const Geometry& geo, const Taps& taps, const McRec& mc, const RefDev* refs,
                         const DstPlanes& dst) {
  mc_rec_impl<UNI_HP>(g, mc_rec_load(mc, g), geo, taps, mc, refs, dst);
}
template <bool UNI_HP = false>
MM_HD void mc_thread_in(int g, const McIn& in, const Geometry& geo, const Taps& taps, const McRec& mc,
                        const RefDev* refs, const DstPlanes& dst) {
  mc_rec_impl<UNI_HP>(g, in, geo, taps, mc, refs, dst);
}

}  // namespace mmpipe
