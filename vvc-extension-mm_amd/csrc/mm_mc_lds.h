// mm_mc_lds.h -- k_mc's device body with quad-staged reference windows (device only).
//
// The arithmetic is mc_thread_rec's (mm_pipeline.h): one lane = one luma 4x4 sub-block and its
// two 4:2:0 chroma 2x2 sub-blocks, both lists, xPredInterBlkMM's per-sub-block dispatch
// (InterPrediction.cpp:776-828) and addAvg / rndRes (Buffer.cpp:551-658).  What changes is how
// the interpolation windows reach the lane:
//
//   * Four consecutive lanes (a "quad": 4 horizontally adjacent sub-blocks of one PU row, or a 2x2
//     group of an 8-wide PU) read overlapping reference windows.  Loaded per lane, every window
//     row costs a 24-byte (luma) / 12-byte (chroma) gather per lane, and the texture-address unit
//     processes such scattered loads one lane-dword at a time.
//   * Instead, each quad loads the union of its four windows as 64-byte rows -- each lane 16
//     contiguous bytes, so one wave instruction reads 16 fully used 64-byte segments -- into an
//     LDS slab owned by the wave, and every lane then reads its own window rows from LDS.
//   * A quad is staged when its four lanes need interior windows of the same reference picture
//     whose union fits 32 samples across and the wave's slab has room; any other lane takes the
//     direct global path (mm_filter.h), so the results never depend on the staging decision.
//
// LDS ordering: the slab is private to one wave and LDS executes a wave's instructions in
// order, so a lane's ds_read after the wave's ds_writes sees them; the asm memory clobbers keep
// the compiler from reordering the slab accesses across the phases.
#pragma once
#include <limits.h>
#include "mm_pipeline.h"

namespace mmlds {
using namespace mmpipe;

constexpr int CELL_DW = 16;  // one staged union row: 32 samples = 64 bytes = 4 lanes x 16 bytes
constexpr int QCELLS = 16;   // rows per quad region: luma 16, or chroma 2 planes x 8
#ifndef MM_MC_QSKEW
#define MM_MC_QSKEW 1  // rotate the quads' regions over the LDS banks
#endif
// Quad region pitch in dwords.  With the skew, quad q's region starts (q & 1) + 8 * ((q >> 1) & 3)
// dwords into its slot, so the 8 quads of a 32-lane LDS group start on 8 different banks (each
// quad's lanes read every other dword).
constexpr int QPITCH = QCELLS * CELL_DW + (MM_MC_QSKEW ? 32 : 0);
constexpr int WAVE_SLAB_DW = 16 * QPITCH;
#ifndef MM_MC_BLOCK
#define MM_MC_BLOCK 256
#endif
constexpr int MC_BLOCK = MM_MC_BLOCK;

#if defined(__HIP_DEVICE_COMPILE__)

// Window rows read from the wave's slab: row r of the window is at base + r * CELL_DW.
struct LdsRows {
  const uint32_t* base;
  template <int ND>
  __device__ __forceinline__ void load(int r, uint32_t* d) const {
#pragma unroll
    for (int k = 0; k < ND; k++) d[k] = base[r * CELL_DW + k];
  }
};

__device__ __forceinline__ void lds_fence() { asm volatile("" ::: "memory"); }

// lane ^ 1 and lane ^ 2 within a quad (DPP quad_perm, no LDS traffic)
__device__ __forceinline__ int quad_xor1(int v) { return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false); }
__device__ __forceinline__ int quad_xor2(int v) { return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false); }
__device__ __forceinline__ int quad_min(int v) {
  v = min(v, quad_xor1(v));
  return min(v, quad_xor2(v));
}
__device__ __forceinline__ int quad_max(int v) {
  v = max(v, quad_xor1(v));
  return max(v, quad_xor2(v));
}

typedef uint32_t u32x4_a16 __attribute__((ext_vector_type(4), aligned(16)));

// Stage the union windows of this lane's quad for NCOMP planes of one reference picture.
//   want : the lane needs an interior window (in range, inside the picture);
//   xs   : even sample at or below the window's first column; y0: window's first row;
//   WIN  : samples read per window row from xs; WR: window rows; RMAX: staged rows per plane;
//   key  : reference slot (a quad stages only windows of one picture).
// Returns whether the lane's windows were staged; row0[c] = the lane's first window row of
// plane c in the slab.  Every lane of the wave must call it (cross-lane operations).  All rows
// are loaded before the first LDS write, so a quad costs one memory round trip.
template <int WIN, int WR, int NCOMP, int RMAX>
__device__ __forceinline__ bool stage_quads(uint32_t* slab, const int16_t* const* planes, int stride, int W, bool want,
                                            int xs, int y0, int key, const uint32_t** row0) {
  static_assert(NCOMP * RMAX <= QCELLS, "quad region");
  const int lane = __lane_id();
  const int k = lane & 3, q = lane >> 2;
  const int xmn = quad_min(want ? xs : INT_MAX), xmx = quad_max(want ? xs : INT_MIN);
  const int ymn = quad_min(want ? y0 : INT_MAX), ymx = quad_max(want ? y0 : INT_MIN);
  const int all = quad_min(want ? 1 : 0);
  const int same = quad_min(key == quad_min(key) ? 1 : 0);
  const int ux = xmn & ~7;  // 16-byte aligned union start
  const int rows = ymx - ymn + WR;
  const bool staged = all && same && xmx + WIN <= ux + 32 && ux + 32 <= W && rows <= RMAX;
  uint32_t* region = slab + q * QPITCH + (MM_MC_QSKEW ? (q & 1) + 8 * ((q >> 1) & 3) : 0);
  u32x4_a16 v[NCOMP][RMAX];
#pragma unroll
  for (int c = 0; c < NCOMP; c++) {
    const int16_t* src = planes[c] + (long)ymn * stride + ux + 8 * k;
#pragma unroll
    for (int r = 0; r < RMAX; r++)
      if (staged && r < rows) v[c][r] = *reinterpret_cast<const u32x4_a16*>(src + (long)r * stride);
  }
  lds_fence();
#pragma unroll
  for (int c = 0; c < NCOMP; c++) {
    uint32_t* dst = region + c * RMAX * CELL_DW + 4 * k;
#pragma unroll
    for (int r = 0; r < RMAX; r++)
      if (staged && r < rows) {
#pragma unroll
        for (int j = 0; j < 4; j++) dst[r * CELL_DW + j] = v[c][r][j];
      }
  }
  lds_fence();
#pragma unroll
  for (int c = 0; c < NCOMP; c++) row0[c] = region + (c * RMAX + (y0 - ymn)) * CELL_DW + ((xs - ux) >> 1);
  return staged;
}

// mc_thread_rec with quad staging.  valid = g < n_sb (lanes past the end still join the
// cross-lane operations); slab = this wave's WAVE_SLAB_DW dwords of LDS.
__device__ __forceinline__ void mc_thread_lds(int g, bool valid, int cls, const Geometry& geo, const Taps& taps,
                                              const McIn& mc, const RefDev* refs, int16_t* dst_y, int dsy,
                                              int16_t* dst_cb, int16_t* dst_cr, int dsc, uint32_t* slab) {
  const PackedTaps& pt = *taps.packed;
  const bool bi = cls == 0;
  const int uni_list = cls == 2 ? 1 : 0;
  const bool used[2] = {valid && (bi || uni_list == 0), valid && (bi || uni_list == 1)};
  mm_int4 L[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
  mm_int2 C[2] = {{0, 0}, {0, 0}};
#pragma unroll
  for (int l = 0; l < 2; l++) {
    if (!used[l]) continue;
    L[l] = mc.lum[l][g];
    if (geo.chroma) C[l] = mc.chr[l][g];
  }
  const int pos = used[0] ? L[0].w : L[1].w;
  const int ox = pos & 0xffff, oy = pos >> 16;

  // ---- luma 4x4, both lists ----
  int16_t pl[2][16];
#pragma unroll
  for (int l = 0; l < 2; l++) {
    if (!__any(used[l])) continue;  // wave-uniform: no lane predicts list l
    const int32_t fx = L[l].x, fy = L[l].y;
    const int xPos = fx >> 4, yPos = fy >> 4, xFrac = fx & 15, yFrac = fy & 15;
    const int slot = L[l].z & 31;
    const RefDev r = refs[slot];
    const bool oor = sb_out_of_range(xPos, yPos, geo.W, geo.H, geo.maxCUw, geo.maxCUh, 4, 4);
    const bool interior = !oor && window_interior<8, 4, 4>(xPos, yPos, geo.W, geo.H);
    const int x0 = xPos - 3;
    const int16_t* planes[1] = {r.y};
    const uint32_t* row0[1];
    const bool staged = stage_quads<12, 11, 1, 16>(slab, planes, r.stride_y, geo.W, used[l] && interior, x0 & ~1, yPos - 3,
                                               slot, row0);
    if (!used[l]) continue;
    const uint32_t* ht = pt.lh[xFrac][x0 & 1];
    const uint32_t* vt = pt.lv[yFrac];
    if (staged) {
      predict_rows<8, 4, 4>(LdsRows{row0[0]}, ht, vt, bi, geo.bd, pl[l]);
    } else if (interior) {
      predict_subblock_interior<8, 4, 4>(r.y, r.stride_y, xPos, yPos, ht, vt, bi, geo.bd, pl[l]);
    } else if (oor) {
#pragma unroll
      for (int i = 0; i < 16; i++) pl[l][i] = 0;
    } else {
      predict_subblock<8, 4, 4>(r.y, r.stride_y, geo.W, geo.H, xPos, yPos, taps.luma[xFrac],
                                taps.luma[yFrac], bi, geo.bd, pl[l]);
    }
  }
  if (valid) {
#pragma unroll
    for (int rr = 0; rr < 4; rr++) {
      int16_t o[4];
#pragma unroll
      for (int c = 0; c < 4; c++) {
        const int i = rr * 4 + c;
        o[c] = bi ? add_avg(pl[0][i], pl[1][i], geo.bd) : (uni_list == 0 ? pl[0][i] : pl[1][i]);
      }
      store_row<4>(dst_y + (long)(oy + rr) * dsy + ox, o, geo.vec_store);
    }
  }
  if (!geo.chroma) return;

  // ---- chroma 2x2 (Cb and Cr share positions), both lists ----
  int16_t pcb[2][4], pcr[2][4];
#pragma unroll
  for (int l = 0; l < 2; l++) {
    if (!__any(used[l])) continue;
    const int32_t fx = C[l].x, fy = C[l].y;
    const int xPos = fx >> 5, yPos = fy >> 5, xFrac = fx & 31, yFrac = fy & 31;
    const int slot = L[l].z & 31;
    const RefDev r = refs[slot];
    const bool oor = sb_out_of_range(xPos, yPos, geo.Wc, geo.Hc, geo.maxCUwc, geo.maxCUhc, 2, 2);
    const bool interior = !oor && window_interior<4, 2, 2>(xPos, yPos, geo.Wc, geo.Hc);
    const int x0 = xPos - 1;
    const int16_t* planes[2] = {r.cb, r.cr};
    const uint32_t* row0[2];
    const bool staged = stage_quads<6, 5, 2, 8>(slab, planes, r.stride_c, geo.Wc, used[l] && interior, x0 & ~1, yPos - 1,
                                             slot, row0);
    if (!used[l]) continue;
    const uint32_t* ht = pt.ch[xFrac][x0 & 1];
    const uint32_t* vt = pt.cv[yFrac];
    if (staged) {
      predict_rows<4, 2, 2>(LdsRows{row0[0]}, ht, vt, bi, geo.bd, pcb[l]);
      predict_rows<4, 2, 2>(LdsRows{row0[1]}, ht, vt, bi, geo.bd, pcr[l]);
    } else if (interior) {
      predict_subblock_interior<4, 2, 2>(r.cb, r.stride_c, xPos, yPos, ht, vt, bi, geo.bd, pcb[l]);
      predict_subblock_interior<4, 2, 2>(r.cr, r.stride_c, xPos, yPos, ht, vt, bi, geo.bd, pcr[l]);
    } else if (oor) {
#pragma unroll
      for (int i = 0; i < 4; i++) pcb[l][i] = pcr[l][i] = 0;
    } else {
      predict_subblock<4, 2, 2>(r.cb, r.stride_c, geo.Wc, geo.Hc, xPos, yPos, taps.chroma[xFrac],
                                taps.chroma[yFrac], bi, geo.bd, pcb[l]);
      predict_subblock<4, 2, 2>(r.cr, r.stride_c, geo.Wc, geo.Hc, xPos, yPos, taps.chroma[xFrac],
                                taps.chroma[yFrac], bi, geo.bd, pcr[l]);
    }
  }
  if (!valid) return;
  const int cx = ox >> 1, cy = oy >> 1;
#pragma unroll
  for (int rr = 0; rr < 2; rr++) {
    int16_t ob[2], orr[2];
#pragma unroll
    for (int c = 0; c < 2; c++) {
      const int i = rr * 2 + c;
      ob[c] = bi ? add_avg(pcb[0][i], pcb[1][i], geo.bd) : (uni_list == 0 ? pcb[0][i] : pcb[1][i]);
      orr[c] = bi ? add_avg(pcr[0][i], pcr[1][i], geo.bd) : (uni_list == 0 ? pcr[0][i] : pcr[1][i]);
    }
    store_row<2>(dst_cb + (long)(cy + rr) * dsc + cx, ob, geo.vec_store);
    store_row<2>(dst_cr + (long)(cy + rr) * dsc + cx, orr, geo.vec_store);
  }
}

#else
// host pass of the kernel translation unit: the kernel body only has to resolve
inline void mc_thread_lds(int, bool, int, const Geometry&, const Taps&, const McIn&, const RefDev*, int16_t*, int,
                          int16_t*, int16_t*, int, uint32_t*) {}
#endif

}  // namespace mmlds
