// mm_filter.h -- integer pel pipeline of xPredInterBlkMM for one sub-block, host + device.
//
// Restates InterpolationFilter::filterCopy / filter<N,isVertical,isFirst,isLast>
// (source/Lib/CommonLib/InterpolationFilter.cpp:392-644, public dispatch :675-809;
// constants InterpolationFilter.h:48-53), the per-sub-block dispatch of
// InterPrediction::xPredInterBlkMM (InterPrediction.cpp:776-828) and AreaBuf<Pel>::addAvg
// (Buffer.cpp:551-582).  Reference planes are addressed with coordinate clamping, which is
// identical to the reference's edge-replicated margin (Picture.cpp:988-1048) for every
// position the out-of-range rule lets through (|reach| <= maxCU + 3 < margin 288).
#pragma once
#include <cstddef>
#include <stdint.h>
#include "mm_numerics.h"

namespace mmflt {

// The pool holding every resident reference picture of a context (device address and size).
struct RefPool {
  const char* base;
  uint32_t bytes;
  // every pool slot has the same layout: slot k's luma plane origin is base + k * pic_bytes + y0,
  // the origin of its interleaved chroma plane (one dword Cb | Cr << 16 per chroma position)
  // base + k * pic_bytes + cb0 (device kernels derive RefDev offsets from slot numbers); stride_c
  // counts chroma positions (dwords)
  uint32_t pic_bytes, y0, cb0;
  int stride_y, stride_c;
};

// m_lumaFilter[16][8] (InterpolationFilter.cpp:82-100)
#define MM_LUMA_TAPS_INIT                                                                           \
  {{0, 0, 0, 64, 0, 0, 0, 0},        {0, 1, -3, 63, 4, -2, 1, 0},     {-1, 2, -5, 62, 8, -3, 1, 0},   \
   {-1, 3, -8, 60, 13, -4, 1, 0},    {-1, 4, -10, 58, 17, -5, 1, 0},  {-1, 4, -11, 52, 26, -8, 3, -1}, \
   {-1, 3, -9, 47, 31, -10, 4, -1},  {-1, 4, -11, 45, 34, -10, 4, -1}, {-1, 4, -11, 40, 40, -11, 4, -1}, \
   {-1, 4, -10, 34, 45, -11, 4, -1}, {-1, 4, -10, 31, 47, -9, 3, -1},  {-1, 3, -8, 26, 52, -11, 4, -1}, \
   {0, 1, -5, 17, 58, -10, 4, -1},   {0, 1, -4, 13, 60, -8, 3, -1},    {0, 1, -3, 8, 62, -5, 2, -1},    \
   {0, 1, -2, 4, 63, -3, 1, 0}}
// m_chromaFilter[32][4] (InterpolationFilter.cpp:187-221)
#define MM_CHROMA_TAPS_INIT                                                                         \
  {{0, 64, 0, 0},   {-1, 63, 2, 0},   {-2, 62, 4, 0},   {-2, 60, 7, -1},  {-2, 58, 10, -2},         \
   {-3, 57, 12, -2}, {-4, 56, 14, -2}, {-4, 55, 15, -2}, {-4, 54, 16, -2}, {-5, 53, 18, -2},        \
   {-6, 52, 20, -2}, {-6, 49, 24, -3}, {-6, 46, 28, -4}, {-5, 44, 29, -4}, {-4, 42, 30, -4},        \
   {-4, 39, 33, -4}, {-4, 36, 36, -4}, {-4, 33, 39, -4}, {-4, 30, 42, -4}, {-4, 29, 44, -5},        \
   {-4, 28, 46, -6}, {-3, 24, 49, -6}, {-2, 20, 52, -6}, {-2, 18, 53, -5}, {-2, 16, 54, -4},        \
   {-2, 15, 55, -4}, {-2, 14, 56, -4}, {-2, 12, 57, -3}, {-2, 10, 58, -2}, {-1, 7, 60, -2},         \
   {0, 4, 62, -2},   {0, 2, 63, -1}}

// Tap pairs for v_dot2 (int16 lo | int16 hi << 16), built at compile time from the tables above.
// The device filter reads every window row as dwords from the even sample at or below its first
// sample (4-byte aligned loads: 2-byte aligned dwordx4 loads measured 15-30 % slower in k_mc), so
// dword m holds the aligned sample pair m and a window starting at an odd sample (parity p = 1)
// is one sample into its first dword.  With
//   A = (f0,f1) (f2,f3) ... (0,0)     B = (0,f0) (f1,f2) ... (f_{N-1},0)     C = (0,0) (f0,f1) ...
//   p = 0: even outputs A, odd outputs B;   p = 1: even outputs B, odd outputs C
// applied to the aligned pairs starting at pair (c >> 1), every output is N/2 + 1 dot2 whatever
// the lane's parity (no divergence).  Vertical pass: even output rows A without its zero pair,
// odd rows B, on the H-output row pairs (2m, 2m+1).
struct PackedTaps {
  uint32_t lh[16][2][10];  // luma H  [phase][parity][even 5 | odd 5]
  uint32_t lv[16][9];      // luma V  [phase][even 4 | odd 5]
  uint32_t ch[32][2][6];   // chroma H [phase][parity][even 3 | odd 3]
  uint32_t cv[32][5];      // chroma V [phase][even 2 | odd 3]
};
// The luma members of PackedTaps, which lead the struct: an LDS copy of its first bytes (k_me_sad)
struct PackedLumaTaps {
  uint32_t lh[16][2][10];
  uint32_t lv[16][9];
};
static_assert(sizeof(PackedLumaTaps) % 16 == 0 && offsetof(PackedTaps, lv) == offsetof(PackedLumaTaps, lv),
              "PackedLumaTaps is the leading part of PackedTaps");
constexpr uint32_t tap_pair_(int lo, int hi) { return ((uint32_t)lo & 0xffffu) | ((uint32_t)hi << 16); }
template <int NT>
constexpr void pair_sets_(const int8_t* f, uint32_t* A, uint32_t* B, uint32_t* C) {
  for (int k = 0; k <= NT / 2; k++) {
    A[k] = k < NT / 2 ? tap_pair_(f[2 * k], f[2 * k + 1]) : 0u;
    B[k] = tap_pair_(k > 0 ? f[2 * k - 1] : 0, k < NT / 2 ? f[2 * k] : 0);
    C[k] = k > 0 ? tap_pair_(f[2 * k - 2], f[2 * k - 1]) : 0u;
  }
}
constexpr PackedTaps make_packed_taps() {
  PackedTaps t{};
  const int8_t L[16][8] = MM_LUMA_TAPS_INIT;
  const int8_t Ch[32][4] = MM_CHROMA_TAPS_INIT;
  for (int ph = 0; ph < 16; ph++) {
    uint32_t A[5] = {}, B[5] = {}, C[5] = {};
    pair_sets_<8>(L[ph], A, B, C);
    for (int k = 0; k < 5; k++) {
      t.lh[ph][0][k] = A[k];
      t.lh[ph][0][5 + k] = B[k];
      t.lh[ph][1][k] = B[k];
      t.lh[ph][1][5 + k] = C[k];
    }
    for (int k = 0; k < 4; k++) t.lv[ph][k] = A[k];
    for (int k = 0; k < 5; k++) t.lv[ph][4 + k] = B[k];
  }
  for (int ph = 0; ph < 32; ph++) {
    uint32_t A[3] = {}, B[3] = {}, C[3] = {};
    pair_sets_<4>(Ch[ph], A, B, C);
    for (int k = 0; k < 3; k++) {
      t.ch[ph][0][k] = A[k];
      t.ch[ph][0][3 + k] = B[k];
      t.ch[ph][1][k] = B[k];
      t.ch[ph][1][3 + k] = C[k];
    }
    for (int k = 0; k < 2; k++) t.cv[ph][k] = A[k];
    for (int k = 0; k < 3; k++) t.cv[ph][2 + k] = B[k];
  }
  return t;
}

constexpr int IF_INTERNAL_PREC = 14;
constexpr int IF_FILTER_PREC = 6;
constexpr int IF_INTERNAL_OFFS = 1 << (IF_INTERNAL_PREC - 1);
MM_HD int if_internal_frac_bits(int bd) { return (IF_INTERNAL_PREC - bd) > 2 ? (IF_INTERNAL_PREC - bd) : 2; }

// shift/offset of filter<N, V, isFirst, isLast> (InterpolationFilter.cpp:594-606)
struct FiltParam {
  int shift, offset;
  bool clip;
};
MM_HD FiltParam filt_param(bool isFirst, bool isLast, int bd) {
  int headRoom = if_internal_frac_bits(bd);
  int shift = IF_FILTER_PREC;
  int offset;
  if (isLast) {
    shift += isFirst ? 0 : headRoom;
    offset = 1 << (shift - 1);
    offset += isFirst ? 0 : IF_INTERNAL_OFFS << IF_FILTER_PREC;
  } else {
    shift -= isFirst ? headRoom : 0;
    offset = isFirst ? -IF_INTERNAL_OFFS * (1 << shift) : 0;
  }
  return {shift, offset, isLast};
}

// ClipPel to [0, maxv]; written as max/min so that the device compiler emits one v_med3_i32
MM_HD int16_t clip_pel(int v, int maxv) {
  const int lo = v > 0 ? v : 0;
  return (int16_t)(lo < maxv ? lo : maxv);
}

// Out-of-range rule of xPredInterBlkMM (InterPrediction.cpp:780): sub-block predicts zeros
MM_HD bool sb_out_of_range(int xPos, int yPos, int Wc, int Hc, int maxCUw, int maxCUh, int sbw, int sbh) {
  return xPos < -maxCUw || yPos < -maxCUh || xPos >= Wc + maxCUw - sbw || yPos >= Hc + maxCUh - sbh;
}

MM_HD int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// Every case of xPredInterBlkMM's per-sub-block dispatch (InterPrediction.cpp:785-826) --
// filterCopy (both fractions 0), filterHor only (yFrac == 0), filterVer only (xFrac == 0) and the
// 2-D filterHor(isFirst, !isLast) + filterVer(!isFirst, rndRes) -- yields exactly the 2-D result
// computed with the phase-0 tap row ({.., 64, ..}) for the zero fraction(s): with taps summing to
// 64 and IF_INTERNAL_OFFS = 8192 the extra stage only adds and removes exact multiples of the
// shift (verified for bit depths 8..12 by tests/test_filter_identity.py).  The kernels therefore
// run the branch-free 2-D form for every sub-block (no divergence between the four cases).

// Predict one sub-block (SBW x SBH, NT taps) from a clamped-address reference plane.
//   bi: keep the 14-bit intermediate (rndRes = !bi), else clip to the bit depth.
//   cx, cy: tap rows for xFrac / yFrac.  out: row-major SBW*SBH.
template <int NT, int SBW, int SBH>
MM_HD void predict_subblock(const int16_t* __restrict__ ref, int stride, int Wc, int Hc, int xPos, int yPos,
                            const int8_t* cx, const int8_t* cy, bool bi, int bd, int16_t* out) {
  constexpr int R = SBH + NT - 1, H0 = NT / 2 - 1;
  const int maxv = (1 << bd) - 1;
  const FiltParam fh = filt_param(true, false, bd);
  const FiltParam fv = filt_param(false, !bi, bd);
  int tmp[R][SBW];
#pragma unroll
  for (int r = 0; r < R; r++) {
    const int16_t* row = ref + (long)clampi(yPos + r - H0, 0, Hc - 1) * stride;
#pragma unroll
    for (int c = 0; c < SBW; c++) {
      int sum = 0;
#pragma unroll
      for (int t = 0; t < NT; t++) sum += row[clampi(xPos + c + t - H0, 0, Wc - 1)] * cx[t];
      tmp[r][c] = (int16_t)((sum + fh.offset) >> fh.shift);
    }
  }
#pragma unroll
  for (int r = 0; r < SBH; r++)
#pragma unroll
    for (int c = 0; c < SBW; c++) {
      int sum = 0;
#pragma unroll
      for (int t = 0; t < NT; t++) sum += tmp[r + t][c] * cy[t];
      int v = (int16_t)((sum + fv.offset) >> fv.shift);
      if (fv.clip) v = clip_pel(v, maxv);
      out[r * SBW + c] = (int16_t)v;
    }
}

// Window fully inside the picture (plus one spare sample to the right): the fast path reads
// whole window rows with dword-aligned loads and needs no clamping.
template <int NT, int SBW, int SBH>
MM_HD bool window_interior(int xPos, int yPos, int Wc, int Hc) {
  return xPos - (NT / 2 - 1) >= 0 && xPos + SBW + NT / 2 + 1 <= Wc && yPos - (NT / 2 - 1) >= 0 &&
         yPos + SBH + NT / 2 <= Hc;
}

// Row segment of L = SBW + NT - 1 samples starting at x, read as dwords from the even index
// below x (planes are 4-byte aligned, stride even).
#if defined(__clang__)  // clang vector types (hipcc); the g++ builds of the CPU twin never load them
typedef uint32_t u32x2_a4 __attribute__((ext_vector_type(2), aligned(4)));
typedef uint32_t u32x3_a4 __attribute__((ext_vector_type(3), aligned(4)));
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
#endif

// ND dwords from a 4-byte aligned address as few wide loads as possible (global_load_dwordx4 /
// x3 / x2 only need dword alignment on CDNA)
template <int ND>
MM_HD void load_dwords(const uint32_t* p, uint32_t* d) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (ND == 6) {
    u32x4_a4 a = *reinterpret_cast<const u32x4_a4*>(p);
    u32x2_a4 b = *reinterpret_cast<const u32x2_a4*>(p + 4);
    d[0] = a.x; d[1] = a.y; d[2] = a.z; d[3] = a.w; d[4] = b.x; d[5] = b.y;
  } else if constexpr (ND == 3) {
    u32x3_a4 a = *reinterpret_cast<const u32x3_a4*>(p);
    d[0] = a.x; d[1] = a.y; d[2] = a.z;
  } else {
#pragma unroll
    for (int k = 0; k < ND; k++) d[k] = p[k];
  }
#else
  for (int k = 0; k < ND; k++) d[k] = p[k];
#endif
}

template <int L>
MM_HD void load_row(const int16_t* __restrict__ row, int x, int* v) {
  constexpr int ND = (L + 2) / 2;
  const uint32_t* p = reinterpret_cast<const uint32_t*>(row + (x & ~1));
  uint32_t d[ND];
  load_dwords<ND>(p, d);
  // odd start: funnel-shift the dword stream by one sample (value selects, no indexed array)
  const bool odd = (x & 1) != 0;
#pragma unroll
  for (int m = 0; m < (L + 1) / 2; m++) {
    const uint32_t nxt = (m + 1 < ND) ? (d[m + 1] << 16) : 0u;
    const uint32_t w = odd ? ((d[m] >> 16) | nxt) : d[m];
    v[2 * m] = (int16_t)(w & 0xffffu);
    if (2 * m + 1 < L) v[2 * m + 1] = (int16_t)(w >> 16);
  }
}

#if defined(__HIP_DEVICE_COMPILE__)
typedef short mm_short2 __attribute__((ext_vector_type(2)));
// a.lo*b.lo + a.hi*b.hi + c, exact (v_dot2c_i32_i16; int16 samples x taps, int32 sums)
__device__ __forceinline__ int dot2_(uint32_t a, uint32_t b, int c) {
  return __builtin_amdgcn_sdot2(__builtin_bit_cast(mm_short2, a), __builtin_bit_cast(mm_short2, b), c, false);
}
__device__ __forceinline__ uint32_t pack_lo16_(uint32_t lo, uint32_t hi) {
  return __builtin_amdgcn_perm(hi, lo, 0x05040100u);  // (lo & 0xffff) | (hi << 16), one v_perm_b32
}
// Head of a dot2 accumulation chain with a uniform seed: the VOP3P form takes the seed from an
// SGPR, where the builtin would materialise it with a v_mov for v_dot2c.
__device__ __forceinline__ int dot2_seed_(uint32_t a, uint32_t b, int seed) {
  int r;
  asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(seed));
  return r;
}

// Window rows of a pooled reference plane through a flat pointer: `base` is the dword holding the
// window's first sample; row r is base + r * row_bytes.  (Raw buffer loads with a per-row SGPR
// offset instead of per-row 64-bit VGPR address arithmetic measured slower: k_mc 140 us vs 114 at
// C3)
struct PtrRows {
  const char* base;
  int row_bytes;
  template <int ND>
  __device__ __forceinline__ void load(int r, uint32_t* d) const {
    typedef uint32_t u4 __attribute__((ext_vector_type(4), aligned(4)));
    typedef uint32_t u2 __attribute__((ext_vector_type(2), aligned(4)));
    typedef uint32_t u3 __attribute__((ext_vector_type(3), aligned(4)));
    const char* p = base + (long)r * row_bytes;
#if defined(MM_PROBE_NOLOAD)  // timing probe (wrong results): the window's words without the load
    for (int k = 0; k < ND; k++) d[k] = (uint32_t)(size_t)p + 0x10001u * k;
    return;
#endif
    if constexpr (ND == 6) {
      const u4 a = *reinterpret_cast<const u4*>(p);
      const u2 b = *reinterpret_cast<const u2*>(p + 16);
      d[0] = a.x; d[1] = a.y; d[2] = a.z; d[3] = a.w; d[4] = b.x; d[5] = b.y;
    } else {
      static_assert(ND == 3, "luma (6) or chroma (3) dwords per window row");
      const u3 a = *reinterpret_cast<const u3*>(p);
      d[0] = a.x; d[1] = a.y; d[2] = a.z;
    }
  }
};

// predict_subblock for an interior window (device): the same integer sums, regrouped as packed
// int16 pairs so that each pair of taps is one v_dot2 (PackedTaps): the rounding offsets seed the
// dot2 chains; the H outputs (Pel, 16 bits) are packed as row pairs (one v_perm each) for the
// vertical pass.  ht / vt: the A | B pair sets of this sub-block's phases.
template <int NT, int SBW, int SBH, class Rows>
__device__ __forceinline__ void predict_rows(const Rows& rows, const uint32_t* __restrict__ ht,
                                             const uint32_t* __restrict__ vt, bool bi, int bd, int16_t* out) {
  constexpr int R = SBH + NT - 1;
  constexpr int L = SBW + NT - 1;
  constexpr int ND = (L + 2) / 2;  // dwords loaded per row (L + 1 samples from the even base)
  constexpr int NP = NT / 2;       // tap pairs of an even V output
  constexpr int NQ = NP + 1;       // tap pairs of an H output / odd V output
  constexpr int RP = (R + 1) / 2;  // packed H-output row pairs
  const int maxv = (1 << bd) - 1;
  const FiltParam fh = filt_param(true, false, bd);
  const FiltParam fv = filt_param(false, !bi, bd);
  uint32_t he[NQ], ho[NQ], ve[NP], vo[NQ];
#pragma unroll
  for (int k = 0; k < NQ; k++) {
    he[k] = ht[k];
    ho[k] = ht[NQ + k];
    vo[k] = vt[NP + k];
  }
#pragma unroll
  for (int k = 0; k < NP; k++) ve[k] = vt[k];
#if defined(MM_PROBE_NOFILTER)  // timing probe (wrong results): the window loads without the filter
  {
    uint32_t acc = 0;
#pragma unroll
    for (int r = 0; r < R; r++) {
      uint32_t d[ND];
      rows.template load<ND>(r, d);
#pragma unroll
      for (int k = 0; k < ND; k++) acc ^= d[k];
    }
#pragma unroll
    for (int i = 0; i < SBW * SBH; i++) out[i] = (int16_t)(acc >> (i & 15));
    return;
  }
#endif
  uint32_t tmp[R + 1][SBW];  // H outputs; only the low 16 bits are used
#pragma unroll
  for (int c = 0; c < SBW; c++) tmp[R][c] = 0u;
#pragma unroll
  for (int r = 0; r < R; r++) {
    uint32_t d[ND];
    rows.template load<ND>(r, d);
#pragma unroll
    for (int c = 0; c < SBW; c++) {
      const uint32_t* tp = (c & 1) ? ho : he;
      int sum = dot2_seed_(d[c >> 1], tp[0], fh.offset);
#pragma unroll
      for (int k = 1; k < NQ; k++) sum = dot2_(d[(c >> 1) + k], tp[k], sum);
      tmp[r][c] = (uint32_t)(sum >> fh.shift);
    }
  }
#pragma unroll
  for (int c = 0; c < SBW; c++) {
    uint32_t pr[RP];  // rows (2m, 2m+1)
#pragma unroll
    for (int m = 0; m < RP; m++) pr[m] = pack_lo16_(tmp[2 * m][c], tmp[2 * m + 1][c]);
#pragma unroll
    for (int r = 0; r < SBH; r++) {
      int sum;
      if (r & 1) {
        sum = dot2_seed_(pr[r >> 1], vo[0], fv.offset);
#pragma unroll
        for (int k = 1; k < NQ; k++) sum = dot2_(pr[(r >> 1) + k], vo[k], sum);
      } else {
        sum = dot2_seed_(pr[r >> 1], ve[0], fv.offset);
#pragma unroll
        for (int k = 1; k < NP; k++) sum = dot2_(pr[(r >> 1) + k], ve[k], sum);
      }
      // isLast: ClipPel of the int result (its magnitude is far below 2^15, so the Pel cast
      // the hp path needs is the identity there); callers pass `bi` as a compile-time constant
      // through the inlined chain, so only one of the two forms is emitted
      const int v = sum >> fv.shift;
      out[r * SBW + c] = fv.clip ? clip_pel(v, maxv) : (int16_t)v;
    }
  }
}
// Rows 0 and 2 of a luma 4x4 14-bit (bi) prediction -- all that MM-DMVR's xDMVRCost reads of a sub-block
// (RdCost subShift 1 over the sub-PU: its even rows, InterPrediction.cpp:2147-2155): the H pass over
// window rows 0..9, the V pass for output rows 0 and 2 only; the same integer sums as predict_rows.
// out: row 0 (4 samples), then row 2.
template <class Rows>
__device__ __forceinline__ void predict_rows02(const Rows& rows, const uint32_t* __restrict__ ht,
                                               const uint32_t* __restrict__ vt, int bd, int16_t* out) {
  constexpr int SBW = 4, R = 10, ND = 6, NP = 4, NQ = 5, RP = 5;
  const FiltParam fh = filt_param(true, false, bd);
  const FiltParam fv = filt_param(false, false, bd);
  uint32_t he[NQ], ho[NQ], ve[NP];
#pragma unroll
  for (int k = 0; k < NQ; k++) {
    he[k] = ht[k];
    ho[k] = ht[NQ + k];
  }
#pragma unroll
  for (int k = 0; k < NP; k++) ve[k] = vt[k];
  uint32_t tmp[R][SBW];
#pragma unroll
  for (int r = 0; r < R; r++) {
    uint32_t d[ND];
    rows.template load<ND>(r, d);
#pragma unroll
    for (int c = 0; c < SBW; c++) {
      const uint32_t* tp = (c & 1) ? ho : he;
      int sum = dot2_seed_(d[c >> 1], tp[0], fh.offset);
#pragma unroll
      for (int k = 1; k < NQ; k++) sum = dot2_(d[(c >> 1) + k], tp[k], sum);
      tmp[r][c] = (uint32_t)(sum >> fh.shift);
    }
  }
#pragma unroll
  for (int c = 0; c < SBW; c++) {
    uint32_t pr[RP];
#pragma unroll
    for (int m = 0; m < RP; m++) pr[m] = pack_lo16_(tmp[2 * m][c], tmp[2 * m + 1][c]);
#pragma unroll
    for (int h = 0; h < 2; h++) {  // output rows 0 (pairs 0..3) and 2 (pairs 1..4)
      int sum = dot2_seed_(pr[h], ve[0], fv.offset);
#pragma unroll
      for (int k = 1; k < NP; k++) sum = dot2_(pr[h + k], ve[k], sum);
      out[4 * h + c] = (int16_t)(sum >> fv.shift);
    }
  }
}
// Window rows staged in LDS: row r of the window is `stride` dwords after row r - 1 (dword-aligned
// rows, read as dwords)
struct LdsRows {
  const uint32_t* base;
  int stride;
  template <int ND>
  __device__ __forceinline__ void load(int r, uint32_t* d) const {
    const uint32_t* p = base + r * stride;
#pragma unroll
    for (int k = 0; k < ND; k++) d[k] = p[k];
  }
};

// Interior window of sub-block (xPos, yPos) of a pooled plane whose first sample is at byte
// `plane_off` of the pool (soff: uniform extra offset).
template <int NT, int SBW, int SBH>
__device__ __forceinline__ void predict_subblock_pool(const RefPool& pool, uint32_t plane_off, int soff,
                                                      int stride, int xPos, int yPos, const uint32_t* __restrict__ ht,
                                                      const uint32_t* __restrict__ vt, bool bi, int bd, int16_t* out) {
  constexpr int H0 = NT / 2 - 1;
  const int x0 = (xPos - H0) & ~1;  // even sample at or below the window start: 4-byte aligned rows
  const PtrRows rows{pool.base + plane_off + soff + (long)((yPos - H0) * stride + x0) * 2, stride * 2};
  predict_rows<NT, SBW, SBH>(rows, ht, vt, bi, bd, out);
}

// Both 4:2:0 chroma 2x2 sub-blocks at (xPos, yPos) from the pool's interleaved chroma plane (dword
// Cb | Cr << 16 per position; `plane_off` = byte offset of position (0, 0), `stride` in positions).
// One window of 5 x 5 positions serves Cb and Cr, so a sub-block touches about half the cache lines
// two separate planes cost (one 20-byte row segment instead of two 12-byte ones per window row).
// The integer sums are those of predict_rows<4, 2, 2> on each plane: per window row the sample
// pairs (s0, s1), (s2, s3) of a plane are one v_perm each from the position dwords, the first output
// is A0 . (s0, s1) + A1 . (s2, s3), the second B0 . (s0, s1) + B1 . (s2, s3) + B2 . (s4, *) with
// s4 taken straight from position dword 4 (B2 = (f3, 0) for Cb; (0, f3) for Cr's high half).
// ht: PackedTaps::ch[xFrac][0] (A0 A1 0 | B0 B1 B2), vt: PackedTaps::cv[yFrac].
__device__ __forceinline__ void predict_chroma_pool_il(const RefPool& pool, uint32_t plane_off, int stride, int xPos,
                                                       int yPos, const uint32_t* __restrict__ ht,
                                                       const uint32_t* __restrict__ vt, bool bi, int bd,
                                                       int16_t* ocb, int16_t* ocr) {
  constexpr int R = 5;  // window rows (2 + 4 - 1)
  typedef uint32_t u4 __attribute__((ext_vector_type(4), aligned(4)));
  const int maxv = (1 << bd) - 1;
  const FiltParam fh = filt_param(true, false, bd);
  const FiltParam fv = filt_param(false, !bi, bd);
  const uint32_t a0 = ht[0], a1 = ht[1], b0 = ht[3], b1 = ht[4], b2 = ht[5], b2r = ht[5] << 16;
  const uint32_t ve0 = vt[0], ve1 = vt[1], vo0 = vt[2], vo1 = vt[3], vo2 = vt[4];
  const char* base = pool.base + plane_off + (long)((yPos - 1) * stride + xPos - 1) * 4;
  uint32_t tb[R + 1][2], tr[R + 1][2];  // H outputs (low 16 bits used); row R is the zero pad
  tb[R][0] = tb[R][1] = tr[R][0] = tr[R][1] = 0u;
#pragma unroll
  for (int r = 0; r < R; r++) {
    const char* p = base + (long)r * stride * 4;
    uint32_t d[5];
#if defined(MM_PROBE_NOLOAD)
    for (int k = 0; k < 5; k++) d[k] = (uint32_t)(size_t)p + 0x10001u * k;
#else
    const u4 q = *reinterpret_cast<const u4*>(p);
    d[0] = q.x; d[1] = q.y; d[2] = q.z; d[3] = q.w;
    d[4] = *reinterpret_cast<const uint32_t*>(p + 16);
#endif
    const uint32_t cb01 = __builtin_amdgcn_perm(d[1], d[0], 0x05040100u);
    const uint32_t cb23 = __builtin_amdgcn_perm(d[3], d[2], 0x05040100u);
    const uint32_t cr01 = __builtin_amdgcn_perm(d[1], d[0], 0x07060302u);
    const uint32_t cr23 = __builtin_amdgcn_perm(d[3], d[2], 0x07060302u);
    tb[r][0] = (uint32_t)(dot2_(cb23, a1, dot2_seed_(cb01, a0, fh.offset)) >> fh.shift);
    tb[r][1] = (uint32_t)(dot2_(d[4], b2, dot2_(cb23, b1, dot2_seed_(cb01, b0, fh.offset))) >> fh.shift);
    tr[r][0] = (uint32_t)(dot2_(cr23, a1, dot2_seed_(cr01, a0, fh.offset)) >> fh.shift);
    tr[r][1] = (uint32_t)(dot2_(d[4], b2r, dot2_(cr23, b1, dot2_seed_(cr01, b0, fh.offset))) >> fh.shift);
  }
#pragma unroll
  for (int pl = 0; pl < 2; pl++) {
    uint32_t(*t)[2] = pl ? tr : tb;
    int16_t* out = pl ? ocr : ocb;
#pragma unroll
    for (int c = 0; c < 2; c++) {
      const uint32_t p0 = pack_lo16_(t[0][c], t[1][c]), p1 = pack_lo16_(t[2][c], t[3][c]),
                     p2 = pack_lo16_(t[4][c], t[5][c]);
      const int s0 = dot2_(p1, ve1, dot2_seed_(p0, ve0, fv.offset)) >> fv.shift;
      const int s1 = dot2_(p2, vo2, dot2_(p1, vo1, dot2_seed_(p0, vo0, fv.offset))) >> fv.shift;
      out[c] = fv.clip ? clip_pel(s0, maxv) : (int16_t)s0;
      out[2 + c] = fv.clip ? clip_pel(s1, maxv) : (int16_t)s1;
    }
  }
}
#else
// predict_subblock for an interior window (host): same arithmetic, window rows read with wide loads
template <int NT, int SBW, int SBH>
MM_HD void predict_subblock_interior(const int16_t* __restrict__ ref, int stride, int xPos, int yPos,
                                     const int8_t* cx, const int8_t* cy, bool bi, int bd, int16_t* out) {
  constexpr int L = SBW + NT - 1, R = SBH + NT - 1, H0 = NT / 2 - 1;
  const int maxv = (1 << bd) - 1;
  const FiltParam fh = filt_param(true, false, bd);
  const FiltParam fv = filt_param(false, !bi, bd);
  int tmp[R][SBW];
  for (int r = 0; r < R; r++) {
    int v[L];
    load_row<L>(ref + (long)(yPos + r - H0) * stride, xPos - H0, v);
    for (int c = 0; c < SBW; c++) {
      int sum = 0;
      for (int t = 0; t < NT; t++) sum += v[c + t] * cx[t];
      tmp[r][c] = (int16_t)((sum + fh.offset) >> fh.shift);
    }
  }
  for (int r = 0; r < SBH; r++)
    for (int c = 0; c < SBW; c++) {
      int sum = 0;
      for (int t = 0; t < NT; t++) sum += tmp[r + t][c] * cy[t];
      int v = (int16_t)((sum + fv.offset) >> fv.shift);
      if (fv.clip) v = clip_pel(v, maxv);
      out[r * SBW + c] = (int16_t)v;
    }
}
#endif

// AreaBuf<Pel>::addAvg (Buffer.cpp:551-582): clip((p0 + p1 + offset) >> shiftNum)
MM_HD int16_t add_avg(int p0, int p1, int bd) {
  const int shiftNum = if_internal_frac_bits(bd) + 1;
  const int offset = (1 << (shiftNum - 1)) + 2 * IF_INTERNAL_OFFS;
  return clip_pel((p0 + p1 + offset) >> shiftNum, (1 << bd) - 1);
}

}  // namespace mmflt
