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
#include <stdint.h>
#include "mm_numerics.h"

namespace mmflt {

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

MM_HD int16_t clip_pel(int v, int maxv) { return (int16_t)(v < 0 ? 0 : (v > maxv ? maxv : v)); }

// Out-of-range rule of xPredInterBlkMM (InterPrediction.cpp:780): sub-block predicts zeros
MM_HD bool sb_out_of_range(int xPos, int yPos, int Wc, int Hc, int maxCUw, int maxCUh, int sbw, int sbh) {
  return xPos < -maxCUw || yPos < -maxCUh || xPos >= Wc + maxCUw - sbw || yPos >= Hc + maxCUh - sbh;
}

MM_HD int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// Predict one sub-block (sbw x sbh, NT taps) from a clamped-address reference plane.
//   bi: keep 14-bit intermediate (rndRes = !bi), else clip to bit depth.
//   coef: tap row for xFrac / yFrac.  out: row-major sbw*sbh.
template <int NT, int SBW, int SBH>
MM_HD void predict_subblock(const int16_t* __restrict__ ref, int stride, int Wc, int Hc, int xPos, int yPos,
                            int xFrac, int yFrac, const int8_t* cx, const int8_t* cy, bool bi, int bd,
                            int16_t* out) {
  const int maxv = (1 << bd) - 1;
  const bool rndRes = !bi;
  if (yFrac == 0) {
    // filterHor(xFrac, isLast = rndRes) -> filterCopy[true][rndRes] or filter<NT,false,true,rndRes>
    for (int r = 0; r < SBH; r++) {
      const int16_t* row = ref + (long)clampi(yPos + r, 0, Hc - 1) * stride;
      for (int c = 0; c < SBW; c++) {
        int v;
        if (xFrac == 0) {
          int s = row[clampi(xPos + c, 0, Wc - 1)];
          if (rndRes)
            v = s;  // isFirst == isLast: plain copy
          else
            v = (int16_t)((int16_t)(s << if_internal_frac_bits(bd)) - (int16_t)IF_INTERNAL_OFFS);
        } else {
          FiltParam fp = filt_param(true, rndRes, bd);
          int sum = 0;
          for (int t = 0; t < NT; t++) sum += row[clampi(xPos + c + t - (NT / 2 - 1), 0, Wc - 1)] * cx[t];
          v = (int16_t)((sum + fp.offset) >> fp.shift);
          if (fp.clip) v = clip_pel(v, maxv);
        }
        out[r * SBW + c] = (int16_t)v;
      }
    }
    return;
  }
  if (xFrac == 0) {
    // filterVer(yFrac, isFirst = true, isLast = rndRes)
    FiltParam fp = filt_param(true, rndRes, bd);
    for (int r = 0; r < SBH; r++)
      for (int c = 0; c < SBW; c++) {
        const int xx = clampi(xPos + c, 0, Wc - 1);
        int sum = 0;
        for (int t = 0; t < NT; t++) sum += ref[(long)clampi(yPos + r + t - (NT / 2 - 1), 0, Hc - 1) * stride + xx] * cy[t];
        int v = (int16_t)((sum + fp.offset) >> fp.shift);
        if (fp.clip) v = clip_pel(v, maxv);
        out[r * SBW + c] = (int16_t)v;
      }
    return;
  }
  // 2-D: filterHor on (SBH + NT - 1) rows into tmp (isFirst, !isLast), then filterVer (!isFirst, rndRes)
  int16_t tmp[(SBH + NT - 1) * SBW];
  FiltParam fh = filt_param(true, false, bd);
  for (int r = 0; r < SBH + NT - 1; r++) {
    const int16_t* row = ref + (long)clampi(yPos + r - (NT / 2 - 1), 0, Hc - 1) * stride;
    for (int c = 0; c < SBW; c++) {
      int sum = 0;
      for (int t = 0; t < NT; t++) sum += row[clampi(xPos + c + t - (NT / 2 - 1), 0, Wc - 1)] * cx[t];
      tmp[r * SBW + c] = (int16_t)((sum + fh.offset) >> fh.shift);
    }
  }
  FiltParam fv = filt_param(false, rndRes, bd);
  for (int r = 0; r < SBH; r++)
    for (int c = 0; c < SBW; c++) {
      int sum = 0;
      for (int t = 0; t < NT; t++) sum += tmp[(r + t) * SBW + c] * cy[t];
      int v = (int16_t)((sum + fv.offset) >> fv.shift);
      if (fv.clip) v = clip_pel(v, maxv);
      out[r * SBW + c] = (int16_t)v;
    }
}

// AreaBuf<Pel>::addAvg (Buffer.cpp:551-582): clip((p0 + p1 + offset) >> shiftNum)
MM_HD int16_t add_avg(int p0, int p1, int bd) {
  const int shiftNum = if_internal_frac_bits(bd) + 1;
  const int offset = (1 << (shiftNum - 1)) + 2 * IF_INTERNAL_OFFS;
  return clip_pel((p0 + p1 + offset) >> shiftNum, (1 << bd) - 1);
}

}  // namespace mmflt
