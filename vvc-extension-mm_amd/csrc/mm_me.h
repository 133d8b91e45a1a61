// mm_me.h -- encoder-side MM motion-estimation candidate evaluation (host + device bodies).
//
// InterSearch::xMVReprojectionInterpolation (EncoderLib/InterSearch.cpp:6277-6385) followed by
// RdCost::xGetSAD (CommonLib/RdCost.cpp:482-517), batched over a window of candidate MVs per
// block: for candidate (i, j) in [-range, range]^2 the block's luma is reprojected with
// mv = centre + (i, j) * step, predicted sub-block by sub-block as a rounded uni prediction
// (rndRes = true; out-of-range margin 0: a sub-block predicts zeros when xPos < 0, yPos < 0,
// xPos >= W - 4 or yPos >= H - 4, InterSearch.cpp:6329-6335) and compared with the original
// picture by SAD (every row, or every other row with sum <<= 1 for subShift 1; FULL_NBIT, so no
// distortion precision shift, TypeDef.h:235-249).
//
// The reference returns a partial SAD once it exceeds the running best
// (maximumDistortionForEarlyExit); such a value only ever loses the comparison, so the search
// decisions equal those made from the full SADs returned here.
#pragma once
#include "mm_pipeline.h"

namespace mmme {
using namespace mmpipe;

// One block of a batch, resolved on the host (reference slot, GED rotation, offsets).
struct MeBlockDev {
  int x, y, w, h;      // luma block
  int mvh, mvv;        // window centre, 1/16 luma
  int model;
  int slot;            // reference slot
  int ged_idx;         // GED rotation table index, -1 if not GED
  int sub_shift;       // 0 or 1
  int n, rows;         // luma 4x4 sub-blocks, Eigen rows (h / 4)
  int elem_off;        // first flat element of this block in the batch (C * n per block)
  int sad_off;         // sads index of candidate 0
};

struct MeWindow {
  int range, step, side, C;  // side = 2 * range + 1, C = side * side
};

// candidate c of the window -> MV offset (row-major over the vertical offset)
MM_HD void me_candidate_mv(const MeWindow& w, const MeBlockDev& b, int c, int* mvh, int* mvv) {
  const int i = c % w.side - w.range, j = c / w.side - w.range;
  *mvh = b.mvh + i * w.step;
  *mvv = b.mvv + j * w.step;
}

// thread per (block, candidate) job: the per-block part of reprojectMotionVectorSubblocks
MM_HD void me_setup_thread(int t, const SeqConst& sc, const MeWindow& w, const MeBlockDev* blocks, const M3* ged,
                           BlockSetup* out) {
  const int bi = t / w.C, c = t - bi * w.C;
  const MeBlockDev& b = blocks[bi];
  int mvh, mvv;
  me_candidate_mv(w, b, c, &mvh, &mvv);
  block_setup(&out[t], sc, b.model, true, b.x, b.y, b.w, b.h, mvh, mvv, b.ged_idx >= 0 ? &ged[b.ged_idx] : nullptr);
}

// thread per (block, candidate, sub-block) element: reprojection, 4x4 luma prediction and its
// SAD contribution.  Returns the (subShift-scaled) SAD of this sub-block and the sads index.
MM_HD uint32_t me_sad_thread(int g, int bi, const SeqConst& sc, const Geometry& geo, const Taps& taps,
                             const MeWindow& w, const MeBlockDev* blocks, const BlockSetup* setups,
                             const MpaCache& cache, const RefDev* refs, const int16_t* org, int org_stride,
                             int* sad_index) {
  const MeBlockDev& b = blocks[bi];
  const int local = g - b.elem_off;
  const int c = local / b.n, e = local - c * b.n;
  *sad_index = b.sad_off + c;
  const BlockSetup& s = setups[bi * w.C + c];
  // Eigen column-major element e of the block's (rows x cols) grid
  const int col = e / b.rows, row = e - col * b.rows;
  const float gx = (float)(b.x + 4 * col) + sc.off, gy = (float)(b.y + 4 * row) + sc.off;
  const bool mpa = b.model >= MPA_FRONT_BACK && b.model <= MPA_TOP_BOTTOM;
  float px = 0.0f, py = 0.0f;
  bool vip = false;
  if (mpa) {
    mpa_lookup(cache, b.model, (b.x >> 2) + col, (b.y >> 2) + row, &px, &py, &vip);
  }
  const bool packet = packet_lane(e, b.n);
  const GridSphere pg = grid_point(cache, b.model, (b.x >> 2) + col, (b.y >> 2) + row, packet);
  int32_t fx, fy;
  reproject_element(sc, s, gx, gy, packet, mpa, px, py, vip, 0, &fx, &fy, pg);
  const int xPos = fx >> 4, yPos = fy >> 4, xFrac = fx & 15, yFrac = fy & 15;
  int16_t p[16];
  if (xPos < 0 || yPos < 0 || xPos >= geo.W - 4 || yPos >= geo.H - 4) {  // maxCUWidth = 0
    for (int i = 0; i < 16; i++) p[i] = 0;
  } else {
    const RefDev r = refs[b.slot];
#if defined(__HIP_DEVICE_COMPILE__)
    if (geo.padded || window_interior<8, 4, 4>(xPos, yPos, geo.W, geo.H)) {
      // padded pool planes: every in-range window is readable without clamping (as in k_mc)
      predict_subblock_pool<8, 4, 4>(taps.pool, r.off_y, 0, r.stride_y, xPos, yPos, taps.packed->lh[xFrac][(xPos - 3) & 1],
                                     taps.packed->lv[yFrac], false, geo.bd, p);
#else
    if (window_interior<8, 4, 4>(xPos, yPos, geo.W, geo.H)) {
      predict_subblock_interior<8, 4, 4>(r.y, r.stride_y, xPos, yPos, taps.luma[xFrac], taps.luma[yFrac], false, geo.bd,
                                         p);
#endif
    } else {
      predict_subblock<8, 4, 4>(r.y, r.stride_y, geo.W, geo.H, xPos, yPos, taps.luma[xFrac], taps.luma[yFrac], false,
                                geo.bd, p);
    }
  }
  // RdCost::xGetSAD over this sub-block's rows of the block (rows 4*row + r; subShift 1 keeps
  // the even block rows, which are the even rows of every sub-block)
  const int16_t* o = org + (long)(b.y + 4 * row) * org_stride + b.x + 4 * col;
  const int rstep = 1 << b.sub_shift;
  uint32_t sum = 0;
  for (int r = 0; r < 4; r += rstep)
    for (int k = 0; k < 4; k++) {
      const int d = (int)o[(long)r * org_stride + k] - (int)p[r * 4 + k];
      sum += (uint32_t)(d < 0 ? -d : d);
    }
  return sum << b.sub_shift;
}

}  // namespace mmme
