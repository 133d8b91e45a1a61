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
  int elem_off;        // first thread of this block in the batch (side * n per block: window row x sub-block)
  int sad_off;         // sads index of candidate 0
};

// The candidates of a block: a (2 range + 1)^2 window of MVs `step` apart (mm_sad_window; k_me_sad
// threads per window row), or a pattern of npat MV offsets shared by every block (mm_sad_pattern: the
// TZ search's 8-point square / diamond, 2-point and star steps and the 9-point refinements,
// InterSearch.cpp:474-526, 6168-6249; one row of npat candidates per block).
constexpr int ME_MAX_PAT = 64;
struct MeWindow {
  int range, step, side, C;  // window: side = 2 * range + 1, C = side * side; pattern: side = C = npat
  int seg16 = 0;             // device: every block of the batch has 16 sub-blocks (k_me_sad's 16-lane sums)
  int npat = 0;              // pattern candidates (0: window)
  // pattern: the staged box's extension beyond the first and last candidates' windows, in samples
  // (the pattern's bounding box relative to those two; 0 for a window, whose extremes they are)
  int box_lx = 0, box_hx = 0, box_ly = 0, box_hy = 0;
  int16_t pat[2 * ME_MAX_PAT] = {};  // pattern offsets (hor, ver), 1/16 luma
};

// candidate c of the window (row-major over the vertical offset) or of the pattern -> its MV
MM_HD void me_candidate_mv(const MeWindow& w, const MeBlockDev& b, int c, int* mvh, int* mvv) {
  if (w.npat) {
    *mvh = b.mvh + w.pat[2 * c];
    *mvv = b.mvv + w.pat[2 * c + 1];
    return;
  }
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

// One luma 4x4 sub-block e of a block against every candidate of one window row j (a thread of
// k_me_sad): what does not depend on the candidate is done once -- the element's grid point, its
// frame-cache / trig-table entries, the model's MV-independent head (mm_models.h motion_head: TAN's
// tangent-plane coordinates about the block centre, GED's rotated spherical coordinates, the sphere
// point of ROT / 3DT) and the original samples the SAD reads -- and per candidate only the model's
// tail, the 8-tap prediction and the SAD (me_cand_sad).  head + tail == model_motion_element, so the
// results are those of a full reprojection per candidate.
struct MeElem {
  float gx, gy, px, py;
  int packet, mpa, vip;
  MotionHead head;
  int col, row;
  int16_t org[16];  // the sub-block's original samples (rows 0..3, or the even rows for subShift 1)
};
// flat thread g of a batch: block bi, window row j, element e (threads of a block: side x n, e fastest)
MM_HD void me_elem_init(int g, int bi, const SeqConst& sc, const MeWindow& w, const MeBlockDev* blocks,
                        const BlockSetup* setups, const MpaCache& cache, const int16_t* org, int org_stride, MeElem* el,
                        int* j_out) {
  const MeBlockDev& b = blocks[bi];
  const int local = g - b.elem_off;
  const int j = local / b.n, e = local - j * b.n;
  *j_out = j;
  // Eigen column-major element e of the block's (rows x cols) grid
  const int col = e / b.rows, row = e - col * b.rows;
  el->col = col;
  el->row = row;
  el->gx = (float)(b.x + 4 * col) + sc.off;
  el->gy = (float)(b.y + 4 * row) + sc.off;
  el->mpa = b.model >= MPA_FRONT_BACK && b.model <= MPA_TOP_BOTTOM;
  float px = 0.0f, py = 0.0f;
  bool vip = false;
  if (el->mpa) mpa_lookup(cache, b.model, (b.x >> 2) + col, (b.y >> 2) + row, &px, &py, &vip);
  el->px = px;
  el->py = py;
  el->vip = vip ? 1 : 0;
  el->packet = packet_lane(e, b.n) ? 1 : 0;
  const GridSphere pg = grid_point(cache, b.model, (b.x >> 2) + col, (b.y >> 2) + row, el->packet != 0);
  // the head needs a setup that is not the zero-MV identity: at most one candidate of the window (or of
  // the pattern, whose offsets are distinct) has a zero MV, so candidate 0 or 1 of the row
  const BlockSetup* s0 = &setups[(long)bi * w.C + (long)j * w.side];
  if (s0->identity && w.side > 1) s0 = s0 + 1;
  el->head = motion_head(sc, *s0, el->gx, el->gy, Math{el->packet != 0}, pg);
  const int16_t* o = org + (long)(b.y + 4 * row) * org_stride + b.x + 4 * col;
  for (int r = 0; r < 4; r++)
    for (int k = 0; k < 4; k++) el->org[r * 4 + k] = o[(long)r * org_stride + k];
}

// The element's reprojected position (1/16 luma) for candidate i of its row j, whose setup is s.
MM_HD void me_cand_pos_s(const MeElem& el, const BlockSetup& s, int i, int j, const SeqConst& sc, int32_t* fx,
                         int32_t* fy) {
  float mx, my;
#if defined(MM_PROBE_ME_NOTAIL)  // timing probe (wrong results): a candidate-dependent position without the model tail
  mx = el.gx + 0.37f * (float)i + s.mvx * 1e-9f;
  my = el.gy + 0.21f * (float)j;
#else
  motion_tail(sc, s, el.head, el.gx, el.gy, Math{el.packet != 0}, el.mpa != 0, el.px, el.py, el.vip != 0, &mx, &my);
#endif
  reproject_finish(sc, el.gx, el.gy, mx, my, el.packet != 0, 0, fx, fy);
}
MM_HD void me_cand_pos(const MeElem& el, int i, int j, int bi, const SeqConst& sc, const MeWindow& w,
                       const BlockSetup* setups, int32_t* fx, int32_t* fy) {
  me_cand_pos_s(el, setups[(long)bi * w.C + (long)j * w.side + i], i, j, sc, fx, fy);
}

// RdCost::xGetSAD over this sub-block's rows of the block (rows 4*row + r; subShift 1 keeps the even
// block rows, which are the even rows of every sub-block), scaled by subShift
MM_HD uint32_t me_sad_of(const MeElem& el, int sub_shift, const int16_t* p) {
  const int rstep = 1 << sub_shift;
  uint32_t sum = 0;
  for (int r = 0; r < 4; r += rstep)
    for (int k = 0; k < 4; k++) {
      const int d = (int)el.org[r * 4 + k] - (int)p[r * 4 + k];
      sum += (uint32_t)(d < 0 ? -d : d);
    }
  return sum << sub_shift;
}

// ME zero rule: a sub-block predicts zeros when its position is out of range (maxCUWidth = 0,
// InterSearch.cpp:6329-6335)
MM_HD bool me_out_of_range(int xPos, int yPos, const Geometry& geo) {
  return xPos < 0 || yPos < 0 || xPos >= geo.W - 4 || yPos >= geo.H - 4;
}

// The (subShift-scaled) SAD of the element's sub-block for candidate i of its row j.
MM_HD uint32_t me_cand_sad(const MeElem& el, int i, int j, int bi, const SeqConst& sc, const Geometry& geo,
                           const Taps& taps, const MeWindow& w, const MeBlockDev* blocks, const BlockSetup* setups,
                           const RefDev* refs) {
  const MeBlockDev& b = blocks[bi];
  int32_t fx, fy;
  me_cand_pos(el, i, j, bi, sc, w, setups, &fx, &fy);
  const int xPos = fx >> 4, yPos = fy >> 4, xFrac = fx & 15, yFrac = fy & 15;
  int16_t p[16];
#if defined(MM_PROBE_ME_NOFILTER)  // timing probe (wrong results): the position without the prediction
  for (int k = 0; k < 16; k++) p[k] = (int16_t)(xPos + k * yPos + xFrac * yFrac);
  if (false) {
#else
  if (me_out_of_range(xPos, yPos, geo)) {
#endif
    for (int k = 0; k < 16; k++) p[k] = 0;
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
  return me_sad_of(el, b.sub_shift, p);
}

#if defined(__HIP_DEVICE_COMPILE__)
// A reference window staged in a wave's LDS (k_me_sad): luma samples [x0, x1) x rows [y0, y1) of the
// wave's reference, x0 even, row r at lds + (r - y0) * stride dwords.
struct MeWin {
  const uint32_t* lds;
  int stride, x0, y0, x1, y1;
};
// me_cand_sad with the window rows read from the staged window when `use` and the candidate's window
// lies inside it; otherwise from the pool as me_cand_sad does (same integer sums either way).  The
// candidate's setup `s` and the luma tap pairs come from the caller (LDS in k_me_sad).
__device__ __forceinline__ uint32_t me_cand_sad_win(const MeElem& el, const BlockSetup& s, int i, int j,
                                                    const SeqConst& sc, const Geometry& geo, const RefPool& pool,
                                                    const PackedLumaTaps* lt, const RefDev& r, int sub_shift,
                                                    const MeWin& win, bool use) {
  int32_t fx, fy;
  me_cand_pos_s(el, s, i, j, sc, &fx, &fy);
  const int xPos = fx >> 4, yPos = fy >> 4, xFrac = fx & 15, yFrac = fy & 15;
  int16_t p[16];
  if (me_out_of_range(xPos, yPos, geo)) {
    for (int k = 0; k < 16; k++) p[k] = 0;
  } else {
    const uint32_t* ht = lt->lh[xFrac][(xPos - 3) & 1];
    const uint32_t* vt = lt->lv[yFrac];
    const int xw = (xPos - 3) & ~1;  // the window's dword-aligned rows: 12 samples from xw, rows yPos - 3 .. yPos + 7
    if (use && xw >= win.x0 && xw + 12 <= win.x1 && yPos - 3 >= win.y0 && yPos + 8 <= win.y1) {
      const LdsRows rows{win.lds + (yPos - 3 - win.y0) * win.stride + ((xw - win.x0) >> 1), win.stride};
      predict_rows<8, 4, 4>(rows, ht, vt, false, geo.bd, p);
    } else {
      predict_subblock_pool<8, 4, 4>(pool, r.off_y, 0, r.stride_y, xPos, yPos, ht, vt, false, geo.bd, p);
    }
  }
  return me_sad_of(el, sub_shift, p);
}
#endif

}  // namespace mmme
