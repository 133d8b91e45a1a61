// mm_dmvr.h -- MM decoder-side motion vector refinement (host + device bodies).
//
// InterPrediction::xProcessDMVRProjected (CommonLib/InterPrediction.cpp:2442-2634), reached from
// xPredInterBi -> xProcessDMVRMM (:2225-2237) for bi PUs that pass PU::checkDMVRCondition
// (UnitTools.cpp:1698-1726).  Per sub-PU of min(w,16) x min(h,16) luma samples:
//   1. luma 14-bit predictions of both lists at the merge MVs, cost = xDMVRCost (SAD over the even
//      rows, :2147-2155); minCost = cost - cost/4; minCost < dx*dy ends the search (no refinement);
//   2. one iteration over the 25 mirrored integer offsets of m_pSearchOffset (InterPrediction.h:107):
//      L0 at merge0 + off, L1 at merge1 - off, cost per offset, first strict minimum in scan order
//      (the centre entry holds the adjusted minCost);
//   3. parabolic sub-pel refinement from the 5 costs around the best offset unless it lies on the
//      window border (xDMVRSubPixelErrorSurface :2157-2175, xSubPelErrorSrfc :1996-2048);
//   4. the sub-PU is predicted as a bi PU at merge0 + mvd / merge1 - mvd (all components, addAvg).
// Steps 1-3 run here (k_dmvr_setup_dev, k_dmvr_reproj_dev + k_dmvr_sad_dev, k_dmvr_decide_dev) inside the picture's device-planned
// launch sequence: the planner (mm_devplan.h) places every sub-PU of an MM_PUF_DMVR PU as a bi PU
// with its reprojection jobs and a SubPuDev record pointing at them, the search runs on the
// records, and k_dmvr_decide writes the refined MVs into those jobs before k_setup reads them --
// step 4 is then the ordinary setup / reprojection / interpolation of the picture.
#pragma once
#include "../../include/mm360.h"
#include "mm_pipeline.h"

namespace mmdmvr {
using namespace mmpipe;

constexpr int N_OFF = 25;  // (2 * DMVR_NUM_ITERATION + 1)^2, CommonDef.h:365-370

struct SubPuDev {
  int x, y, w, h;      // luma sub-PU
  int mv[2][2];        // merge MVs, 1/16
  int ref_poc[2];
  int slot[2];
  int ged_idx[2];      // GED rotation per list (-1 if not GED)
  int model;           // both lists (checkDMVRCondition: equal models)
  int n, rows;         // luma 4x4 sub-blocks, Eigen rows
  int elem_off;        // first cost element: N_OFF * n per sub-PU
  int jidx[4];         // the sub-PU's reprojection jobs [2 * list + comp] in the picture plan (-1: none)
};

// m_pSearchOffset[i] = (i % 5 - 2, i / 5 - 2)
MM_HD int off_x(int i) { return i % 5 - 2; }
MM_HD int off_y(int i) { return i / 5 - 2; }

// job = (sub-PU s, offset o, list l) -> setups[(s * N_OFF + o) * 2 + l]
MM_HD void dmvr_setup_thread(int t, const SeqConst& sc, const SubPuDev* sp, const M3* ged, BlockSetup* out) {
  const int l = t & 1, so = t >> 1, s = so / N_OFF, o = so - s * N_OFF;
  const SubPuDev& u = sp[s];
  const int sgn = l ? -1 : 1;
  const int mvh = u.mv[l][0] + sgn * (off_x(o) << 4), mvv = u.mv[l][1] + sgn * (off_y(o) << 4);
  block_setup(&out[t], sc, u.model, true, u.x, u.y, u.w, u.h, mvh, mvv, u.ged_idx[l] >= 0 ? &ged[u.ged_idx[l]] : nullptr);
}

// element = (sub-PU, offset, luma 4x4 sub-block) -> the reprojected luma positions of both lists
// (1/16 pel): L0 at merge0 + offset, L1 at merge1 - offset (setups[(s * N_OFF + o) * 2 + l]).
// The search runs as two kernels like the picture path -- this VALU-heavy reprojection (k_reproj's
// footprint), then the window-load-heavy prediction + SAD (k_mc's) -- since one kernel doing both
// needed 163-179 VGPRs (2 waves per SIMD) and ran at half the rate (profiles/r03_ab_dmvr_split.txt).
MM_HD void dmvr_reproj_thread(int g, int si, const SeqConst& sc, const SubPuDev* sp, const BlockSetup* setups,
                              const MpaCache& cache, mm_int2* pos) {
  const SubPuDev& u = sp[si];
  const int local = g - u.elem_off;
  const int o = local / u.n, e = local - o * u.n;
  const int col = e / u.rows, row = e - col * u.rows;
  const float gx = (float)(u.x + 4 * col) + sc.off, gy = (float)(u.y + 4 * row) + sc.off;
  const bool mpa = u.model >= MPA_FRONT_BACK && u.model <= MPA_TOP_BOTTOM;
  float px = 0.0f, py = 0.0f;
  bool vip = false;
  if (mpa) {
    mpa_lookup(cache, u.model, (u.x >> 2) + col, (u.y >> 2) + row, &px, &py, &vip);
  }
  const bool packet = packet_lane(e, u.n);
  const GridSphere pg = grid_point(cache, u.model, (u.x >> 2) + col, (u.y >> 2) + row, packet);
#pragma unroll
  for (int l = 0; l < 2; l++) {
    int32_t fx, fy;
    reproject_element(sc, setups[(si * N_OFF + o) * 2 + l], gx, gy, packet, mpa, px, py, vip, 0, &fx, &fy, pg);
    mm_int2 q;
    q.x = fx;
    q.y = fy;
    pos[2 * (long)g + l] = q;
  }
}

// element g's two 14-bit luma predictions from its positions and its share of xDMVRCost (SAD over
// the even rows of the sub-PU, which are the even rows of each 4x4 sub-block).
// *cost_index = s * N_OFF + o.
MM_HD uint32_t dmvr_sad_thread(int g, int si, const Geometry& geo, const Taps& taps, const SubPuDev* sp,
                               const mm_int2* pos, const RefDev* refs, int* cost_index) {
  const SubPuDev& u = sp[si];
  const int local = g - u.elem_off;
  const int o = local / u.n;
  *cost_index = si * N_OFF + o;
  int16_t p[2][16];
#pragma unroll
  for (int l = 0; l < 2; l++) {
    const mm_int2 q = pos[2 * (long)g + l];
    const int32_t fx = q.x, fy = q.y;
    const int xPos = fx >> 4, yPos = fy >> 4, xFrac = fx & 15, yFrac = fy & 15;
    const RefDev r = refs[u.slot[l]];
    if (sb_out_of_range(xPos, yPos, geo.W, geo.H, geo.maxCUw, geo.maxCUh, 4, 4)) {
      for (int i = 0; i < 16; i++) p[l][i] = 0;
#if defined(__HIP_DEVICE_COMPILE__)
    } else if (geo.padded || window_interior<8, 4, 4>(xPos, yPos, geo.W, geo.H)) {
      // padded pool planes: every in-range window is readable without clamping (as in k_mc)
      predict_subblock_pool<8, 4, 4>(taps.pool, r.off_y, 0, r.stride_y, xPos, yPos, taps.packed->lh[xFrac][(xPos - 3) & 1],
                                     taps.packed->lv[yFrac], true, geo.bd, p[l]);
#else
    } else if (window_interior<8, 4, 4>(xPos, yPos, geo.W, geo.H)) {
      predict_subblock_interior<8, 4, 4>(r.y, r.stride_y, xPos, yPos, taps.luma[xFrac], taps.luma[yFrac], true, geo.bd,
                                         p[l]);
#endif
    } else {
      predict_subblock<8, 4, 4>(r.y, r.stride_y, geo.W, geo.H, xPos, yPos, taps.luma[xFrac], taps.luma[yFrac], true,
                                geo.bd, p[l]);
    }
  }
  uint32_t sum = 0;
#pragma unroll
  for (int rr = 0; rr < 4; rr += 2)
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int d = (int)p[0][rr * 4 + k] - (int)p[1][rr * 4 + k];
      sum += (uint32_t)(d < 0 ? -d : d);
    }
  return sum;
}

// div_for_maxq7 (InterPrediction.cpp:1958-1994)
MM_HD int div_for_maxq7(long long N, long long D) {
  int sign = 0, q = 0;
  if (N < 0) {
    sign = 1;
    N = -N;
  }
  D = D << 3;
  if (N >= D) {
    N -= D;
    q++;
  }
  q = q << 1;
  D = D >> 1;
  if (N >= D) {
    N -= D;
    q++;
  }
  q = q << 1;
  if (N >= (D >> 1)) q++;
  return sign ? -q : q;
}

// xSubPelErrorSrfc (InterPrediction.cpp:1996-2048); sad: centre, left, top, right, bottom
MM_HD void sub_pel_error_surface(const unsigned long long* sad, int* delta) {
  for (int axis = 0; axis < 2; axis++) {
    const unsigned long long a = sad[1 + axis], b = sad[3 + axis];  // (-1, +1) neighbours
    const long long num = (long long)((a - b) << 4);
    const long long den = (long long)(a + b - (sad[0] << 1));
    if (den != 0) {
      if (a != sad[0] && b != sad[0])
        delta[axis] = div_for_maxq7(num, den);
      else
        delta[axis] = (a == sad[0]) ? -8 : 8;
    }
  }
}

MM_HD int clip_mv_storage(int v) {  // Mv::clipToStorageBitDepth, MV_BITS = 18
  const int lo = -(1 << 17), hi = (1 << 17) - 1;
  return v < lo ? lo : (v > hi ? hi : v);
}

// The refinement decision of one sub-PU from its 25 costs: the total L0 delta (1/16 luma)
MM_HD void dmvr_decide(const SubPuDev& u, const uint32_t* c, int* tdx_out, int* tdy_out) {
  unsigned long long sad[N_OFF];
  for (int i = 0; i < N_OFF; i++) sad[i] = c[i];
  int tdx = 0, tdy = 0;  // total delta, 1/16
  unsigned long long minCost = sad[12] - (sad[12] >> 2);
  if (minCost >= (unsigned long long)(u.w * u.h)) {  // else: notZeroCost = false, no refinement
    sad[12] = minCost;
    int best = 12;
    for (int i = 0; i < N_OFF; i++)
      if (sad[i] < minCost) {
        minCost = sad[i];
        best = i;
      }
    tdx = off_x(best) << 4;
    tdy = off_y(best) << 4;
    if (tdx != 32 && tdx != -32 && tdy != 32 && tdy != -32) {
      const unsigned long long sb[5] = {sad[best], sad[best - 1], sad[best - 5], sad[best + 1], sad[best + 5]};
      int d[2] = {0, 0};
      sub_pel_error_surface(sb, d);
      tdx += d[0];
      tdy += d[1];
    }
  }
  *tdx_out = tdx;
  *tdy_out = tdy;
}

// thread per sub-PU: the decision, and the refined MVs (merge0 + delta, merge1 - delta, clipped to
// the MV storage range as pu.mvdL0SubPu is applied) written into the sub-PU's planned jobs, which
// k_setup reads next.  mvd (optional): the delta per sub-PU.
MM_HD void dmvr_decide_jobs_thread(int s, const SubPuDev* sp, const uint32_t* costs, JobDev* jobs, int32_t* mvd) {
  const SubPuDev& u = sp[s];
  int tdx, tdy;
  dmvr_decide(u, costs + (size_t)s * N_OFF, &tdx, &tdy);
  for (int k = 0; k < 4; k++) {
    if (u.jidx[k] < 0) continue;
    const int l = k >> 1, sg = l ? -1 : 1;
    JobDev& j = jobs[u.jidx[k]];
    j.mv_hor = clip_mv_storage(u.mv[l][0] + sg * tdx);
    j.mv_ver = clip_mv_storage(u.mv[l][1] + sg * tdy);
  }
  if (mvd) {
    mvd[2 * s] = tdx;
    mvd[2 * s + 1] = tdy;
  }
}

}  // namespace mmdmvr
