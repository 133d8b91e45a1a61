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
// Steps 1-3 run here inside the picture's device-planned launch sequence (mm_kernels.hip): the
// centre setups and the centre cost of every sub-PU (k_dmvr_setup_dev, k_dmvr_centre_dev; a sub-PU
// whose centre ends the search keeps its merge MVs), then for the surviving sub-PUs only --
// compacted into a list -- the 24 other offsets' setups, positions and the search, all inside one
// wave per survivor (k_dmvr_search_dev): the planner (mm_devplan.h) places every sub-PU of an MM_PUF_DMVR PU as a bi PU
// with its reprojection jobs and a SubPuDev record pointing at them, the search runs on the
// records, and the search writes the refined MVs into those jobs before k_setup reads them --
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

// The block setup of sub-PU u at offset o for list l: reprojectMotionVectorSubblocks of the sub-PU at
// merge0 + offset (L0) / merge1 - offset (L1), InterPrediction.cpp:2510-2515, 2544-2549.
MM_HD void dmvr_setup(const SeqConst& sc, const SubPuDev& u, int o, int l, const M3* ged, BlockSetup* out) {
  const int sgn = l ? -1 : 1;
  const int mvh = u.mv[l][0] + sgn * (off_x(o) << 4), mvv = u.mv[l][1] + sgn * (off_y(o) << 4);
  block_setup(out, sc, u.model, true, u.x, u.y, u.w, u.h, mvh, mvv, u.ged_idx[l] >= 0 ? &ged[u.ged_idx[l]] : nullptr);
}
// The sub-PU's centre terms for list l (mm_models.h centre_terms): what its 25 offsets' setups share
MM_HD void dmvr_centre_terms(const SeqConst& sc, const SubPuDev& u, int l, const M3* ged, CentreTerms* ct) {
  const float cx = (float)u.x + ((float)u.w - 1.0f) / 2.0f, cy = (float)u.y + ((float)u.h - 1.0f) / 2.0f;
  centre_terms(ct, sc, u.model, cx, cy, u.ged_idx[l] >= 0 ? &ged[u.ged_idx[l]] : nullptr);
}
// dmvr_setup from the sub-PU's centre terms: the MV part of the setup only (the same bits)
MM_HD void dmvr_offset_setup(const SeqConst& sc, const SubPuDev& u, int o, int l, const CentreTerms& ct, const M3* ged,
                             BlockSetup* out) {
  const int sgn = l ? -1 : 1;
  const int mvh = u.mv[l][0] + sgn * (off_x(o) << 4), mvv = u.mv[l][1] + sgn * (off_y(o) << 4);
  setup_from_centre(out, sc, u.model, true, mv_to_float(mvh), mv_to_float(mvv), ct,
                    u.ged_idx[l] >= 0 ? &ged[u.ged_idx[l]] : nullptr);
}
// k_dmvr_setup_dev thread t: the centre terms of (sub-PU t / 2, list t % 2) and its centre setup,
// setups[t] (the other offsets' setups are derived from the terms by the search of the survivors)
MM_HD void dmvr_centre_setup_thread(int t, const SeqConst& sc, const SubPuDev* sp, const M3* ged, BlockSetup* out,
                                    CentreTerms* cterms) {
  const SubPuDev& u = sp[t >> 1];
  CentreTerms ct;
  dmvr_centre_terms(sc, u, t & 1, ged, &ct);
  cterms[t] = ct;
  dmvr_offset_setup(sc, u, N_OFF / 2, t & 1, ct, ged, &out[t]);
}

// Luma 4x4 sub-block e (Eigen column-major index over the sub-PU) of one list at offset o: its
// reprojected position (1/16 pel) -- L0 at merge0 + offset, L1 at merge1 - offset, from the
// (sub-PU, offset, list) setup b (reprojectMotionVectorSubblocks of the sub-PU at that MV,
// InterPrediction.cpp:2510-2515, 2544-2549).
MM_HD void dmvr_position(const SeqConst& sc, const SubPuDev& u, const BlockSetup& b, const MpaCache& cache, int e,
                         int32_t* fx, int32_t* fy) {
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
  reproject_element(sc, b, gx, gy, packet, mpa, px, py, vip, 0, fx, fy, pg);
}

// The 24 non-centre offsets (the centre is evaluated first, for every sub-PU): offset index o of
// the k-th non-centre offset.
MM_HD int dmvr_outer_offset(int k) { return k < N_OFF / 2 ? k : k + 1; }

// Luma 4x4 sub-block e of list l at n_offs offsets (the j-th offset's setup: setup_of(j)): its
// reprojected positions (1/16 pel), out(j, fx, fy).  The element's grid terms and the MV-independent head of its
// model (motion_head: TAN's tangent-plane coordinates, GED's rotated spherical coordinates) are
// computed once, the tail per offset: the same operations as dmvr_position per offset.
template <class Setup, class Out>
MM_HD void dmvr_positions_offsets(const SeqConst& sc, const SubPuDev& u, int l, int e, const MpaCache& cache,
                                  Setup setup_of, int n_offs, Out out) {
  const int col = e / u.rows, row = e - col * u.rows;
  const float gx = (float)(u.x + 4 * col) + sc.off, gy = (float)(u.y + 4 * row) + sc.off;
  const bool mpa = u.model >= MPA_FRONT_BACK && u.model <= MPA_TOP_BOTTOM;
  float px = 0.0f, py = 0.0f;
  bool vip = false;
  if (mpa) {
    mpa_lookup(cache, u.model, (u.x >> 2) + col, (u.y >> 2) + row, &px, &py, &vip);
  }
  const bool packet = packet_lane(e, u.n);
  const Math m{packet};
  const GridSphere pg = grid_point(cache, u.model, (u.x >> 2) + col, (u.y >> 2) + row, packet);
  MotionHead h{};
  bool have_head = false;
  for (int j = 0; j < n_offs; j++) {
    const BlockSetup& b = setup_of(j);
    if (!have_head && !b.identity) {  // a zero-MV setup is the identity and carries no TAN terms
      h = motion_head(sc, b, gx, gy, m, pg);
      have_head = true;
    }
    float mx, my;
    motion_tail(sc, b, h, gx, gy, m, mpa, px, py, vip, &mx, &my);
    int32_t fx, fy;
    reproject_finish(sc, gx, gy, mx, my, packet, 0, &fx, &fy);
    out(j, fx, fy);
  }
}

// xDMVRCost's share of one 4x4 sub-block: SAD of its rows 0 and 2 (the sub-PU's even rows, RdCost
// subShift 1) between the two 14-bit predictions p0 / p1, given as those two rows (8 samples each).
MM_HD uint32_t dmvr_sad_rows02(const int16_t* p0, const int16_t* p1) {
  uint32_t sum = 0;
  for (int k = 0; k < 8; k++) {
    const int d = (int)p0[k] - (int)p1[k];
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

// The refinement decision of one sub-PU from its 25 costs: the total L0 delta (1/16 luma).  The costs
// are read in place (c may be LDS); the centre entry stands for the adjusted minCost, as
// pSADsArray[0] does in the reference (:2526).
MM_HD void dmvr_decide(const SubPuDev& u, const uint32_t* c, int* tdx_out, int* tdy_out) {
  int tdx = 0, tdy = 0;  // total delta, 1/16
  const unsigned long long centre = (unsigned long long)c[12] - (c[12] >> 2);
  if (centre >= (unsigned long long)(u.w * u.h)) {  // else: notZeroCost = false, no refinement
    auto sad = [&](int i) -> unsigned long long { return i == 12 ? centre : (unsigned long long)c[i]; };
    unsigned long long minCost = centre;
    int best = 12;
    for (int i = 0; i < N_OFF; i++)
      if (sad(i) < minCost) {
        minCost = sad(i);
        best = i;
      }
    tdx = off_x(best) << 4;
    tdy = off_y(best) << 4;
    if (tdx != 32 && tdx != -32 && tdy != 32 && tdy != -32) {
      const unsigned long long sb[5] = {sad(best), sad(best - 1), sad(best - 5), sad(best + 1), sad(best + 5)};
      int d[2] = {0, 0};
      sub_pel_error_surface(sb, d);
      tdx += d[0];
      tdy += d[1];
    }
  }
  *tdx_out = tdx;
  *tdy_out = tdy;
}

// The refined MVs of sub-PU s (merge0 + delta, merge1 - delta, clipped to the MV storage range as
// pu.mvdL0SubPu is applied, InterPrediction.cpp:2602-2606) written into its planned jobs, which
// k_setup reads next.  mvd (optional): the delta per sub-PU.
MM_HD void dmvr_apply(int s, const SubPuDev& u, int tdx, int tdy, JobDev* jobs, int32_t* mvd) {
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

#if !defined(__HIP_DEVICE_COMPILE__)
// The search of sub-PU s, sequentially (CPU twin): the centre cost, the early exit, the other 24
// offsets, the decision -- the same per-element bodies the device search kernel runs in parallel
// (mm_kernels.hip k_dmvr_search_dev), with the host's clamped-address filter.
inline void dmvr_search_host(int s, const SeqConst& sc, const Geometry& geo, const Taps& taps, const SubPuDev* sp,
                             const M3* ged, const MpaCache& cache, const RefDev* refs, JobDev* jobs, int32_t* mvd) {
  const SubPuDev& u = sp[s];
  BlockSetup setups[N_OFF][2];
  for (int o = 0; o < N_OFF; o++)
    for (int l = 0; l < 2; l++) dmvr_setup(sc, u, o, l, ged, &setups[o][l]);
  uint32_t cost[N_OFF];
  for (int i = 0; i < N_OFF; i++) cost[i] = 0;
  // every offset's positions, as the device computes them (centre: dmvr_position; the 24 others:
  // dmvr_positions_offsets, head once per element)
  int32_t pos[N_OFF][16][2][2];
  for (int e = 0; e < u.n; e++)
    for (int l = 0; l < 2; l++) {
      dmvr_position(sc, u, setups[N_OFF / 2][l], cache, e, &pos[N_OFF / 2][e][l][0], &pos[N_OFF / 2][e][l][1]);
      dmvr_positions_offsets(sc, u, l, e, cache, [&](int j) -> const BlockSetup& { return setups[dmvr_outer_offset(j)][l]; },
                             N_OFF - 1,
                             [&](int j, int32_t fx, int32_t fy) {
                               pos[dmvr_outer_offset(j)][e][l][0] = fx;
                               pos[dmvr_outer_offset(j)][e][l][1] = fy;
                             });
    }
  auto eval = [&](int o) {
    uint32_t sum = 0;
    for (int e = 0; e < u.n; e++) {
      int32_t fx[2], fy[2];
      for (int l = 0; l < 2; l++) {
        fx[l] = pos[o][e][l][0];
        fy[l] = pos[o][e][l][1];
      }
      int16_t p[2][16];
      for (int l = 0; l < 2; l++) {
        const int xPos = fx[l] >> 4, yPos = fy[l] >> 4, xFrac = fx[l] & 15, yFrac = fy[l] & 15;
        const RefDev& r = refs[u.slot[l]];
        if (sb_out_of_range(xPos, yPos, geo.W, geo.H, geo.maxCUw, geo.maxCUh, 4, 4)) {
          for (int i = 0; i < 16; i++) p[l][i] = 0;
        } else {
          predict_subblock<8, 4, 4>(r.y, r.stride_y, geo.W, geo.H, xPos, yPos, taps.luma[xFrac], taps.luma[yFrac], true,
                                    geo.bd, p[l]);
        }
      }
      const int16_t a[8] = {p[0][0], p[0][1], p[0][2], p[0][3], p[0][8], p[0][9], p[0][10], p[0][11]};
      const int16_t b[8] = {p[1][0], p[1][1], p[1][2], p[1][3], p[1][8], p[1][9], p[1][10], p[1][11]};
      sum += dmvr_sad_rows02(a, b);
    }
    return sum;
  };
  cost[12] = eval(12);
  const uint32_t minc = cost[12] - (cost[12] >> 2);
  if (minc >= (uint32_t)(u.w * u.h))  // else the early exit: dmvr_decide reads only the centre
    for (int o = 0; o < N_OFF; o++)
      if (o != 12) cost[o] = eval(o);
  int tdx, tdy;
  dmvr_decide(u, cost, &tdx, &tdy);
  dmvr_apply(s, u, tdx, tdy, jobs, mvd);
}
#endif

}  // namespace mmdmvr
