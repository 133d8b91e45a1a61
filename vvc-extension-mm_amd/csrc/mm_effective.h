// mm_effective.h -- the effective blocks of a decoded PU's motion compensation (host C++).
//
// Restates the control flow of InterPrediction::motionCompensation (SRC/InterPrediction.cpp:
// 1681-1810) down to the calls that reach xPredInterBlkMM, for MM PUs:
//   * BDOF pre-check (:1736-1775, motion model NOT considered) on a bi PU wider or taller than
//     MAX_BDOF_APPLICATION_REGION (16) without DMVR -> xSubPuBio (:361-453): min(16, w) x
//     min(16, h) sub-PUs, each motion-compensated on its own (the reprojection block centre is
//     the sub-PU's);
//   * SbTMVP (mergeType != MRG_TYPE_DEFAULT_N) -> xSubPuMC (:283-359): runs of identical
//     MotionInfo (MotionInfo.h:196-219: interDir, refIdx, mv, motionModel) on the 8x8 sub-block
//     grid are merged into strips along the longer PU side, unless a reference is scaled;
//   * xCheckIdenticalMotion (:248-281): a bi PU whose lists point at the same reference POC with
//     the same MV (the motion model is not compared) is predicted from list 0 alone;
//   * DMVR (pu.mvRefine && PU::checkDMVRCondition, UnitTools.cpp:1698-1726) -> xPredInterBi's
//     xProcessDMVRProjected, i.e. the mm_pred_dmvr list.
// SRC = source/Lib/CommonLib.  SbTMVP sub-block motion identifies references by POC (refIdx ->
// POC is one-to-one in the caller's lists).
#pragma once
#include <cstdint>
#include <cstdlib>
#include <vector>

#include "../../include/mm360.h"

namespace mmeff {

constexpr int MAX_BDOF_APPLICATION_REGION = 16;  // CommonDef.h:191
constexpr int ATMVP_SUB_BLOCK_SIZE = 3;          // CommonDef.h:420 (8x8)

inline bool is_bi(const mm_pu_desc& d) { return d.ref_poc[0] >= 0 && d.ref_poc[1] >= 0; }

// PU::isBiPredFromDifferentDirEqDistPoc (UnitTools.cpp:4466-4487)
inline bool bi_diff_dir_eq_dist(const mm_pu_desc& d, int cur_poc, uint32_t flags) {
  if (!is_bi(d) || (flags & MM_PU_LONGTERM)) return false;
  const int d0 = cur_poc - d.ref_poc[0], d1 = cur_poc - d.ref_poc[1];
  return (long)d0 * d1 < 0 && std::abs(d0) == std::abs(d1);
}

// MotionInfo::operator== (MotionInfo.h:196-219) on the fields an MM PU carries
inline bool same_motion(const mm_pu_desc& a, const mm_pu_desc& b) {
  for (int l = 0; l < 2; l++) {
    if ((a.ref_poc[l] >= 0) != (b.ref_poc[l] >= 0)) return false;  // interDir
    if (a.ref_poc[l] < 0) continue;
    if (a.ref_poc[l] != b.ref_poc[l] || a.mv[l][0] != b.mv[l][0] || a.mv[l][1] != b.mv[l][1] ||
        a.model[l] != b.model[l])
      return false;
  }
  return true;
}

class Deriver {
 public:
  Deriver(const mm_tool_flags& t, std::vector<mm_pu_desc>* mc, std::vector<mm_pu_desc>* dmvr)
      : t_(t), mc_(mc), dmvr_(dmvr) {}

  // motionCompensation(pu, predBuf, REF_PIC_LIST_X) of one decoded PU
  int run(const mm_pu_motion& m, const mm_pu_desc* sub) {
    const mm_pu_desc& d = m.pu;
    if (d.w < 4 || d.h < 4 || (d.w & 3) || (d.h & 3) || (d.ref_poc[0] < 0 && d.ref_poc[1] < 0)) return MM_ERR_ARG;
    if (is_bi(d) && d.w + d.h == 12) return MM_ERR_ARG;  // "invalid 4x8/8x4 bi-predicted blocks" (:1722)
    if (m.flags & MM_PU_SUBPU) {
      if (!sub || m.sub_motion < 0) return MM_ERR_ARG;
      return sub_pu_mc(m, sub + m.sub_motion);
    }
    return motion_compensation(d, m.flags, m.cur_poc, false);
  }

 private:
  // motionCompensation body for a PU with uniform motion; sub_pu_mc: called from xSubPuMC
  int motion_compensation(const mm_pu_desc& d, uint32_t flags, int cur_poc, bool sub_pu_mc) {
    bool bio = false;
    if (t_.bdof && !sub_pu_mc) {  // :1736-1775
      bio = !(flags & MM_PU_WEIGHTED) && bi_diff_dir_eq_dist(d, cur_poc, flags) && d.h >= 8 && d.w >= 8 &&
            d.h * d.w >= 128;
      if (flags & MM_PU_CIIP) bio = false;
      if (flags & MM_PU_SMVD) bio = false;
      if (t_.bcw && d.bcw_idx != MM_BCW_DEFAULT) bio = false;
      if (flags & MM_PU_MMVD_ENC2) bio = false;
    }
    if (flags & MM_PU_REF_SCALED) bio = false;
    const bool dmvr = !sub_pu_mc && (flags & MM_PU_MVREFINE) && check_dmvr(d, flags, cur_poc);
    if ((d.w > MAX_BDOF_APPLICATION_REGION || d.h > MAX_BDOF_APPLICATION_REGION) && bio && !dmvr) {
      // xSubPuBio (:361-453): every sub-PU runs motionCompensation with the PU's flags; it is
      // at most 16x16, so it does not split again
      const int sw = d.w < MAX_BDOF_APPLICATION_REGION ? d.w : MAX_BDOF_APPLICATION_REGION;
      const int sh = d.h < MAX_BDOF_APPLICATION_REGION ? d.h : MAX_BDOF_APPLICATION_REGION;
      for (int y = d.y; y < d.y + d.h; y += sh)
        for (int x = d.x; x < d.x + d.w; x += sw) {
          mm_pu_desc s = d;
          s.x = x;
          s.y = y;
          s.w = sw;
          s.h = sh;
          const int rc = motion_compensation(s, flags, cur_poc, false);
          if (rc) return rc;
        }
      return MM_OK;
    }
    leaf(d, dmvr);
    return MM_OK;
  }

  // PU::checkDMVRCondition (UnitTools.cpp:1698-1726)
  bool check_dmvr(const mm_pu_desc& d, uint32_t flags, int cur_poc) const {
    if (!t_.dmvr) return false;
    return (flags & MM_PU_MERGE) && !(flags & MM_PU_CIIP) && !(flags & MM_PU_MMVD) && d.model[0] == d.model[1] &&
           bi_diff_dir_eq_dist(d, cur_poc, flags) && d.h >= 8 && d.w >= 8 && d.h * d.w >= 128 &&
           d.bcw_idx == MM_BCW_DEFAULT && !(flags & MM_PU_WEIGHTED) && !(flags & MM_PU_REF_SCALED);
  }

  // mergeType == DEFAULT_N branch: xCheckIdenticalMotion, else xPredInterBi (DMVR inside)
  void leaf(const mm_pu_desc& d, bool dmvr) {
    mm_pu_desc o = d;
    o.flags = 0;
    o.reserved[0] = o.reserved[1] = 0;
    if (is_bi(d) && !t_.wp_bi && d.ref_poc[0] == d.ref_poc[1] && d.mv[0][0] == d.mv[1][0] &&
        d.mv[0][1] == d.mv[1][1]) {
      o.ref_poc[1] = -1;  // xPredInterUni(pu, REF_PIC_LIST_0, ..., bi = false)
      o.mv[1][0] = o.mv[1][1] = 0;
      o.model[1] = 0;
      mc_->push_back(o);
      return;
    }
    if (dmvr)
      dmvr_->push_back(o);
    else
      mc_->push_back(o);
  }

  // xSubPuMC (:283-359): sub is the PU's (w/8) x (h/8) SbTMVP motion field, raster order
  int sub_pu_mc(const mm_pu_motion& m, const mm_pu_desc* sub) {
    const mm_pu_desc& d = m.pu;
    const int num_line = (d.w >> ATMVP_SUB_BLOCK_SIZE) > 1 ? (d.w >> ATMVP_SUB_BLOCK_SIZE) : 1;
    const int num_col = (d.h >> ATMVP_SUB_BLOCK_SIZE) > 1 ? (d.h >> ATMVP_SUB_BLOCK_SIZE) : 1;
    const int pu_h = num_col == 1 ? d.h : 1 << ATMVP_SUB_BLOCK_SIZE;
    const int pu_w = num_line == 1 ? d.w : 1 << ATMVP_SUB_BLOCK_SIZE;
    auto mi = [&](int x, int y) -> const mm_pu_desc& {  // pu.getMotionInfo(Position{x, y})
      const int i = (y - d.y) / pu_h, j = (x - d.x) / pu_w;
      return sub[i * num_line + j];
    };
    const bool ver = d.h > d.w;
    const int fst_start = ver ? d.x : d.y, sec_start = ver ? d.y : d.x;
    const int fst_end = ver ? d.x + d.w : d.y + d.h, sec_end = ver ? d.y + d.h : d.x + d.w;
    const int fst_step = ver ? pu_w : pu_h, sec_step = ver ? pu_h : pu_w;
    const bool scaled = (m.flags & MM_PU_REF_SCALED) != 0;
    for (int fst = fst_start; fst < fst_end; fst += fst_step) {
      for (int sec = sec_start; sec < sec_end; sec += sec_step) {
        const int x = ver ? fst : sec, y = ver ? sec : fst;
        const mm_pu_desc& cur = mi(x, y);
        int length = sec_step, later = sec + sec_step;
        while (later < sec_end) {
          const mm_pu_desc& nxt = ver ? mi(fst, later) : mi(later, fst);
          if (!scaled && same_motion(nxt, cur))
            length += sec_step;
          else
            break;
          later += sec_step;
        }
        mm_pu_desc s = cur;  // subPu = curMi: motion (and the CU's BCW index)
        s.x = x;
        s.y = y;
        s.w = ver ? pu_w : length;
        s.h = ver ? length : pu_h;
        s.bcw_idx = d.bcw_idx;
        if (s.ref_poc[0] < 0 && s.ref_poc[1] < 0) return MM_ERR_ARG;
        // the sub-PU: mergeType DEFAULT_N, mvRefine false, m_subPuMC = true (no BDOF split)
        const int rc = motion_compensation(s, m.flags & ~(MM_PU_MVREFINE | MM_PU_SUBPU), m.cur_poc, true);
        if (rc) return rc;
        sec = later - sec_step;
      }
    }
    return MM_OK;
  }

  const mm_tool_flags& t_;
  std::vector<mm_pu_desc>* mc_;
  std::vector<mm_pu_desc>* dmvr_;
};

}  // namespace mmeff
