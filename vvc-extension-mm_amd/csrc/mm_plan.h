// mm_plan.h -- host-side planning of one mm_reproject / mm_pred call (C++ host code).
//
// Turns the caller's block / PU descriptors into the flat work lists the kernels walk:
//   jobs   one per reprojectMotionVectorSubblocks call (PU x list x {luma, chroma})
//   pus    one per PU, with its reference slots and job indices
// plus prefix offsets and 64-element chunk starts for O(1) item lookup in the kernels.  It also
// resolves reference POCs to slots and GED epipoles to rotation matrices
// (EpipoleList::findEpipole + GeodesicMotionModel::setEpipole).  Shared by the C-ABI
// (mm_kernels.hip) and the CPU twin of the test suite.
#pragma once
#include <algorithm>
#include <array>
#include <map>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/mm360.h"
#include "mm_pipeline.h"

namespace mmplan {
using namespace mmpipe;

struct Plan {
  std::vector<JobDev> jobs;
  std::vector<int> job_off, job_chunk;
  std::vector<PuDev> pus;
  std::vector<int> pu_off, pu_chunk;
  std::vector<int> ref_pocs;  // slot -> POC
  std::vector<M3> ged;
  int n_elems = 0, n_sb = 0;
  std::string err;
};

using EpipoleMap = std::map<std::pair<int, int>, std::array<int32_t, 3>>;

struct SeqInfo {
  mm_seq_params prm;
  int W, H, chroma;
};

inline SeqInfo seq_info(const mm_seq_params& p) { return {p, p.width, p.height, p.chroma_format == 1}; }

inline bool is_ged(int m) { return m >= GEODESIC_X && m <= GEODESIC_CAMPOSE; }

// EpipoleList::findEpipoleFixed lookup order (EpipoleList.cpp:19-36)
inline bool find_epipole(const EpipoleMap& epi, int cur, int ref, std::array<int32_t, 3>* out) {
  auto it = epi.find({cur, ref});
  if (it == epi.end()) it = epi.find({cur, -1});
  if (it == epi.end()) it = epi.find({-1, -1});
  if (it == epi.end()) return false;
  *out = it->second;
  return true;
}

inline void build_chunks(const std::vector<int>& off, int total, std::vector<int>* chunk) {
  int nchunks = (total + 63) / 64;
  chunk->assign(nchunks > 0 ? nchunks : 1, 0);
  int j = 0, n = (int)off.size();
  for (int c = 0; c < nchunks; c++) {
    int g = c * 64;
    while (j + 1 < n && off[j + 1] <= g) j++;
    (*chunk)[c] = j;
  }
}

class Planner {
 public:
  Planner(const SeqInfo& s, const EpipoleMap& e, Plan* p) : seq_(s), epi_(e), plan_(p) { *plan_ = Plan(); }

  int model_ok(int m) {
    if (m <= CLASSIC || m >= NUM_MODELS) return fail(MM_ERR_MODEL, "invalid or CLASSIC motion model " + std::to_string(m));
    if (!(seq_.prm.active_models & (1u << m))) return fail(MM_ERR_MODEL, "motion model not active: " + std::to_string(m));
    return MM_OK;
  }

  // GED rotation for (model, cur, ref); X/Y/Z use fixed epipoles (MVReprojection.cpp:44-52)
  int ged_index(int model, int cur, int ref, int* idx) {
    auto key = std::make_tuple(model, model == GEODESIC_CAMPOSE ? cur : 0, model == GEODESIC_CAMPOSE ? ref : 0);
    auto it = ged_map_.find(key);
    if (it != ged_map_.end()) {
      *idx = it->second;
      return MM_OK;
    }
    V3 e;
    if (model == GEODESIC_X)
      e = {1.0f, 0.0f, 0.0f};
    else if (model == GEODESIC_Y)
      e = {0.0f, 1.0f, 0.0f};
    else if (model == GEODESIC_Z)
      e = {0.0f, 0.0f, 1.0f};
    else {
      std::array<int32_t, 3> q;
      if (!find_epipole(epi_, cur, ref, &q))
        return fail(MM_ERR_NOEPIPOLE,
                    "No epipole for (curPOC, refPOC) = (" + std::to_string(cur) + ", " + std::to_string(ref) + ")");
      e = {fixed_to_float(q[0], 24), fixed_to_float(q[1], 24), fixed_to_float(q[2], 24)};
    }
    plan_->ged.push_back(ged_rotation(e));
    *idx = (int)plan_->ged.size() - 1;
    ged_map_.emplace(key, *idx);
    return MM_OK;
  }

  // lx, ly: block position in luma units; cw, ch: size in component units
  int add_job(int lx, int ly, int cw, int ch, int comp, int model, int mvh, int mvv, int cur, int ref) {
    JobDev j{};
    j.x = lx;
    j.y = ly;
    j.cw = cw;
    j.ch = ch;
    j.comp = comp;
    j.model = model;
    j.mv_hor = mvh;
    j.mv_ver = mvv;
    j.ged_idx = -1;
    if (is_ged(model)) {
      int rc = ged_index(model, cur, ref, &j.ged_idx);
      if (rc) return rc;
    }
    const int sb = comp ? 2 : 4;
    j.rows = ch / sb;
    j.n = (cw / sb) * (ch / sb);
    j.offset = plan_->n_elems;
    plan_->n_elems += j.n;
    plan_->jobs.push_back(j);
    plan_->job_off.push_back(j.offset);
    return MM_OK;
  }

  int plan_blocks(const mm_block_desc* blocks, int n) {
    for (int i = 0; i < n; i++) {
      const mm_block_desc& b = blocks[i];
      int rc = model_ok(b.model);
      if (rc) return rc;
      if (b.comp < 0 || b.comp > 2 || (b.comp > 0 && !seq_.chroma)) return fail(MM_ERR_ARG, "invalid component");
      const int cs = b.comp ? 1 : 0, sb = b.comp ? 2 : 4;
      const int Wc = seq_.W >> cs, Hc = seq_.H >> cs;
      if (b.w <= 0 || b.h <= 0 || b.w % sb || b.h % sb || b.x < 0 || b.y < 0 || b.x % sb || b.y % sb ||
          b.x + b.w > Wc || b.y + b.h > Hc)
        return fail(MM_ERR_ARG, "block " + std::to_string(i) + " outside the picture or off the sub-block grid");
      rc = add_job(b.x << cs, b.y << cs, b.w, b.h, b.comp ? 1 : 0, b.model, b.mv_hor, b.mv_ver, b.cur_poc, b.ref_poc);
      if (rc) return rc;
    }
    finish_jobs();
    return MM_OK;
  }

  // MPA chroma reprojection == luma reprojection, element for element, when every element of the
  // block is a packet lane both in the luma frame cache and in the chroma block:
  //  * the chroma grid (LinSpaced 2*xc + off + 4i) holds the luma grid values (4i + off);
  //  * the chroma block's toPerspective (packet for N % 4 == 0) equals the frame cache entry
  //    (packet for frame index < Nf - Nf % 4) -- same function, same inputs, same packet mode;
  //  * the motion (mv * sign), toProjection and NaN fallback are identical;
  //  * (x - off) * 16 == ((x - off) / 2) * 32 exactly (power-of-two scalings).
  // So the 1/32-pel chroma result equals the 1/16-pel luma result and k_mc reads the luma job.
  bool chroma_aliases_luma(int model, int w, int h) const {
    if (model < MPA_FRONT_BACK || model > MPA_TOP_BOTTOM) return false;
    const long nf = (long)(seq_.W / 4) * (seq_.H / 4);
    const int n = (w / 4) * (h / 4);
    return n >= 4 && n % 4 == 0 && nf % 4 == 0;
  }

  // has_ref(poc) -> bool: is the reference uploaded
  template <typename HasRef>
  int plan_pus(int cur_poc, const mm_pu_desc* pus, int n, HasRef has_ref) {
    std::map<int, int> slot_of;
    for (int i = 0; i < n; i++) {
      const mm_pu_desc& u = pus[i];
      if (u.w < 4 || u.h < 4 || u.w > 128 || u.h > 128 || (u.w & 3) || (u.h & 3) || (u.x & 3) || (u.y & 3) ||
          u.x < 0 || u.y < 0 || u.x + u.w > seq_.W || u.y + u.h > seq_.H)
        return fail(MM_ERR_ARG, "PU " + std::to_string(i) + " outside the picture or not 4x4 aligned");
      PuDev d{};
      d.x = u.x;
      d.y = u.y;
      d.w = u.w;
      d.h = u.h;
      int used = 0;
      for (int l = 0; l < 2; l++) {
        d.ref_slot[l] = -1;
        d.job[l][0] = d.job[l][1] = -1;
        if (u.ref_poc[l] < 0) continue;
        used++;
        int rc = model_ok(u.model[l]);
        if (rc) return rc;
        if (!has_ref(u.ref_poc[l]))
          return fail(MM_ERR_NOREF, "reference POC " + std::to_string(u.ref_poc[l]) + " not uploaded");
        auto sit = slot_of.find(u.ref_poc[l]);
        if (sit == slot_of.end()) {
          plan_->ref_pocs.push_back(u.ref_poc[l]);
          sit = slot_of.emplace(u.ref_poc[l], (int)plan_->ref_pocs.size() - 1).first;
        }
        d.ref_slot[l] = sit->second;
        for (int comp = 0; comp < (seq_.chroma ? 2 : 1); comp++) {
          if (comp == 1 && chroma_aliases_luma(u.model[l], u.w, u.h)) {
            d.job[l][1] = d.job[l][0];
            continue;
          }
          d.job[l][comp] = (int)plan_->jobs.size();
          rc = add_job(u.x, u.y, u.w >> comp, u.h >> comp, comp, u.model[l], u.mv[l][0], u.mv[l][1], cur_poc,
                       u.ref_poc[l]);
          if (rc) return rc;
        }
      }
      if (!used) return fail(MM_ERR_ARG, "PU " + std::to_string(i) + " uses no reference list");
      plan_->pus.push_back(d);
    }
    finish_jobs();
    // k_mc enumeration grouped by prediction class (bi, uni L0, uni L1): a wave then runs one
    // class's code path instead of both lists masked
    auto cls = [](const PuDev& d) { return d.ref_slot[0] >= 0 && d.ref_slot[1] >= 0 ? 0 : (d.ref_slot[0] >= 0 ? 1 : 2); };
    std::stable_sort(plan_->pus.begin(), plan_->pus.end(),
                     [&](const PuDev& a, const PuDev& b) { return cls(a) < cls(b); });
    for (auto& d : plan_->pus) {
      d.sb_offset = plan_->n_sb;
      plan_->n_sb += (d.w / 4) * (d.h / 4);
      plan_->pu_off.push_back(d.sb_offset);
    }
    build_chunks(plan_->pu_off, plan_->n_sb, &plan_->pu_chunk);
    return MM_OK;
  }

 private:
  // Enumerate jobs grouped by (component, model, packet/scalar) so that the waves of k_setup and
  // k_reproj run one model path each instead of every model's path (divergence).  j.offset keeps
  // each job's place in the result array; job_off is the prefix over the enumeration order.
  void finish_jobs() {
    const int n = (int)plan_->jobs.size();
    std::vector<int> order(n);
    for (int i = 0; i < n; i++) order[i] = i;
    auto key = [&](int i) {
      const JobDev& j = plan_->jobs[i];
      return (j.comp * 64 + j.model) * 2 + (j.n < 4 ? 1 : 0);
    };
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return key(a) < key(b); });
    std::vector<int> inv(n);
    std::vector<JobDev> sorted(n);
    for (int i = 0; i < n; i++) {
      sorted[i] = plan_->jobs[order[i]];
      inv[order[i]] = i;
    }
    plan_->jobs.swap(sorted);
    for (auto& d : plan_->pus)
      for (int l = 0; l < 2; l++)
        for (int c = 0; c < 2; c++)
          if (d.job[l][c] >= 0) d.job[l][c] = inv[d.job[l][c]];
    plan_->job_off.resize(n);
    int acc = 0;
    for (int i = 0; i < n; i++) {
      plan_->job_off[i] = acc;
      acc += plan_->jobs[i].n;
    }
    build_chunks(plan_->job_off, plan_->n_elems, &plan_->job_chunk);
    if (plan_->ged.empty()) plan_->ged.push_back(M3{});
  }
  int fail(int code, const std::string& m) {
    plan_->err = m;
    return code;
  }
  SeqInfo seq_;
  const EpipoleMap& epi_;
  Plan* plan_;
  std::map<std::tuple<int, int, int>, int> ged_map_;
};

}  // namespace mmplan
