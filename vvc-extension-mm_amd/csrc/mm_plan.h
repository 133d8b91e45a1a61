// mm_plan.h -- host-side planning (C++ host code).
//
//  * Planner::plan_blocks: the parity API mm_reproject -- one job per
//    reprojectMotionVectorSubblocks call, prefix offsets and 64-element chunk starts for O(1)
//    item lookup in the kernels, GED epipoles resolved to rotation matrices
//    (EpipoleList::findEpipole + GeodesicMotionModel::setEpipole).
//  * build_pic_tables: the per-picture constants of the device-planned prediction path
//    (mm_devplan.h): reference slots, and for each slot the GEODESIC_CAMPOSE rotation of its
//    (curPOC, refPOC) epipole.
// Shared by the C-ABI (mm_kernels.hip) and the CPU twin of the test suite.
#pragma once
#include <algorithm>
#include <array>
#include <cmath>
#include <map>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/mm360.h"
#include "mm_devplan.h"
#include "mm_me.h"
#include "mm_dmvr.h"
#include "mm_epipole.h"
#include "mm_mvp.h"
#include "mm_pipeline.h"

namespace mmplan {
using namespace mmpipe;

struct Plan {
  std::vector<JobDev> jobs;
  std::vector<int> job_off, job_chunk;
  std::vector<int> ref_pocs;  // slot -> POC
  std::vector<M3> ged;
  int n_elems = 0, n_sb = 0;
  std::string err;
};

using EpipoleMap = mmepi::EpipoleList;

struct SeqInfo {
  mm_seq_params prm;
  int W, H, chroma;
};

inline SeqInfo seq_info(const mm_seq_params& p) { return {p, p.width, p.height, p.chroma_format == 1}; }

// The sequence constants of MVReprojection::init (MVReprojection.cpp:7-39, Projection.h:127-130)
inline SeqConst seq_const(const mm_seq_params& p) {
  SeqConst sc;
  sc.Wf = (float)p.width;
  sc.Hf = (float)p.height;
  sc.off = p.mm_offset4x4 == 4 ? 1.5f : (float)p.mm_offset4x4;  // MVReprojection.cpp:10
  sc.focal = (float)(1. / std::tan(M_PI / p.height));          // Projection.h:127-130
  sc.res = (float)(M_PI / p.height);                           // MVReprojection.cpp:27,33,39
  sc.ged_flavor = p.ged_flavor;
  return sc;
}

inline bool is_ged(int m) { return m >= GEODESIC_X && m <= GEODESIC_CAMPOSE; }

// EpipoleList::findEpipoleFixed lookup order (EpipoleList.cpp:19-36), available entries only
inline bool find_epipole(const EpipoleMap& epi, int cur, int ref, std::array<int32_t, 3>* out) {
  return epi.find(cur, ref, out);
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
      int gi = -1;
      int rc = ged_index(model, cur, ref, &gi);
      if (rc) return rc;
      j.ged_idx = (int16_t)gi;
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
      // JobDev stores block sizes in 8 bits and element counts in 16 bits: a block is at most one
      // CTU (128 x 128 luma, VVC's MAX_CU_SIZE) in component units, as every VVC PU is
      if (b.w <= 0 || b.h <= 0 || b.w > 128 || b.h > 128 || b.w % sb || b.h % sb || b.x < 0 || b.y < 0 ||
          b.x % sb || b.y % sb || b.x + b.w > Wc || b.y + b.h > Hc)
        return fail(MM_ERR_ARG, "block " + std::to_string(i) +
                                    " outside the picture, off the sub-block grid or larger than 128x128");
      rc = add_job(b.x << cs, b.y << cs, b.w, b.h, b.comp ? 1 : 0, b.model, b.mv_hor, b.mv_ver, b.cur_poc, b.ref_poc);
      if (rc) return rc;
    }
    finish_jobs();
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
    std::vector<JobDev> sorted(n);
    for (int i = 0; i < n; i++) sorted[i] = plan_->jobs[order[i]];
    plan_->jobs.swap(sorted);
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

// Per-picture tables of mm_pred_device: slots = the resident references (POC order), GED X/Y/Z
// fixed epipoles (MVReprojection.cpp:44-52) and the camera-pose epipole of (cur_poc, slot POC)
// when the epipole list has one (EpipoleList.cpp:19-36; a PU that needs a missing one raises
// MM_ERR_NOEPIPOLE on the device).
// The per-call tables of n_pics pictures (cur_pocs[q]) predicted by one launch chain against the
// context's resident references: the slots are shared, the GEODESIC_CAMPOSE rotation of (cur of
// picture q, reference s) is ged[ged_cam[q][s]]; equal epipoles share one rotation entry.
inline int build_pic_tables(const SeqInfo& s, const EpipoleMap& epi, const int* cur_pocs, int n_pics,
                            const std::vector<std::pair<int, RefDev>>& refs, mmdev::PicTables* t,
                            std::string* err) {
  if ((int)refs.size() > mmdev::MAX_SLOTS) {
    *err = "more than " + std::to_string(mmdev::MAX_SLOTS) + " resident reference pictures";
    return MM_ERR_ARG;
  }
  if (n_pics < 1 || n_pics > mmdev::MAX_PICS) {
    *err = "1.." + std::to_string(mmdev::MAX_PICS) + " pictures per call";
    return MM_ERR_ARG;
  }
  *t = mmdev::PicTables{};
  t->n_slots = (int)refs.size();
  t->n_pics = n_pics;
  t->W = s.W;
  t->H = s.H;
  t->chroma = s.chroma ? 1 : 0;
  t->active = s.prm.active_models;
  t->nf_mod4 = (int)(((long)(s.W / 4) * (s.H / 4)) % 4);
  t->only_list = -1;
  const V3 fixed[3] = {{1.0f, 0.0f, 0.0f}, {0.0f, 1.0f, 0.0f}, {0.0f, 0.0f, 1.0f}};
  for (int i = 0; i < 3; i++) t->ged[i] = ged_rotation(fixed[i]);
  for (int q = 0; q < mmdev::MAX_PICS; q++)
    for (int k = 0; k < mmdev::MAX_SLOTS; k++) t->ged_cam[q][k] = -1;
  std::vector<std::array<int32_t, 3>> used;  // epipoles of ged[3 ..]
  for (int k = 0; k < t->n_slots; k++) {
    t->poc[k] = refs[k].first;
    t->ref[k] = refs[k].second;
    for (int q = 0; q < n_pics; q++) {
      std::array<int32_t, 3> e;
      if (!find_epipole(epi, cur_pocs[q], refs[k].first, &e)) continue;
      int idx = -1;
      for (size_t u = 0; u < used.size(); u++)
        if (used[u] == e) idx = 3 + (int)u;
      if (idx < 0) {
        if ((int)used.size() == mmdev::MAX_SLOTS) {
          *err = "more than " + std::to_string(mmdev::MAX_SLOTS) + " distinct camera-pose epipoles in one call";
          return MM_ERR_ARG;
        }
        used.push_back(e);
        idx = 3 + (int)used.size() - 1;
        V3 v = {fixed_to_float(e[0], 24), fixed_to_float(e[1], 24), fixed_to_float(e[2], 24)};
        t->ged[idx] = ged_rotation(v);
      }
      t->ged_cam[q][k] = (int8_t)idx;
    }
  }
  return MM_OK;
}
// Distinct camera-pose epipoles the pictures cur_pocs[0..n) need against the resident references:
// one call's rotation table holds MAX_SLOTS of them (a single picture never needs more, it has at
// most MAX_SLOTS references), so mm_pred_device_multi cuts its pictures into runs that fit.
inline int count_cam_epipoles(const EpipoleMap& epi, const int* cur_pocs, int n,
                              const std::vector<std::pair<int, RefDev>>& refs) {
  std::vector<std::array<int32_t, 3>> used;
  for (const auto& r : refs)
    for (int q = 0; q < n; q++) {
      std::array<int32_t, 3> e;
      if (find_epipole(epi, cur_pocs[q], r.first, &e) && std::find(used.begin(), used.end(), e) == used.end())
        used.push_back(e);
    }
  return (int)used.size();
}
inline int build_pic_tables(const SeqInfo& s, const EpipoleMap& epi, int cur_poc,
                            const std::vector<std::pair<int, RefDev>>& refs, mmdev::PicTables* t,
                            std::string* err) {
  return build_pic_tables(s, epi, &cur_poc, 1, refs, t, err);
}

// ---- encoder candidate windows (mm_sad_window) ---------------------------------------------
// Batches of blocks with at most ME_BATCH_JOBS (block, candidate) jobs each; every block is
// validated as the reference's CHECKs / preconditions would (geometry, model, reference,
// epipole) before anything runs.
constexpr long ME_BATCH_JOBS = 1L << 22;  // 224 MB of setups; C5: ~3.8 K blocks, 2 M k_me_sad threads per batch

struct MeBatch {
  std::vector<mmme::MeBlockDev> blocks;
  std::vector<int> blk_off, chunk;  // element offsets per block, 64-element chunk starts
  int n_jobs = 0;
  long n_elems = 0;
};

// host_chunks false: the 64-element chunk starts are left to the device (k_me_chunks) -- at C5 they
// are 16 M entries per call, which the host would write and copy over PCIe
inline int plan_me_window(const SeqInfo& s, const mmdev::PicTables& t, const mm_me_block* blocks, int n,
                          const mmme::MeWindow& w, std::vector<MeBatch>* batches, std::string* err,
                          bool host_chunks = true) {
  batches->clear();
  MeBatch cur;
  for (int i = 0; i < n; i++) {
    const mm_me_block& b = blocks[i];
    if (b.w < 4 || b.h < 4 || b.w > 128 || b.h > 128 || (b.w & 3) || (b.h & 3) || (b.x & 3) || (b.y & 3) ||
        b.x < 0 || b.y < 0 || b.x > s.W - b.w || b.y > s.H - b.h || b.sub_shift < 0 || b.sub_shift > 1) {
      *err = "ME block " + std::to_string(i) + " outside the picture, not 4x4 aligned or invalid subShift";
      return MM_ERR_ARG;
    }
    if (b.model <= CLASSIC || b.model >= NUM_MODELS || !(t.active & (1u << b.model))) {
      *err = "ME block " + std::to_string(i) + ": invalid, CLASSIC or inactive motion model";
      return MM_ERR_MODEL;
    }
    int slot = -1;
    for (int k = 0; k < t.n_slots; k++)
      if (t.poc[k] == b.ref_poc) slot = k;
    if (slot < 0) {
      *err = "ME block " + std::to_string(i) + ": reference POC " + std::to_string(b.ref_poc) + " not uploaded";
      return MM_ERR_NOREF;
    }
    int ged = -1;
    if (b.model == GEODESIC_CAMPOSE) {
      if (t.ged_cam[0][slot] < 0) {
        *err = "ME block " + std::to_string(i) + ": no epipole for (curPOC, refPOC)";
        return MM_ERR_NOEPIPOLE;
      }
      ged = t.ged_cam[0][slot];
    } else if (b.model >= GEODESIC_X && b.model <= GEODESIC_Z) {
      ged = b.model - GEODESIC_X;
    }
    const int nsb = (b.w / 4) * (b.h / 4);
    if (!cur.blocks.empty() && (long)cur.n_jobs + w.C > ME_BATCH_JOBS) {
      batches->push_back(std::move(cur));
      cur = MeBatch();
    }
    mmme::MeBlockDev d;
    d.x = b.x;
    d.y = b.y;
    d.w = b.w;
    d.h = b.h;
    d.mvh = b.mv_hor;
    d.mvv = b.mv_ver;
    d.model = b.model;
    d.slot = slot;
    d.ged_idx = ged;
    d.sub_shift = b.sub_shift;
    d.n = nsb;
    d.rows = b.h / 4;
    d.elem_off = (int)cur.n_elems;
    d.sad_off = i * w.C;
    cur.blocks.push_back(d);
    cur.blk_off.push_back(d.elem_off);
    cur.n_jobs += w.C;
    cur.n_elems += (long)(w.npat ? 1 : w.side) * nsb;  // k_me_sad thread per (window row, sub-block)
  }
  if (!cur.blocks.empty()) batches->push_back(std::move(cur));
  if (host_chunks)
    for (auto& bt : *batches) build_chunks(bt.blk_off, (int)bt.n_elems, &bt.chunk);
  return MM_OK;
}

// ---- MM-MVP (mm_mvp_convert[_device]) ------------------------------------------------------------
// The available entries of an EpipoleList in key order: the device table the MVP kernel resolves
// GEODESIC_CAMPOSE epipoles from (mmmvp::epi_find).
inline void epi_entries(const EpipoleMap& epi, std::vector<mmmvp::EpiDev>* out) {
  out->clear();
  for (const auto& kv : epi.entries()) {
    if (!kv.second.available) continue;
    mmmvp::EpiDev e;
    e.cur = kv.first.first;
    e.ref = kv.first.second;
    for (int i = 0; i < 3; i++) e.q[i] = kv.second.q[i];
    out->push_back(e);
  }
}

}  // namespace mmplan
