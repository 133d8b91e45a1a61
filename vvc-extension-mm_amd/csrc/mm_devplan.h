// mm_devplan.h -- device-side planning of one picture's PU list (host + device bodies).
//
// mm_pred_device takes the caller's PU descriptors where they already are (HBM) and plans on the
// device, so that one picture's whole MM path -- dispatch, per-block setup, reprojection,
// interpolation, bi-averaging -- is a fixed sequence of launches with no host round trip:
//
//   k_plan_count  thread per PU: classify (InterPrediction::xPredInterUni's MM branch,
//                 InterPrediction.cpp:455-533, plus argument CHECKs), then
//                 workgroup-aggregated counts per PU class and per job key
//   k_plan_place  thread per PU: place the PU and its reprojection jobs in their buckets
//                 (class-sorted PUs, (component, model, packet)-sorted jobs), write JobDev /
//                 PuDev, prefix offsets and 64-element chunk starts
//   k_setup, k_reproj, k_mc  as for the host plan, sizes read from PlanMeta
//
// Order inside a bucket follows atomic arrival and only affects speed: every PU writes its own
// samples, so results do not depend on it.  The classification and emission bodies below are
// shared with the CPU twin (tests/native/host_twin.cpp), which places PUs sequentially.
#pragma once
#include "../../include/mm360.h"
#include "mm_pipeline.h"

namespace mmdev {
using namespace mmpipe;

constexpr int MAX_SLOTS = 16;  // reference pictures addressable by one picture (2 lists x 8)
// PU buckets: class (bi, uni L0, uni L1) x sub-block alignment.  PUs whose sub-block count is a
// multiple of 4 come first (buckets 0-2), so every aligned group of 4 consecutive sub-blocks
// (a lane quad of k_mc) lies inside one PU; the rest (4x8 / 8x4 / 4x4 ...) follow (buckets 3-5).
constexpr int N_PU_KEYS = 6;
MM_HD int pu_key(int cls, int n_sb) { return cls + ((n_sb & 3) ? 3 : 0); }
// class of flat luma sub-block g from the bucket bases (PlanMeta::sb_base)
// sb_base is non-decreasing, so the last bucket starting at or before g is the number of bucket
// starts k >= 1 at or before g: every start is read unconditionally (one batch of scalar loads in
// k_mc, not a chain of dependent load-compare-branch steps)
MM_HD int sb_class(int g, const int* sb_base) {
  int k = 0;
#pragma unroll
  for (int i = 1; i < N_PU_KEYS; i++) k += g >= sb_base[i] ? 1 : 0;
  return k % 3;
}
constexpr int N_JOB_KEYS = 64;

// Per-picture constant tables, passed by value as kernel arguments.
struct PicTables {
  int n_slots;
  int poc[MAX_SLOTS];
  int ged_cam[MAX_SLOTS];  // GED table index of GEODESIC_CAMPOSE for (cur, poc[s]), -1 = no epipole
  RefDev ref[MAX_SLOTS];
  M3 ged[3 + MAX_SLOTS];   // [0..2] GEODESIC_X/Y/Z, [3+s] CAMPOSE of slot s
  int W, H, chroma;
  uint32_t active;
  int nf_mod4;             // (W/4 * H/4) % 4, frame-cache packet tail (MPA chroma aliasing)
  int only_list;           // -1: normal prediction; 0/1: mm_pred_list of that list (other list ignored)
  RefPool pool;            // the context's reference pool (device interior filters)
};

// Offsets of everything k_plan_place produced; written by k_plan_place's first thread.
struct PlanMeta {
  int n_pus, n_sb, n_jobs, n_elems;
  int pu_base[N_PU_KEYS], sb_base[N_PU_KEYS];
  int job_base[N_JOB_KEYS], elem_base[N_JOB_KEYS];
};

// Host-side bucket counters of the sequential planners (CPU twin).  64-bit words pack
// (items, elements): lo 32 bits = count, hi 32 bits = elements.
struct PlanCounters {
  unsigned long long pu_tot[N_PU_KEYS], pu_cur[N_PU_KEYS];
  unsigned long long job_tot[N_JOB_KEYS], job_cur[N_JOB_KEYS];
};

struct JobPlan {
  int valid, key, n, rows, cw, ch, comp, model, mv_hor, mv_ver, ged_idx, list;
};

struct PuPlan {
  int code;     // MM_OK or the error this PU raises
  int cls;      // 0 bi, 1 uni L0, 2 uni L1
  int key;      // PU bucket (pu_key)
  int n_sb;     // luma 4x4 sub-blocks
  int slot[2];
  int bcw;      // BCW weight index (bi), MM_BCW_DEFAULT otherwise
  JobPlan job[4];   // [2 * list + comp]; fixed slots keep the struct in registers
  int alias[2]; // list's chroma job aliases its luma job
};

MM_HD int job_key(int comp, int model, int n) { return (comp * 16 + model) * 2 + (n < 4 ? 1 : 0); }

// MPA chroma reprojection == luma reprojection, element for element, when every element of the
// block is a packet lane both in the luma frame cache and in the chroma block:
//  * the chroma grid (LinSpaced 2*xc + off + 4i) holds the luma grid values (4i + off);
//  * the chroma block's toPerspective (packet for N % 4 == 0) equals the frame cache entry
//    (packet for frame index < Nf - Nf % 4) -- same function, same inputs, same packet mode;
//  * the motion (mv * sign), toProjection and NaN fallback are identical;
//  * (x - off) * 16 == ((x - off) / 2) * 32 exactly (power-of-two scalings).
// So the 1/32-pel chroma result equals the 1/16-pel luma result and k_mc reads the luma job
// (checked on every grid size by the CPU test suite: test_mpa_chroma_equals_luma_for_packet_blocks).
MM_HD bool mpa_chroma_aliases(const PicTables& t, int model, int w, int h) {
  if (model < MPA_FRONT_BACK || model > MPA_TOP_BOTTOM) return false;
  const int n = (w / 4) * (h / 4);
  return n >= 4 && n % 4 == 0 && t.nf_mod4 == 0;
}

// Classification of one PU: argument checks (the reference CHECKs sizes and models), slot and GED lookup,
// and the list of reprojection jobs it needs.
MM_HD void classify_pu(const mm_pu_desc& u, const PicTables& t, PuPlan* p) {
  p->code = MM_OK;
  for (int k = 0; k < 4; k++) p->job[k].valid = 0;
  p->cls = 0;
  p->key = 0;
  p->n_sb = 0;
  p->slot[0] = p->slot[1] = -1;
  p->alias[0] = p->alias[1] = 0;
  p->bcw = MM_BCW_DEFAULT;
  if (u.w < 4 || u.h < 4 || u.w > 128 || u.h > 128 || (u.w & 3) || (u.h & 3) || (u.x & 3) || (u.y & 3) || u.x < 0 ||
      u.y < 0 || u.x > t.W - u.w || u.y > t.H - u.h) {
    p->code = MM_ERR_ARG;
    return;
  }
  // mm_pred_list: the PU must use the list (selects, not an index: a runtime index into `u` would
  // demote the descriptor from registers to LDS)
  if ((t.only_list == 0 && u.ref_poc[0] < 0) || (t.only_list == 1 && u.ref_poc[1] < 0)) {
    p->code = MM_ERR_ARG;
    return;
  }
  int used = 0;
#pragma unroll
  for (int l = 0; l < 2; l++) {
    if (u.ref_poc[l] < 0 || (t.only_list >= 0 && l != t.only_list)) continue;
    used++;
    const int m = u.model[l];
    if (m <= CLASSIC || m >= NUM_MODELS || !(t.active & (1u << m))) {
      p->code = MM_ERR_MODEL;
      return;
    }
    int s = -1;
    for (int k = 0; k < t.n_slots; k++)
      if (t.poc[k] == u.ref_poc[l]) s = k;
    if (s < 0) {
      p->code = MM_ERR_NOREF;
      return;
    }
    p->slot[l] = s;
    int ged = -1;
    if (m == GEODESIC_CAMPOSE) {
      if (t.ged_cam[s] < 0) {
        p->code = MM_ERR_NOEPIPOLE;
        return;
      }
      ged = t.ged_cam[s];
    } else if (m >= GEODESIC_X && m <= GEODESIC_Z) {
      ged = m - GEODESIC_X;
    }
#pragma unroll
    for (int comp = 0; comp < 2; comp++) {
      if (comp == 1 && !t.chroma) continue;
      if (comp == 1 && mpa_chroma_aliases(t, m, u.w, u.h)) {
        p->alias[l] = 1;
        continue;
      }
      const int sb = comp ? 2 : 4;
      JobPlan& j = p->job[2 * l + comp];
      j.valid = 1;
      j.cw = u.w >> comp;
      j.ch = u.h >> comp;
      j.rows = j.ch / sb;
      j.n = (j.cw / sb) * j.rows;
      j.comp = comp;
      j.model = m;
      j.mv_hor = u.mv[l][0];
      j.mv_ver = u.mv[l][1];
      j.ged_idx = ged;
      j.list = l;
      j.key = job_key(comp, m, j.n);
    }
  }
  if (!used) {
    p->code = MM_ERR_ARG;
    return;
  }
  p->cls = (p->slot[0] >= 0 && p->slot[1] >= 0) ? 0 : (p->slot[0] >= 0 ? 1 : 2);
  if (p->cls == 0) {  // CU::bcwIdx, Rom.cpp:203 g_BcwWeights[BCW_NUM]
    if (u.bcw_idx < 0 || u.bcw_idx > 4) {
      p->code = MM_ERR_ARG;
      return;
    }
    p->bcw = u.bcw_idx;
  }
  p->n_sb = (u.w / 4) * (u.h / 4);
  p->key = pu_key(p->cls, p->n_sb);
}

MM_HD unsigned long long status_word(int pu_index, int code) {
  return ~(((unsigned long long)(unsigned)pu_index << 8) | (unsigned)code);  // atomicMax keeps the lowest PU
}

MM_HD unsigned long long pack_count(int items, int elems) {
  return ((unsigned long long)(unsigned)elems << 32) | (unsigned)items;
}
MM_HD int packed_items(unsigned long long v) { return (int)(v & 0xffffffffull); }
MM_HD int packed_elems(unsigned long long v) { return (int)(v >> 32); }

// Exclusive prefix of the bucket totals -> PlanMeta (one thread).
MM_HD void plan_meta(const PlanCounters& c, PlanMeta* m) {
  int acc = 0, sacc = 0;
  for (int k = 0; k < N_PU_KEYS; k++) {
    m->pu_base[k] = acc;
    m->sb_base[k] = sacc;
    acc += packed_items(c.pu_tot[k]);
    sacc += packed_elems(c.pu_tot[k]);
  }
  m->n_pus = acc;
  m->n_sb = sacc;
  acc = sacc = 0;
  for (int k = 0; k < N_JOB_KEYS; k++) {
    m->job_base[k] = acc;
    m->elem_base[k] = sacc;
    acc += packed_items(c.job_tot[k]);
    sacc += packed_elems(c.job_tot[k]);
  }
  m->n_jobs = acc;
  m->n_elems = sacc;
}

// Item `idx` covers flat elements [off, off + n): it starts every 64-element chunk whose first
// element it holds (find_item's chunk table).
MM_HD void write_chunks(int* chunk, int idx, int off, int n) {
  for (int e = (off + 63) & ~63; e < off + n; e += 64) chunk[e >> 6] = idx;
}

// Emit the jobs of the PU placed at luma sub-block offset sb_off; job_idx/job_elem_off are the
// placed positions of the valid p.job[k].  The PU itself needs no record: its luma job of the
// first used list writes the per-sub-block meta word k_mc reads (JobDev::meta_hi).
MM_HD void emit_pu(const mm_pu_desc& u, const PuPlan& p, int sb_off, const int* job_idx, const int* job_elem_off,
                   JobDev* jobs, int* job_off, int* job_chunk) {
  const int primary = p.cls == 2 ? 1 : 0;
  const int meta_hi = (p.slot[0] < 0 ? 0 : p.slot[0]) | ((p.slot[1] < 0 ? 0 : p.slot[1]) << 4) | (p.bcw << 8);
  for (int i = 0; i < 4; i++) {
    const JobPlan& jp = p.job[i];
    if (!jp.valid) continue;
    JobDev j;
    j.x = u.x;
    j.y = u.y;
    j.cw = jp.cw;
    j.ch = jp.ch;
    j.comp = jp.comp;
    j.model = jp.model;
    j.mv_hor = jp.mv_hor;
    j.mv_ver = jp.mv_ver;
    j.ged_idx = jp.ged_idx;
    j.n = jp.n;
    j.rows = jp.rows;
    j.offset = job_elem_off[i];
    j.sb_base = sb_off;
    j.pu_cols = u.w / 4;
    j.list = jp.list;
    j.slot = p.slot[jp.list];
    j.alias = jp.comp == 0 ? p.alias[jp.list] : 0;
    j.meta_hi = meta_hi | ((jp.comp == 0 && jp.list == primary) ? MM_META_PRIMARY : 0);
    jobs[job_idx[i]] = j;
    job_off[job_idx[i]] = job_elem_off[i];
    write_chunks(job_chunk, job_idx[i], job_elem_off[i], jp.n);
  }
}

}  // namespace mmdev
