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
#include "mm_dmvr.h"
#include "mm_pipeline.h"

namespace mmdev {
using namespace mmpipe;
using mmdmvr::N_OFF;
using mmdmvr::SubPuDev;

constexpr int MAX_SLOTS = 16;  // reference pictures addressable by one picture (2 lists x 8)
// Pictures one launch chain predicts together (mm_pred_device_multi): independent pictures -- the
// leaves of a random-access temporal layer -- share the planning, setup, reprojection and
// interpolation launches; each PU carries its picture index (PuPlan::seg, McRec meta bits 14-15).
constexpr int MAX_PICS = MM_MAX_PICS;
// PU buckets: N_BANDS vertical strips of the picture (by the PU's left column), or one bucket.
// Inside a bucket PUs keep the list's (decode, raster-CTU) order -- k_plan_place places them with
// a block-wide scan per bucket -- so the sub-block enumeration k_mc reads is spatial, and k_mc
// handles bi and uni sub-blocks in one body (the McRec meta word says which lists a sub-block
// uses), so no class buckets are needed.  k_mc runs band r on the workgroups of one XCD
// (mm_kernels.hip k_mc_dev), so the sub-blocks an XCD has in flight share reference lines in its
// L2: with strips (PU_STRIPS) band r is strip r, walked CTU row by CTU row -- an XCD's working set
// is a compact region of the picture -- otherwise it is an eighth of the list (a run of CTU rows
// across the whole width).  (64 picture-row bins measured the same k_mc as one bucket and planned
// slower: profiles/r03_ab_pu_keys.txt; strips: profiles/r03_ab_pu_strips.txt.)
constexpr bool PU_STRIPS = false;
constexpr int N_BANDS = 8;
constexpr int N_PU_KEYS = PU_STRIPS ? N_BANDS : 1;
MM_HD int pu_key(int x, int W) {
  if (!PU_STRIPS) return 0;
  const int k = (int)(((long)x * N_BANDS) / W);
  return k < N_BANDS - 1 ? k : N_BANDS - 1;
}

// band r = sub-blocks [band[r], band[r + 1]): the strips' buckets, or an equal split of the list
MM_HD void band_cut(const int* sb_base, int n_sb, int* band) {
  for (int r = 0; r <= N_BANDS; r++) {
    if (PU_STRIPS)
      band[r] = r < N_PU_KEYS ? sb_base[r] : n_sb;
    else
      band[r] = (int)((long)n_sb * r / N_BANDS);
  }
}
constexpr int N_JOB_KEYS = 64;
constexpr int DMVR_KEY = N_PU_KEYS + N_JOB_KEYS;  // one bucket of MM-DMVR sub-PUs after the PU and job keys

// Per-picture constant tables, passed by value as kernel arguments.
struct PicTables {
  int n_slots;
  int poc[MAX_SLOTS];
  int8_t ged_cam[MAX_PICS][MAX_SLOTS];  // GED table index of GEODESIC_CAMPOSE for (cur of picture q, poc[s]), -1: none
  RefDev ref[MAX_SLOTS];
  M3 ged[3 + MAX_SLOTS];   // [0..2] GEODESIC_X/Y/Z, [3+s] CAMPOSE of slot s
  int W, H, chroma;
  uint32_t active;
  int nf_mod4;             // (W/4 * H/4) % 4, frame-cache packet tail (MPA chroma aliasing)
  int only_list;           // -1: normal prediction; 0/1: mm_pred_list of that list (other list ignored)
  int dmvr;                // MM_PUF_DMVR PUs allowed (mm_set_dmvr: the picture's DMVR enable)
  RefPool pool;            // the context's reference pool (device interior filters)
  uint32_t pool_slot4[MAX_SLOTS / 4];  // pool slot of table slot s: byte s % 4 of word s / 4 (device)
  int n_pics;              // pictures of the call (mm_pred_device_multi; 1 otherwise)
};

// The PU lists of a call's pictures (device pointers), one index space: picture q holds PUs
// [base[q], base[q + 1]).  Read by select, never by a per-lane index into the kernel argument.
struct PuSegs {
  const mm_pu_desc* p[MAX_PICS];
  int base[MAX_PICS + 1];
  int n_pics;
};
// picture of PU index i (uniform loop)
MM_HD int pu_seg(const PuSegs& s, int i) {
  int q = 0;
#pragma unroll
  for (int k = 1; k < MAX_PICS; k++) q += (k < s.n_pics && i >= s.base[k]) ? 1 : 0;
  return q;
}
MM_HD mm_pu_desc load_pu(const PuSegs& s, int i, int q) {
  const mm_pu_desc* p = s.p[0];
#pragma unroll
  for (int k = 1; k < MAX_PICS; k++) p = q == k ? s.p[k] : p;
  int b = s.base[0];
#pragma unroll
  for (int k = 1; k < MAX_PICS; k++) b = q == k ? s.base[k] : b;
  return p[i - b];
}

// Offsets of everything k_plan_place produced; written by k_plan_place's first thread.
struct PlanMeta {
  int n_pus, n_sb, n_jobs, n_elems;
  int pu_base[N_PU_KEYS], sb_base[N_PU_KEYS];
  int job_base[N_JOB_KEYS], elem_base[N_JOB_KEYS];
  int n_sub, n_dmvr_elems;  // MM-DMVR sub-PU records and their cost elements (N_OFF * n each)
  int band[N_BANDS + 1];    // k_mc's bands of the sub-block enumeration (band_cut)
};

// Host-side bucket counters of the sequential planners (CPU twin).  64-bit words pack
// (items, elements): lo 32 bits = count, hi 32 bits = elements.
struct PlanCounters {
  unsigned long long pu_tot[N_PU_KEYS], pu_cur[N_PU_KEYS];
  unsigned long long job_tot[N_JOB_KEYS], job_cur[N_JOB_KEYS];
  unsigned long long dmvr_tot, dmvr_cur;
};

struct JobPlan {
  int valid, key, n, rows, cw, ch, comp, model, mv_hor, mv_ver, ged_idx, list;
};

struct PuPlan {
  int code;     // MM_OK or the error this PU raises
  int seg;      // picture of the call (mm_pred_device_multi)
  int cls;      // 0 bi, 1 uni L0, 2 uni L1
  int key;      // PU bucket (pu_key)
  int n_sb;     // luma 4x4 sub-blocks (of the whole PU)
  int slot[2];
  int bcw;      // BCW weight index (bi), MM_BCW_DEFAULT otherwise
  JobPlan job[4];   // [2 * list + comp]; fixed slots keep the struct in registers (per sub-PU for DMVR)
  int alias[2]; // list's chroma job aliases its luma job
  // MM_PUF_DMVR: the PU is placed as n_items = sx * sy sub-PUs of sub_w x sub_h luma samples
  // (xProcessDMVRProjected, InterPrediction.cpp:2452-2486: min(w, 16) x min(h, 16)), each one bi PU
  // bucket item with its own jobs and one DMVR record; n_items = 1 otherwise
  int dmvr, n_items, sub_w, sub_h, sx;
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
MM_HD void classify_pu(const mm_pu_desc& u, const PicTables& t, PuPlan* p, int seg = 0) {
  p->code = MM_OK;
  p->seg = seg;
  for (int k = 0; k < 4; k++) p->job[k].valid = 0;
  p->cls = 0;
  p->key = 0;
  p->n_sb = 0;
  p->slot[0] = p->slot[1] = -1;
  p->alias[0] = p->alias[1] = 0;
  p->bcw = MM_BCW_DEFAULT;
  p->dmvr = 0;
  p->n_items = 1;
  p->sub_w = u.w;
  p->sub_h = u.h;
  p->sx = 1;
  if (u.w < 4 || u.h < 4 || u.w > 128 || u.h > 128 || (u.w & 3) || (u.h & 3) || (u.x & 3) || (u.y & 3) || u.x < 0 ||
      u.y < 0 || u.x > t.W - u.w || u.y > t.H - u.h) {
    p->code = MM_ERR_ARG;
    return;
  }
  // unknown flag bits and nonzero reserved words (a stale 48-byte descriptor layout) fail loudly
  if (u.reserved[0] | u.reserved[1] | (int)(u.flags & ~MM_PUF_DMVR) | (int)((u.flags & MM_PUF_DMVR) && !t.dmvr)) {
    p->code = MM_ERR_ARG;
    return;
  }
  if (u.flags & MM_PUF_DMVR) {
    // the parts of PU::checkDMVRCondition (UnitTools.cpp:1698-1726) the descriptor carries: bi, equal
    // models, BCW_DEFAULT, w, h >= 8, w * h >= 128; sub-PUs tile the PU (16-multiples beyond 16)
    if (u.w < 8 || u.h < 8 || u.w * u.h < 128 || (u.w > 16 && (u.w & 15)) || (u.h > 16 && (u.h & 15)) ||
        u.ref_poc[0] < 0 || u.ref_poc[1] < 0 || u.model[0] != u.model[1] || u.bcw_idx != MM_BCW_DEFAULT ||
        t.only_list >= 0) {
      p->code = MM_ERR_ARG;
      return;
    }
    p->dmvr = 1;
    p->sub_w = u.w < 16 ? u.w : 16;
    p->sub_h = u.h < 16 ? u.h : 16;
    p->sx = u.w / p->sub_w;
    p->n_items = p->sx * (u.h / p->sub_h);
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
    int s = -1, cam = -1;  // the tables are read at uniform indices (no per-lane index into the argument)
    for (int k = 0; k < t.n_slots; k++)
      if (t.poc[k] == u.ref_poc[l]) {
        s = k;
        int c = t.ged_cam[0][k];
#pragma unroll
        for (int q = 1; q < MAX_PICS; q++) c = seg == q ? t.ged_cam[q][k] : c;
        cam = c;
      }
    if (s < 0) {
      p->code = MM_ERR_NOREF;
      return;
    }
    p->slot[l] = s;
    int ged = -1;
    if (m == GEODESIC_CAMPOSE) {
      if (cam < 0) {
        p->code = MM_ERR_NOEPIPOLE;
        return;
      }
      ged = cam;
    } else if (m >= GEODESIC_X && m <= GEODESIC_Z) {
      ged = m - GEODESIC_X;
    }
#pragma unroll
    for (int comp = 0; comp < 2; comp++) {
      if (comp == 1 && !t.chroma) continue;
      if (comp == 1 && mpa_chroma_aliases(t, m, p->sub_w, p->sub_h)) {
        p->alias[l] = 1;
        continue;
      }
      const int sb = comp ? 2 : 4;
      JobPlan& j = p->job[2 * l + comp];
      j.valid = 1;
      j.cw = p->sub_w >> comp;
      j.ch = p->sub_h >> comp;
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
  p->key = pu_key(u.x, t.W);
}


MM_HD unsigned long long status_word(int pu_index, int code) {
  return ~(((unsigned long long)(unsigned)pu_index << 8) | (unsigned)code);  // atomicMax keeps the lowest PU
}

MM_HD unsigned long long pack_count(int items, int elems) {
  return ((unsigned long long)(unsigned)elems << 32) | (unsigned)items;
}
MM_HD int packed_items(unsigned long long v) { return (int)(v & 0xffffffffull); }
MM_HD int packed_elems(unsigned long long v) { return (int)(v >> 32); }

// The bucket counts one classified PU adds: (items, elements) of its PU bucket, of each job key, and
// of the DMVR bucket (sub-PU records, cost elements)
MM_HD unsigned long long pu_count(const PuPlan& p) { return pack_count(p.n_items, p.n_sb); }
MM_HD unsigned long long job_count(const PuPlan& p, int k) { return pack_count(p.n_items, p.n_items * p.job[k].n); }
MM_HD unsigned long long dmvr_count(const PuPlan& p) {
  return pack_count(p.n_items, p.n_items * N_OFF * (p.sub_w / 4) * (p.sub_h / 4));
}

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
  band_cut(m->sb_base, m->n_sb, m->band);
  acc = sacc = 0;
  for (int k = 0; k < N_JOB_KEYS; k++) {
    m->job_base[k] = acc;
    m->elem_base[k] = sacc;
    acc += packed_items(c.job_tot[k]);
    sacc += packed_elems(c.job_tot[k]);
  }
  m->n_jobs = acc;
  m->n_elems = sacc;
  m->n_sub = packed_items(c.dmvr_tot);
  m->n_dmvr_elems = packed_elems(c.dmvr_tot);
}

// Item `idx` covers flat elements [off, off + n): it starts every 64-element chunk whose first
// element it holds (find_item's chunk table).
MM_HD void write_chunks(int* chunk, int idx, int off, int n) {
  for (int e = (off + 63) & ~63; e < off + n; e += 64) chunk[e >> 6] = idx;
}

// Emit the jobs of the PU placed at luma sub-block offset sb_off; job_idx/job_elem_off are the
// placed positions of the valid p.job[k].  The PU itself needs no record: its luma job of the
// first used list writes the per-sub-block meta word k_mc reads (JobDev::meta_hi).
// An MM_PUF_DMVR PU is emitted as its p.n_items sub-PUs in raster order (InterPrediction.cpp:
// 2481-2484): sub-PU s takes job job_idx[k] + s of every key, its sub-blocks follow sub-PU s - 1's,
// and its DMVR record (merge MVs, the indices of its jobs) goes to sub_idx + s, with its cost
// elements at sub_elem_off + s * N_OFF * n.
MM_HD void emit_pu(const mm_pu_desc& u, const PuPlan& p, int sb_off, const int* job_idx, const int* job_elem_off,
                   JobDev* jobs, int* job_off, int* job_chunk, int sub_idx = 0, int sub_elem_off = 0,
                   SubPuDev* subs = nullptr, int* sub_off = nullptr, int* sub_chunk = nullptr) {
  const int primary = p.cls == 2 ? 1 : 0;
  const int meta_hi = (p.slot[0] < 0 ? 0 : p.slot[0]) | ((p.slot[1] < 0 ? 0 : p.slot[1]) << 4) | (p.bcw << 8) |
                      (p.slot[0] >= 0 ? MM_META_USE0 : 0) | (p.slot[1] >= 0 ? MM_META_USE1 : 0) |
                      (p.seg << MM_META_SEG_SHIFT);
  const int n_sb_sub = (p.sub_w / 4) * (p.sub_h / 4);
  for (int s = 0; s < p.n_items; s++) {
    const int x = u.x + (s % p.sx) * p.sub_w, y = u.y + (s / p.sx) * p.sub_h;
    int jk[4] = {-1, -1, -1, -1};
    for (int i = 0; i < 4; i++) {
      const JobPlan& jp = p.job[i];
      if (!jp.valid) continue;
      JobDev j;
      j.x = x;
      j.y = y;
      j.cw = jp.cw;
      j.ch = jp.ch;
      j.comp = jp.comp;
      j.model = jp.model;
      j.mv_hor = jp.mv_hor;
      j.mv_ver = jp.mv_ver;
      j.ged_idx = jp.ged_idx;
      j.n = jp.n;
      j.rows = jp.rows;
      j.offset = job_elem_off[i] + s * jp.n;
      j.sb_base = sb_off + s * n_sb_sub;
      j.pu_cols = p.sub_w / 4;
      j.list = jp.list;
      j.slot = p.slot[jp.list];
      j.alias = jp.comp == 0 ? p.alias[jp.list] : 0;
      j.meta_hi = meta_hi | ((jp.comp == 0 && jp.list == primary) ? MM_META_PRIMARY : 0);
      jk[i] = job_idx[i] + s;
      jobs[jk[i]] = j;
      job_off[jk[i]] = j.offset;
      write_chunks(job_chunk, jk[i], j.offset, jp.n);
    }
    if (p.dmvr) {
      SubPuDev d;
      d.x = x;
      d.y = y;
      d.w = p.sub_w;
      d.h = p.sub_h;
      for (int l = 0; l < 2; l++) {
        d.mv[l][0] = u.mv[l][0];
        d.mv[l][1] = u.mv[l][1];
        d.ref_poc[l] = u.ref_poc[l];
        d.slot[l] = p.slot[l];
        d.ged_idx[l] = p.job[2 * l].ged_idx;
      }
      d.model = u.model[0];
      d.n = n_sb_sub;
      d.rows = p.sub_h / 4;
      d.elem_off = sub_elem_off + s * N_OFF * n_sb_sub;
      for (int k = 0; k < 4; k++) d.jidx[k] = jk[k];
      subs[sub_idx + s] = d;
      sub_off[sub_idx + s] = d.elem_off;
      write_chunks(sub_chunk, sub_idx + s, d.elem_off, N_OFF * n_sb_sub);
    }
  }
}

}  // namespace mmdev
