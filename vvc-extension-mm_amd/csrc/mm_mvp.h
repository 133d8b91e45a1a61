// mm_mvp.h -- MM motion-vector prediction across motion models (host + device bodies).
//
// MVReprojection::motionVectorInDesiredMotionModel (CommonLib/MVReprojection.cpp:168-217): a
// neighbouring / collocated candidate's MV, given in its own motion model, is converted into the
// MV of the current PU's model that shifts `position` to the same place.  The candidate's
// modelMotion runs on a 1x1 array (N = 1, so every operation is Eigen's scalar path), then the
// desired model's motionVectorForEquivalentPixelShiftAt (scalar Array2/Array3 code) inverts it.
// The reference calls this per candidate inside the merge / AMVP list derivation (UnitTools.cpp
// call sites); here a whole batch of candidates is converted at once.
#pragma once
#include "../../include/mm360.h"
#include "mm_models.h"

namespace mmmvp {
using namespace mmmod;

// The available entries of the context's EpipoleList in key order (std::map<(cur, ref)> order),
// resident on the device so that queries resolve their GEODESIC_CAMPOSE epipole where they are.
struct EpiDev {
  int32_t cur, ref;
  int32_t q[3];  // Q24
};
struct EpiTable {
  const EpiDev* e;
  int n;
};

// lexicographic (cur, ref) order of std::pair<int, int>
MM_HD bool epi_key_less(int c0, int r0, int c1, int r1) { return c0 < c1 || (c0 == c1 && r0 < r1); }
MM_HD int epi_lookup_exact(const EpiTable& t, int cur, int ref) {
  int lo = 0, hi = t.n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (epi_key_less(t.e[mid].cur, t.e[mid].ref, cur, ref))
      lo = mid + 1;
    else
      hi = mid;
  }
  return (lo < t.n && t.e[lo].cur == cur && t.e[lo].ref == ref) ? lo : -1;
}
// EpipoleList::findEpipoleFixed (EpipoleList.cpp:19-36): (cur, ref), then (cur, -1), then (-1, -1),
// available entries only (the table holds no other); -1 where the reference CHECKs
MM_HD int epi_find(const EpiTable& t, int cur, int ref) {
  int i = epi_lookup_exact(t, cur, ref);
  if (i < 0) i = epi_lookup_exact(t, cur, -1);
  if (i < 0) i = epi_lookup_exact(t, -1, -1);
  return i;
}

// GED rotation of one side of a query (MVReprojection.cpp:44-52 fixed epipoles for GEODESIC_X/Y/Z,
// EpipoleList::findEpipole + GeodesicMotionModel::setEpipole for CAMPOSE).  *entry: the CAMPOSE
// table entry (-1 otherwise).  false: CAMPOSE without an epipole.
MM_HD bool mvp_ged(const EpiTable& t, int model, int cur, int ref, M3* rot, int* entry) {
  *entry = -1;
  V3 e;
  if (model == GEODESIC_X)
    e = {1.0f, 0.0f, 0.0f};
  else if (model == GEODESIC_Y)
    e = {0.0f, 1.0f, 0.0f};
  else if (model == GEODESIC_Z)
    e = {0.0f, 0.0f, 1.0f};
  else if (model == GEODESIC_CAMPOSE) {
    const int k = epi_find(t, cur, ref);
    if (k < 0) return false;
    *entry = k;
    e = {fixed_to_float(t.e[k].q[0], 24), fixed_to_float(t.e[k].q[1], 24), fixed_to_float(t.e[k].q[2], 24)};
  } else {
    return true;
  }
  *rot = ged_rotation(e);
  return true;
}

// The argument checks of one query (the reference CHECKs / preconditions): MM_OK, MM_ERR_MODEL or
// MM_ERR_ARG.  Models: CLASSIC is always active.
MM_HD int mvp_validate(const mm_mvp_query& x, uint32_t active) {
  const int ms[2] = {x.model_orig, x.model_desired};
  for (int k = 0; k < 2; k++) {
    const int m = ms[k];
    if (m < CLASSIC || m >= NUM_MODELS || !((active | 1u) & (1u << m))) return MM_ERR_MODEL;
  }
  if (x.shift_hor < 0 || x.shift_hor > 8 || x.shift_ver < 0 || x.shift_ver > 8 || x.cand_w <= 0 || x.cand_h <= 0 ||
      x.cur_w <= 0 || x.cur_h <= 0)
    return MM_ERR_ARG;
  return MM_OK;
}

// The early returns of motionVectorInDesiredMotionModel (MVReprojection.cpp:172-181): a zero MV,
// or equal models (for GEODESIC_CAMPOSE only with equal epipoles).  Needs no epipole unless both
// sides are CAMPOSE.  Returns true and writes o[] when one applies; *code = MM_ERR_NOEPIPOLE when
// the comparison of the two CAMPOSE epipoles finds none.
MM_HD bool mvp_early(const mm_mvp_query& x, const EpiTable& t, int32_t* o, int* code) {
  *code = MM_OK;
  if (x.mv_hor == 0 && x.mv_ver == 0) {
    o[0] = o[1] = 0;
    return true;
  }
  if (x.model_desired != x.model_orig) return false;
  if (x.model_desired == GEODESIC_CAMPOSE) {
    const int eo = epi_find(t, x.cur_poc_orig, x.ref_poc_orig), ed = epi_find(t, x.cur_poc_desired, x.ref_poc_desired);
    if (eo < 0 || ed < 0) {
      *code = MM_ERR_NOEPIPOLE;
      return true;
    }
    if (!(t.e[eo].q[0] == t.e[ed].q[0] && t.e[eo].q[1] == t.e[ed].q[1] && t.e[eo].q[2] == t.e[ed].q[2])) return false;
  }
  o[0] = x.mv_hor;
  o[1] = x.mv_ver;
  return true;
}

// Scalar ERP toSphere / fromSphere (Projection.cpp Array2TCoord / Array3TCoord overloads)
MM_HD V3 erp_to_sphere1(float x, float y, const SeqConst& s) { return erp_to_sphere(x, y, s, Math{0}); }

// *MotionModel::motionVectorForEquivalentPixelShiftAt for the desired model
MM_HD void equivalent_mv(const SeqConst& s, int model, const M3* ged, float px, float py, float sx, float sy,
                         float cx, float cy, float* mvx, float* mvy) {
  const Math m{0};
  switch (model) {
    case CLASSIC:  // TranslationalMotionModel.cpp:15-18
      *mvx = sx - px;
      *mvy = sy - py;
      return;
    case MPA_FRONT_BACK:
    case MPA_LEFT_RIGHT:
    case MPA_TOP_BOTTOM: {  // MotionPlaneAdaptiveMotionModel.cpp:76-100, scalar toPerspective :137-161
      float ox, oy, qx, qy;
      bool vo, vq;
      mpa_to_perspective(model, px, py, s, m, &ox, &oy, &vo, false);
      mpa_to_perspective(model, sx, sy, s, m, &qx, &qy, &vq, false);
      if (vo != vq) {  // switched between the real and the virtual image plane
        *mvx = 0.0f;
        *mvy = 0.0f;
        return;
      }
      const float sign = vq ? -1.0f : 1.0f;
      *mvx = (qx - ox) * sign;
      *mvy = (qy - oy) * sign;
      return;
    }
    case TANGENTIAL: {  // TangentialMotionModel.cpp:50-85 (std::sin / std::cos on floats)
      const V3 spc = cart_to_sph(erp_to_sphere1(cx, cy, s), m, false);
      const float epsC = PI_2_F - spc.y, alphaC = spc.z;
      const V3 sp0 = cart_to_sph(erp_to_sphere1(px, py, s), m, false);
      const V3 sp1 = cart_to_sph(erp_to_sphere1(sx, sy, s), m, false);
      float xs[2], ys[2];
      const V3* sps[2] = {&sp0, &sp1};
      for (int k = 0; k < 2; k++) {
        const float eps = PI_2_F - sps[k]->y, alpha = sps[k]->z;
        const float dA = alpha - alphaC;
        const float sEc = g_sinf(epsC), cEc = g_cosf(epsC), se = g_sinf(eps), ce = g_cosf(eps), cdA = g_cosf(dA);
        const float cosPsi = sEc * se + (cEc * ce) * cdA;
        ys[k] = (se * cEc - (sEc * ce) * cdA) / cosPsi;
        xs[k] = (g_sinf(dA) * ce) / cosPsi;
      }
      *mvx = (xs[0] - xs[1]) / s.res;
      *mvy = (ys[0] - ys[1]) / s.res;
      return;
    }
    case THREE_D_TRANSLATIONAL: {  // ThreeDTranslationalMotionModel.cpp:26-38
      const V3 c3c = erp_to_sphere1(cx, cy, s);
      const V3 c3 = erp_to_sphere1(px, py, s);
      const V3 c3m = erp_to_sphere1(sx, sy, s);
      const V3 cm = {(c3m.x - c3.x) + c3c.x, (c3m.y - c3.y) + c3c.y, (c3m.z - c3.z) + c3c.z};
      float ox, oy;
      erp_from_sphere(cm, s, m, false, &ox, &oy);
      *mvx = ox - cx;
      *mvy = oy - cy;
      return;
    }
    case ROTATIONAL: {  // RotationalMotionModel.cpp:80-101
      const V3 spc = cart_to_sph(erp_to_sphere1(cx, cy, s), m, false);
      const V3 c3 = erp_to_sphere1(px, py, s);
      const V3 c3m = erp_to_sphere1(sx, sy, s);
      const M3 unrotPhi = angle_axis(-spc.z, 0.0f, 0.0f, 1.0f);
      const M3 unrotTheta = angle_axis((float)(PI_2_D - (double)spc.y), 0.0f, 1.0f, 0.0f);
      const M3 R = mat_mul(unrotTheta, unrotPhi);
      const V3 a = cart_to_sph(mat_vec(R, c3), m, false);
      const V3 am = cart_to_sph(mat_vec(R, c3m), m, false);
      *mvx = (a.z - am.z) / s.res;
      *mvy = (am.y - a.y) / s.res;
      return;
    }
    case GEODESIC_X:
    case GEODESIC_Y:
    case GEODESIC_Z:
    case GEODESIC_CAMPOSE: {  // GeodesicMotionModel.cpp:178-221
      const V3 sp = cart_to_sph(mat_vec(*ged, erp_to_sphere1(px, py, s)), m, false);
      const V3 spm = cart_to_sph(mat_vec(*ged, erp_to_sphere1(sx, sy, s)), m, false);
      if (s.ged_flavor == 0) {
        *mvx = (spm.y - sp.y) / s.res;
      } else {
        const V3 spc = cart_to_sph(mat_vec(*ged, erp_to_sphere1(cx, cy, s)), m, false);
        const float dTheta = spm.y - sp.y;
        const float k = g_sinf(dTheta + sp.y) / g_sinf(dTheta);
        const float dThetaC = g_atanf(g_sinf(spc.y) / (k - g_cosf(spc.y)));
        *mvx = dThetaC / s.res;
      }
      *mvy = (spm.z - sp.z) / s.res;
      return;
    }
    default:
      *mvx = *mvy = 0.0f;
  }
}

// Step 1 of motionVectorInDesiredMotionModel: the candidate's modelMotion on the 1x1 array
// {position}, centred on the candidate block (MVReprojection.cpp:183-197).  false: no epipole.
MM_HD bool mvp_candidate_motion(const SeqConst& s, const mm_mvp_query& q, const EpiTable& t, float* sx, float* sy) {
  M3 rot;
  int entry;
  if (!mvp_ged(t, q.model_orig, q.cur_poc_orig, q.ref_poc_orig, &rot, &entry)) return false;
  const float mvx = mv_to_float_shift(q.mv_hor, q.shift_hor), mvy = mv_to_float_shift(q.mv_ver, q.shift_ver);
  BlockSetup b;
  block_setup_f(&b, s, q.model_orig, false, q.cand_x, q.cand_y, q.cand_w, q.cand_h, mvx, mvy, &rot);
  model_motion_element(s, b, (float)q.pos_x, (float)q.pos_y, false, false, 0.0f, 0.0f, false, sx, sy);
  return true;
}

// Step 2: the desired model's equivalent MV, centred on the current block, NaN -> zero MV,
// std::round to fixed point (MVReprojection.cpp:199-216).  false: no epipole.
MM_HD bool mvp_desired_mv(const SeqConst& s, const mm_mvp_query& q, const EpiTable& t, float sx, float sy, int32_t* o) {
  M3 rot;
  int entry;
  if (!mvp_ged(t, q.model_desired, q.cur_poc_desired, q.ref_poc_desired, &rot, &entry)) return false;
  const float cx = (float)q.cur_x + ((float)q.cur_w - 1.0f) / 2.0f;
  const float cy = (float)q.cur_y + ((float)q.cur_h - 1.0f) / 2.0f;
  float ex, ey;
  equivalent_mv(s, q.model_desired, &rot, (float)q.pos_x, (float)q.pos_y, sx, sy, cx, cy, &ex, &ey);
  if (isnanf_(ex) || isnanf_(ey)) {
    o[0] = o[1] = 0;
    return true;
  }
  const float rx = roundf_(ex * (float)(1 << q.shift_hor)), ry = roundf_(ey * (float)(1 << q.shift_ver));
  o[0] = (fabsf_(rx) < 2147483648.0f) ? (int32_t)rx : (int32_t)0x80000000u;  // static_cast<int>
  o[1] = (fabsf_(ry) < 2147483648.0f) ? (int32_t)ry : (int32_t)0x80000000u;
  return true;
}

// motionVectorInDesiredMotionModel for one query (host twin; the kernel runs the same steps with
// its queries regrouped by model between the steps).  Returns MM_OK or the query's error code.
MM_HD int mvp_query(const SeqConst& s, const mm_mvp_query& q, uint32_t active, const EpiTable& t, int32_t* o) {
  o[0] = o[1] = 0;
  int code = mvp_validate(q, active);
  if (code) return code;
  if (mvp_early(q, t, o, &code)) return code;
  float sx, sy;
  if (!mvp_candidate_motion(s, q, t, &sx, &sy)) return MM_ERR_NOEPIPOLE;
  if (!mvp_desired_mv(s, q, t, sx, sy, o)) return MM_ERR_NOEPIPOLE;
  return MM_OK;
}

}  // namespace mmmvp
