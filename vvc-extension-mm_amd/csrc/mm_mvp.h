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

struct MvpQueryDev {
  mm_mvp_query q;
  int ged_orig, ged_desired;  // GED rotation table index per side, -1 if not GED
  int same_epipole;           // both GEODESIC_CAMPOSE epipoles equal (findEpipole == findEpipole)
};

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

// motionVectorInDesiredMotionModel for one query -> fixed-point MV (shift_hor / shift_ver bits)
MM_HD void mvp_thread(int t, const SeqConst& s, const MvpQueryDev* qs, const M3* ged, int32_t* out) {
  const MvpQueryDev& d = qs[t];
  const mm_mvp_query& q = d.q;
  int32_t* o = out + 2 * t;
  if (q.mv_hor == 0 && q.mv_ver == 0) {
    o[0] = o[1] = 0;
    return;
  }
  if (q.model_desired == q.model_orig && (q.model_desired != GEODESIC_CAMPOSE || d.same_epipole)) {
    o[0] = q.mv_hor;
    o[1] = q.mv_ver;
    return;
  }
  const float mvx = mv_to_float_shift(q.mv_hor, q.shift_hor), mvy = mv_to_float_shift(q.mv_ver, q.shift_ver);
  // candidate's modelMotion on the 1x1 array {position}, centred on the candidate block
  BlockSetup b;
  block_setup_f(&b, s, q.model_orig, false, q.cand_x, q.cand_y, q.cand_w, q.cand_h, mvx, mvy,
                d.ged_orig >= 0 ? &ged[d.ged_orig] : nullptr);
  float sx, sy;
  model_motion_element(s, b, (float)q.pos_x, (float)q.pos_y, false, false, 0.0f, 0.0f, false, &sx, &sy);
  // desired model's equivalent MV, centred on the current block
  const float cx = (float)q.cur_x + ((float)q.cur_w - 1.0f) / 2.0f;
  const float cy = (float)q.cur_y + ((float)q.cur_h - 1.0f) / 2.0f;
  float ex, ey;
  equivalent_mv(s, q.model_desired, d.ged_desired >= 0 ? &ged[d.ged_desired] : nullptr, (float)q.pos_x,
                (float)q.pos_y, sx, sy, cx, cy, &ex, &ey);
  if (isnanf_(ex) || isnanf_(ey)) {
    o[0] = o[1] = 0;
    return;
  }
  const float rx = roundf_(ex * (float)(1 << q.shift_hor)), ry = roundf_(ey * (float)(1 << q.shift_ver));
  o[0] = (fabsf_(rx) < 2147483648.0f) ? (int32_t)rx : (int32_t)0x80000000u;  // static_cast<int>
  o[1] = (fabsf_(ry) < 2147483648.0f) ? (int32_t)ry : (int32_t)0x80000000u;
}

}  // namespace mmmvp
