// mm_models.h -- per-sub-block restatement of the reference's ERP projection and the five
// 360-degree motion models, written once for host and device.
//
// The reference evaluates each model on Eigen arrays holding one element per 4x4 luma
// (2x2 chroma) sub-block (MVReprojection::reprojectMotionVectorSubblocks,
// source/Lib/CommonLib/MVReprojection.cpp:80-166).  Element-wise every array expression is a
// fixed sequence of float32 operations; the only cross-element effect is Eigen's packet/tail
// split (elements [0, N - N%4) evaluated with SSE packets), which decides per expression
// whether sin/cos/sqrt are the Cephes packet kernels or glibc scalar calls.
// Here one call evaluates one element; the caller passes `packet` for that element.
//
// File:line citations are into /root/reference/source/Lib/CommonLib.
#pragma once
#include "mm_numerics.h"

namespace mmmod {
using namespace mmnum;

// MotionModelID (TypeDef.h:865-879)
enum ModelId : int {
  CLASSIC = 0,
  MPA_FRONT_BACK = 1,
  MPA_LEFT_RIGHT = 2,
  MPA_TOP_BOTTOM = 3,
  TANGENTIAL = 4,
  THREE_D_TRANSLATIONAL = 5,
  ROTATIONAL = 6,
  GEODESIC_X = 7,
  GEODESIC_Y = 8,
  GEODESIC_Z = 9,
  GEODESIC_CAMPOSE = 10,
  NUM_MODELS = 11
};

constexpr float PI_F = 3.14159274101257324f;     // TCoord(M_PI)
constexpr float TWO_PI_F = 6.28318548202514648f;  // TCoord(2) * TCoord(M_PI)
constexpr float PI_2_F = 1.57079637050628662f;    // float(M_PI_2) (double constant in array expr)
constexpr double PI_2_D = 1.57079632679489661923;  // M_PI_2

struct V3 {
  float x, y, z;
};

// Sequence constants (MVReprojection::init, MVReprojection.cpp:7-65; Projection.h:127-130)
struct SeqConst {
  float Wf, Hf;    // luma picture width/height as float
  float off;       // m_offset4x4 (code 4 -> 1.5)
  float focal;     // float(1. / tan(M_PI / H)) -- ERP focal, reused by MPA's perspective
  float res;       // float(M_PI / H) -- angle resolution of TAN/ROT/GED
  int ged_flavor;  // 0 VISHWANATH_ORIGINAL, 1 VISHWANATH_MODULATED (EncApp.cpp:755 hard-codes 1)
};

// ------------------------------------------------------------------------------------------
// Coordinate conversions (Coordinate.cpp).  `arr` selects the Eigen array form (clamp as
// cwiseMin(1).cwiseMax(-1): NaN passes through) versus the scalar Array3 form (std::max then
// std::min: NaN -> -1).
// ------------------------------------------------------------------------------------------
MM_HD float clamp_unit_(float v, bool arr) {
  if (arr) {
    v = (1.0f < v) ? 1.0f : v;    // std::min(v, 1)
    v = (v < -1.0f) ? -1.0f : v;  // std::max(v, -1)
    return v;
  }
  float w = (-1.0f < v) ? v : -1.0f;  // std::max(-1, v)
  return (w < 1.0f) ? w : 1.0f;       // std::min(1, w)
}

// cartesianToSpherical (Coordinate.cpp:32-38 array / :40-45 scalar): returns R, theta, phi
MM_HD V3 cart_to_sph(V3 p, Math m, bool arr) {
  float R = m.sqrt((p.x * p.x + p.y * p.y) + p.z * p.z);
  float th = g_acosf(clamp_unit_(p.z / R, arr));
  float ph = g_atan2f(p.y, p.x);
  return {R, th, ph};
}

// sphericalToCartesian with explicit R (Coordinate.cpp:47-53)
MM_HD V3 sph_to_cart(float R, float th, float ph, Math m) {
  float st = m.sin(th);
  return {(R * st) * m.cos(ph), (R * st) * m.sin(ph), R * m.cos(th)};
}

// ------------------------------------------------------------------------------------------
// EquirectangularProjection (Projection.cpp:213-249 in SURVEY numbering; pixelOffset = 0)
// ------------------------------------------------------------------------------------------
MM_HD float erp_phi(float x, const SeqConst& s) { return ((-((x + 0.0f) / s.Wf)) * 2.0f) * PI_F; }
MM_HD float erp_theta(float y, const SeqConst& s) { return ((y + 0.0f) / s.Hf) * PI_F; }
MM_HD V3 erp_to_sphere(float x, float y, const SeqConst& s, Math m) {
  return sph_to_cart(1.0f, erp_theta(y, s), erp_phi(x, s), m);
}
// The same point from precomputed (sin, cos) of theta and phi: sph_to_cart(1, theta, phi)
MM_HD V3 sph_from_trig(float st, float ct, float sp, float cp) { return {(1.0f * st) * cp, (1.0f * st) * sp, 1.0f * ct}; }

MM_HD void erp_from_sphere(V3 p, const SeqConst& s, Math m, bool arr, float* ox, float* oy) {
  V3 sp = cart_to_sph(p, m, arr);
  float phi = sp.z > 0.0f ? sp.z - TWO_PI_F : sp.z;
  *ox = ((-(phi / TWO_PI_F)) * s.Wf) - 0.0f;
  *oy = ((sp.y / PI_F) * s.Hf) - 0.0f;
}

// ------------------------------------------------------------------------------------------
// PerspectiveProjection, optical centre (0,0) (Projection.cpp:119-211 in SURVEY numbering)
// ------------------------------------------------------------------------------------------
MM_HD void persp_from_sphere(V3 s3, float f, Math m, float* ox, float* oy, bool* vip, bool arr = true) {
  V3 rot = {s3.y, -s3.z, -s3.x};
  V3 sp = cart_to_sph(rot, m, arr);
  float polarR = f * g_tanf(sp.y);
  *ox = polarR * m.cos(sp.z) + 0.0f;
  *oy = polarR * m.sin(sp.z) + 0.0f;
  *vip = polarR < 0.0f;
}

MM_HD V3 persp_to_sphere(float x, float y, bool vip, const SeqConst& s, Math m) {
  x = x - 0.0f;
  y = y - 0.0f;
  float r = m.sqrt(x * x + y * y);
  float phi = g_atan2f(y, x);
  float theta = g_atanf(r / s.focal);
  float v = vip ? 1.0f : 0.0f;
  theta = theta - v * (2.0f * theta - PI_F);
  phi = phi - v * PI_F;
  V3 c = sph_to_cart(1.0f, theta, phi, m);
  return {-c.z, c.x, -c.y};
}

// MotionPlaneAdaptiveMotionModel::toPerspective (array, MotionPlaneAdaptiveMotionModel.cpp:111-135)
MM_HD void mpa_to_perspective(int plane, float gx, float gy, const SeqConst& s, Math m, float* px,
                              float* py, bool* vip, bool arr = true) {
  V3 sph = erp_to_sphere(gx, gy, s, m);
  V3 q;
  if (plane == MPA_FRONT_BACK)
    q = sph;
  else if (plane == MPA_LEFT_RIGHT)
    q = {sph.y, -sph.x, sph.z};
  else
    q = {-sph.z, sph.y, sph.x};
  persp_from_sphere(q, s.focal, m, px, py, vip, arr);
}

// toPerspective of one element outside the frame cache (MPA chroma blocks that do not alias the
// luma job, Eigen tail lanes): out of line, the per-picture path rarely takes it
MM_HD_COLD void mpa_to_perspective_cold(int plane, float gx, float gy, const SeqConst& s, int packet, float* px,
                                        float* py, bool* vip) {
  mpa_to_perspective(plane, gx, gy, s, Math{packet}, px, py, vip);
}

// MotionPlaneAdaptiveMotionModel::toProjection (array, MotionPlaneAdaptiveMotionModel.cpp:163-187)
MM_HD void mpa_to_projection(int plane, float px, float py, bool vip, const SeqConst& s, Math m,
                             float* ox, float* oy) {
  V3 q = persp_to_sphere(px, py, vip, s, m);
  V3 sph;
  if (plane == MPA_FRONT_BACK)
    sph = q;
  else if (plane == MPA_LEFT_RIGHT)
    sph = {-q.y, q.x, q.z};
  else
    sph = {q.z, q.y, -q.x};
  erp_from_sphere(sph, s, m, true, ox, oy);
}

// ------------------------------------------------------------------------------------------
// 3x3 products: Eigen 3.3.7 lazy coefficient-based product, coefficient = p0 + (p1 + p2)
// (redux_novec_unroller halves).  Row-major storage m[3*i + j].
// ------------------------------------------------------------------------------------------
struct M3 {
  float m[9];
};
MM_HD float dot3_(float a0, float b0, float a1, float b1, float a2, float b2) {
#if MM_PROD3_MODE
  return (a0 * b0 + a1 * b1) + a2 * b2;
#else
  return a0 * b0 + (a1 * b1 + a2 * b2);
#endif
}
MM_HD M3 mat_mul(const M3& A, const M3& B) {
  M3 C;
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++)
      C.m[3 * i + j] = dot3_(A.m[3 * i], B.m[j], A.m[3 * i + 1], B.m[3 + j], A.m[3 * i + 2], B.m[6 + j]);
  return C;
}
MM_HD V3 mat_vec(const M3& A, V3 v) {
  return {dot3_(A.m[0], v.x, A.m[1], v.y, A.m[2], v.z), dot3_(A.m[3], v.x, A.m[4], v.y, A.m[5], v.z),
          dot3_(A.m[6], v.x, A.m[7], v.y, A.m[8], v.z)};
}
MM_HD V3 matT_vec(const M3& A, V3 v) {
  return {dot3_(A.m[0], v.x, A.m[3], v.y, A.m[6], v.z), dot3_(A.m[1], v.x, A.m[4], v.y, A.m[7], v.z),
          dot3_(A.m[2], v.x, A.m[5], v.y, A.m[8], v.z)};
}
MM_HD M3 mat_transpose(const M3& A) {
  return {{A.m[0], A.m[3], A.m[6], A.m[1], A.m[4], A.m[7], A.m[2], A.m[5], A.m[8]}};
}

// Eigen 3.3.7 AngleAxis<float>::toRotationMatrix (Geometry/AngleAxis.h), axis given exactly
MM_HD M3 angle_axis(float angle, float ax, float ay, float az) {
  float s = g_sinf(angle), c = g_cosf(angle);
  float sx = s * ax, sy = s * ay, sz = s * az;
  float omc = 1.0f - c;
  float cx = omc * ax, cy = omc * ay, cz = omc * az;
  M3 r;
  float tmp = cx * ay;
  r.m[1] = tmp - sz;
  r.m[3] = tmp + sz;
  tmp = cx * az;
  r.m[2] = tmp + sy;
  r.m[6] = tmp - sy;
  tmp = cy * az;
  r.m[5] = tmp - sx;
  r.m[7] = tmp + sx;
  r.m[0] = cx * ax + c;
  r.m[4] = cy * ay + c;
  r.m[8] = cz * az + c;
  return r;
}

// GeodesicMotionModel::setEpipole (GeodesicMotionModel.cpp:14-46)
MM_HD M3 ged_rotation(V3 e) {
  float n = sqrtf_((e.x * e.x + e.y * e.y) + e.z * e.z);
  V3 pa = {e.x / n, e.y / n, e.z / n};
  V3 cr = {-pa.y, pa.x, 0.0f};
  float s = sqrtf_((cr.x * cr.x + cr.y * cr.y) + cr.z * cr.z);
  M3 R;
  if (s == 0.0f) {
    R = {{1, 0, 0, 0, 1, 0, 0, 0, 1}};
    if (pa.z < 0.0f) R.m[8] = -1.0f;
    return R;
  }
  float zmin = (pa.z < 1.0f) ? pa.z : 1.0f;         // std::min(TCoord(1), z)
  float c = (-1.0f < zmin) ? zmin : -1.0f;           // std::max(TCoord(-1), .)
  M3 K = {{0.0f, -cr.z, cr.y, cr.z, 0.0f, -cr.x, -cr.y, cr.x, 0.0f}};
  M3 K2 = mat_mul(K, K);
  float f = (1.0f - c) / (s * s);
  for (int i = 0; i < 9; i++) {
    float I = (i == 0 || i == 4 || i == 8) ? 1.0f : 0.0f;
    R.m[i] = (I + K.m[i]) + K2.m[i] * f;
  }
  return mat_transpose(R);
}

// EpipoleList::findEpipole -> FloatingFixedConversion::fixedToFloating(.., 24) (Coordinate.cpp:76-80)
MM_HD float fixed_to_float(int32_t v, int prec) {
  return (float)(v >> prec) + (float)(v & ((1 << prec) - 1)) / (float)(1 << prec);
}

// ------------------------------------------------------------------------------------------
// Per-block (per PU x list x component) setup: everything the reference computes once per
// reprojectMotionVectorSubblocks call, before the per-element arrays.
// ------------------------------------------------------------------------------------------
// 56 bytes: the per-model constants share M's storage (k_setup streams one record per job to
// HBM and k_reproj reads it back per element, so the record is kept to what any one model needs).
struct BlockSetup {
  int16_t model;
  int16_t identity;  // model returns the input grid unchanged (zero-MV shortcut)
  float mvx, mvy;    // motion vector as float (MVReprojection.cpp:123-124)
  M3 M;              // GED rotation (setEpipole) or ROT rotationMatrixReally; TAN: sE, cE, alphaC
                     // in m[0..2]; 3DT: the 3D motion vector in m[0..2]
  float k;           // GED MODULATED parameter
  float pad_;
};
static_assert(sizeof(BlockSetup) == 56, "BlockSetup is seven 8-byte words");
MM_HD float tan_sE(const BlockSetup& b) { return b.M.m[0]; }
MM_HD float tan_cE(const BlockSetup& b) { return b.M.m[1]; }
MM_HD float tan_alphaC(const BlockSetup& b) { return b.M.m[2]; }

MM_HD float mv_to_float(int32_t v) { return (float)(v >> 4) + (float)(v & 15) / 16.0f; }
// MV as floating point with `shift` fractional bits (MVReprojection.cpp:123-124, 185-186)
MM_HD float mv_to_float_shift(int32_t v, int shift) {
  return (float)(v >> shift) + (float)(v & ((1 << shift) - 1)) / (float)(1 << shift);
}

MM_HD void block_setup_f(BlockSetup* b, const SeqConst& s, int model, bool luma, int pos_x, int pos_y, int size_w,
                         int size_h, float mvx, float mvy, const M3* ged_rot);
MM_HD void block_setup(BlockSetup* b, const SeqConst& s, int model, bool luma, int pos_x, int pos_y,
                       int size_w, int size_h, int32_t mv_hor, int32_t mv_ver, const M3* ged_rot) {
  block_setup_f(b, s, model, luma, pos_x, pos_y, size_w, size_h, mv_to_float(mv_hor), mv_to_float(mv_ver), ged_rot);
}
// The MV-independent part of a block setup: what the model derives from the block centre alone
// (TAN: sin / cos of the centre's elevation complement and its azimuth; 3DT: the centre's sphere
// point; ROT: the un-rotation about the centre; GED MODULATED: the polar angle of the rotated centre).
// block_setup_f is centre_terms + setup_from_centre; MM-DMVR, whose 25 offsets share one centre,
// computes the centre terms once per (sub-PU, list) and only the MV part per offset.
struct CentreTerms {
  float t[9];
  float cx, cy;  // the block centre in component units (MVReprojection.cpp:133)
};
MM_HD void centre_terms(CentreTerms* ct, const SeqConst& s, int model, float cx, float cy, const M3* ged_rot) {
  for (int i = 0; i < 9; i++) ct->t[i] = 0.0f;
  ct->cx = cx;
  ct->cy = cy;
  const Math sc{false};
  switch (model) {
    case TANGENTIAL: {  // TangentialMotionModel.cpp:8-48
      V3 c3 = erp_to_sphere(cx, cy, s, sc);
      V3 sp = cart_to_sph(c3, sc, false);
      float epsC = (float)(PI_2_D - (double)sp.y);
      ct->t[2] = sp.z;  // alphaC
#if MM_TAN_CENTRE_MODE
      ct->t[0] = g_sinf(epsC);  // sE
      ct->t[1] = g_cosf(epsC);  // cE
#else
      ct->t[0] = sinf_via_double(epsC);  // sE: unqualified sin(float) -> double ::sin
      ct->t[1] = cosf_via_double(epsC);  // cE
#endif
    } break;
    case THREE_D_TRANSLATIONAL: {  // ThreeDTranslationalMotionModel.cpp:7-24
      V3 c = erp_to_sphere(cx, cy, s, sc);
      ct->t[0] = c.x;
      ct->t[1] = c.y;
      ct->t[2] = c.z;
    } break;
    case ROTATIONAL: {  // RotationalMotionModel.cpp:8-78
      V3 sp = cart_to_sph(erp_to_sphere(cx, cy, s, sc), sc, false);
      M3 unrotPhi = angle_axis(-sp.z, 0.0f, 0.0f, 1.0f);
      M3 unrotTheta = angle_axis((float)(PI_2_D - (double)sp.y), 0.0f, 1.0f, 0.0f);
      M3 unrot = mat_mul(unrotTheta, unrotPhi);
      for (int i = 0; i < 9; i++) ct->t[i] = unrot.m[i];
    } break;
    case GEODESIC_X:
    case GEODESIC_Y:
    case GEODESIC_Z:
    case GEODESIC_CAMPOSE:  // GeodesicMotionModel.cpp:101-176
      if (s.ged_flavor == 1) {
        V3 c3 = erp_to_sphere(cx, cy, s, sc);
        V3 cr = mat_vec(*ged_rot, c3);
        V3 sp = cart_to_sph(cr, sc, false);
        ct->t[0] = sp.y;
      }
      break;
    default:
      break;
  }
}
// The zero-MV shortcut of the models that have one (chroma only for GED: only modelMotion shortcuts)
MM_HD bool setup_is_identity(int model, bool luma, float mvx, float mvy) {
  const bool zero = (mvx == 0.0f && mvy == 0.0f);
  if (model == TANGENTIAL || model == THREE_D_TRANSLATIONAL || model == ROTATIONAL) return zero;
  if (model >= GEODESIC_X && model <= GEODESIC_CAMPOSE) return !luma && zero;
  return false;
}
// The setup at MV (mvx, mvy) from the block's centre terms
MM_HD void setup_from_centre(BlockSetup* b, const SeqConst& s, int model, bool luma, float mvx, float mvy,
                             const CentreTerms& ct, const M3* ged_rot) {
  b->model = (int16_t)model;
  b->mvx = mvx;
  b->mvy = mvy;
  b->identity = 0;
  b->k = 0.0f;
  b->pad_ = 0.0f;
  for (int i = 0; i < 9; i++) b->M.m[i] = 0.0f;
  if (model >= GEODESIC_X && model <= GEODESIC_CAMPOSE) b->M = *ged_rot;
  if (setup_is_identity(model, luma, mvx, mvy)) {
    b->identity = 1;
    return;
  }
  const Math sc{false};
  switch (model) {
    case TANGENTIAL:
      b->M.m[2] = ct.t[2];
      b->M.m[0] = ct.t[0];
      b->M.m[1] = ct.t[1];
      break;
    case THREE_D_TRANSLATIONAL: {
      V3 cm = erp_to_sphere(ct.cx + b->mvx, ct.cy + b->mvy, s, sc);
      b->M.m[0] = cm.x - ct.t[0];
      b->M.m[1] = cm.y - ct.t[1];
      b->M.m[2] = cm.z - ct.t[2];
    } break;
    case ROTATIONAL: {
      M3 rot = mat_mul(angle_axis(-b->mvx * s.res, 0.0f, 0.0f, 1.0f),
                       angle_axis(b->mvy * s.res, 0.0f, 1.0f, 0.0f));
      M3 unrot;
      for (int i = 0; i < 9; i++) unrot.m[i] = ct.t[i];
      M3 unrotT = mat_transpose(unrot);
      b->M = mat_mul(unrotT, mat_mul(rot, unrot));
    } break;
    case GEODESIC_X:
    case GEODESIC_Y:
    case GEODESIC_Z:
    case GEODESIC_CAMPOSE:
      if (s.ged_flavor == 1) {
        float rm = s.res * b->mvx;
        b->k = g_sinf(ct.t[0] + rm) / g_sinf(rm);
      }
      break;
    default:
      break;  // MPA: no shortcut, no per-block constants
  }
}
MM_HD void block_setup_f(BlockSetup* b, const SeqConst& s, int model, bool luma, int pos_x, int pos_y, int size_w,
                         int size_h, float mvx, float mvy, const M3* ged_rot) {
  // block centre in component units (MVReprojection.cpp:133)
  const float cx = (float)pos_x + ((float)size_w - 1.0f) / 2.0f;
  const float cy = (float)pos_y + ((float)size_h - 1.0f) / 2.0f;
  CentreTerms ct;
  if (setup_is_identity(model, luma, mvx, mvy)) {  // the centre is not needed
    for (int i = 0; i < 9; i++) ct.t[i] = 0.0f;
    ct.cx = cx;
    ct.cy = cy;
  } else {
    centre_terms(&ct, s, model, cx, cy, ged_rot);
  }
  setup_from_centre(b, s, model, luma, mvx, mvy, ct, ged_rot);
}

// ------------------------------------------------------------------------------------------
// One element of <Model>::modelMotion[Cached] followed by the NaN fallback and fixed-point
// rounding of reprojectMotionVectorSubblocks (MVReprojection.cpp:147-164).
//   gx, gy   : the element's grid coordinate (luma-scaled, incl. the 4x4 offset)
//   packet   : Eigen packet lane for this element within its block (N >= 4, index < N - N%4)
//   pers*    : MPA luma only -- the frame-cache perspective coordinates of this element
//   chroma_shift : 0 for luma, 1 for 4:2:0 chroma; fixed precision = 4 + chroma_shift bits
// ------------------------------------------------------------------------------------------
// <Model>::modelMotion[Cached] of one element: the moved position as computed (before the NaN
// fallback, offset removal and rounding).  CLASSIC (TranslationalMotionModel::modelMotion,
// TranslationalMotionModel.cpp:8-13) adds the MV.
// grid (optional, .valid): toSphere(gx, gy) of this element, taken from the separable per-column /
// per-row trig table of the frame grid (mm_pipeline.h MpaCache) -- the same values, computed once.
// Passed by value: a pointer to a caller's local would keep that local in scratch memory.
// tan (optional, .tan_valid): TAN's first step on this grid point -- (alpha, sin(eps), cos(eps)) of
// cartesianToSpherical(toSphere(grid)), eps = pi/2 - theta (TangentialMotionModel.cpp:16-22) -- from
// the per-grid-point table (mm_pipeline.h MpaCache::tan_grid): it depends only on the grid point and
// the element's packet flavour, not on the block.
struct GridSphere {
  V3 p;
  int valid;  // int, not bool (see Math)
  int tan_valid;
  float alpha, se, ce;
};
MM_HD GridSphere no_grid() {
  GridSphere g;
  g.p = {0.0f, 0.0f, 0.0f};
  g.valid = 0;
  g.tan_valid = 0;
  g.alpha = g.se = g.ce = 0.0f;
  return g;
}
// The TAN grid entry of sphere point p in flavour m (what model_motion_element computes first)
MM_HD void tan_grid_entry(V3 p, Math m, float* alpha, float* se, float* ce) {
  const V3 sp = cart_to_sph(p, m, true);
  const float eps = PI_2_F - sp.y;
  *alpha = sp.z;
  *se = m.sin(eps);
  *ce = m.cos(eps);
}
// model_motion_element in two parts.  The head is what does not depend on the block's MV: the
// element's sphere point and, for TAN, the tangent-plane coordinates (xP, yP) of the element about the
// block centre (the setup's sE, cE, alphaC come from the centre only), for GED the spherical
// coordinates of the rotated point (the setup's rotation M is the epipole's or the axis', whatever
// the MV).  A block searched over many MVs (MM-DMVR's offsets) computes the head once per element and
// the tail per MV; model_motion_element is head + tail, so both give the same bits.  The head needs
// a setup that is not the zero-MV identity (TAN leaves sE, cE, alphaC unset there).
struct MotionHead {
  V3 p;           // toSphere(grid) of TAN / 3DT / ROT / GED
  V3 ged_sp;      // GED: cart_to_sph(M p)
  float xP, yP;   // TAN: tangent-plane coordinates
  float se, ce;   // TAN: the element's sin / cos of its elevation complement
};
MM_HD MotionHead motion_head(const SeqConst& s, const BlockSetup& b, float gx, float gy, const Math& m,
                             const GridSphere& grid) {
  MotionHead h;
  h.p = {0.0f, 0.0f, 0.0f};
  h.ged_sp = {0.0f, 0.0f, 0.0f};
  h.xP = h.yP = h.se = h.ce = 0.0f;
  const bool mpa = b.model >= MPA_FRONT_BACK && b.model <= MPA_TOP_BOTTOM;
  if (b.model == CLASSIC || b.identity || b.model >= NUM_MODELS || mpa) return h;
  if (!grid.tan_valid) h.p = grid.valid ? grid.p : erp_to_sphere(gx, gy, s, m);
  if (b.model == TANGENTIAL) {  // TangentialMotionModel.cpp:8-48, up to the MV
    float alpha;
    if (grid.tan_valid) {
      alpha = grid.alpha;
      h.se = grid.se;
      h.ce = grid.ce;
    } else {
      tan_grid_entry(h.p, m, &alpha, &h.se, &h.ce);
    }
    const float sE = tan_sE(b), cE = tan_cE(b), alphaC = tan_alphaC(b);
    float dA = alpha - alphaC;
    float cdA = m.cos(dA);
    float cosPsi = sE * h.se + (cE * h.ce) * cdA;
    h.yP = (h.se * cE - (sE * h.ce) * cdA) / cosPsi;
    h.xP = (m.sin(dA) * h.ce) / cosPsi;
  } else if (b.model >= GEODESIC_X) {  // GeodesicMotionModel.cpp:101-176, up to the MV
    h.ged_sp = cart_to_sph(mat_vec(b.M, h.p), m, true);
  }
  return h;
}
MM_HD void motion_tail(const SeqConst& s, const BlockSetup& b, const MotionHead& h, float gx, float gy, const Math& m,
                       bool mpa_cached, float pers_x, float pers_y, bool pers_vip, float* omx, float* omy) {
  if (b.model == CLASSIC) {
    *omx = gx + b.mvx;
    *omy = gy + b.mvy;
    return;
  }
  if (b.identity || b.model >= NUM_MODELS) {
    *omx = gx;
    *omy = gy;
    return;
  }
  // Every model ends in EquirectangularProjection::fromSphere of a moved sphere point q; the
  // switch computes q and the shared tail projects it (one copy of the acosf/atan2f code).
  V3 q;
  switch (b.model) {
    case MPA_FRONT_BACK:
    case MPA_LEFT_RIGHT:
    case MPA_TOP_BOTTOM: {  // MotionPlaneAdaptiveMotionModel.cpp:26-74
      float px, py;
      bool vip;
      if (mpa_cached) {
        px = pers_x;
        py = pers_y;
        vip = pers_vip;
      } else {
        mpa_to_perspective_cold(b.model, gx, gy, s, m.packet, &px, &py, &vip);
      }
      float sign = vip ? -1.0f : 1.0f;
      px = px + b.mvx * sign;
      py = py + b.mvy * sign;
      // toProjection (:163-187) up to the ERP step
      V3 c = persp_to_sphere(px, py, vip, s, m);
      if (b.model == MPA_FRONT_BACK)
        q = c;
      else if (b.model == MPA_LEFT_RIGHT)
        q = {-c.y, c.x, c.z};
      else
        q = {c.z, c.y, -c.x};
    } break;
    case TANGENTIAL: {  // TangentialMotionModel.cpp:8-48, from the MV on
      const float sE = tan_sE(b), cE = tan_cE(b), alphaC = tan_alphaC(b);
      float yM = h.yP - b.mvy * s.res;
      float xM = h.xP - b.mvx * s.res;
      float rho = m.sqrt(xM * xM + yM * yM);
      float eta = g_atanf(rho);
      float gamma = (rho * cE) * m.cos(eta) - (yM * sE) * m.sin(eta);
      float alphaM = alphaC + g_atanf((xM * g_sinf(eta)) / gamma);
      float epsM = g_asinf(g_cosf(eta) * sE + ((yM * g_sinf(eta)) * cE) / rho);
      q = sph_to_cart(1.0f, PI_2_F - epsM, alphaM, m);
    } break;
    case THREE_D_TRANSLATIONAL:  // ThreeDTranslationalMotionModel.cpp:7-24
      q = {h.p.x + b.M.m[0], h.p.y + b.M.m[1], h.p.z + b.M.m[2]};  // 3D motion vector
      break;
    case ROTATIONAL:  // RotationalMotionModel.cpp:66-77
      q = mat_vec(b.M, h.p);
      break;
    default: {  // GEODESIC_X/Y/Z/CAMPOSE, GeodesicMotionModel.cpp:101-176, from the MV on
      const V3 sp = h.ged_sp;
      float th;
      if (s.ged_flavor == 1)
        th = sp.y + g_atanf(g_sinf(sp.y) / (b.k - g_cosf(sp.y)));
      else
        th = sp.y + s.res * b.mvx;
      float ph = sp.z + s.res * b.mvy;
      V3 c = sph_to_cart(sp.x, th, ph, m);
      q = matT_vec(b.M, c);
    } break;
  }
  erp_from_sphere(q, s, m, true, omx, omy);
}
MM_HD void model_motion_element(const SeqConst& s, const BlockSetup& b, float gx, float gy, bool packet,
                                bool mpa_cached, float pers_x, float pers_y, bool pers_vip, float* omx, float* omy,
                                GridSphere grid = no_grid()) {
  const Math m{packet};
  motion_tail(s, b, motion_head(s, b, gx, gy, m, grid), gx, gy, m, mpa_cached, pers_x, pers_y, pers_vip, omx, omy);
}

// NaN -> unmoved (MVReprojection.cpp:151-154), remove offset, rescale, round to fixed point
MM_HD void reproject_finish(const SeqConst& s, float gx, float gy, float mx, float my, bool packet, int chroma_shift,
                            int32_t* fx, int32_t* fy);

MM_HD void reproject_element(const SeqConst& s, const BlockSetup& b, float gx, float gy, bool packet,
                             bool mpa_cached, float pers_x, float pers_y, bool pers_vip,
                             int chroma_shift, int32_t* fx, int32_t* fy, GridSphere grid = no_grid()) {
  float mx, my;
  model_motion_element(s, b, gx, gy, packet, mpa_cached, pers_x, pers_y, pers_vip, &mx, &my, grid);
  reproject_finish(s, gx, gy, mx, my, packet, chroma_shift, fx, fy);
}
MM_HD void reproject_finish(const SeqConst& s, float gx, float gy, float mx, float my, bool packet, int chroma_shift,
                            int32_t* fx, int32_t* fy) {
  if (isnanf_(mx) || isnanf_(my)) {
    mx = gx;
    my = gy;
  }
  mx = mx - s.off;
  my = my - s.off;
  if (chroma_shift) {
    mx = mx / 2.0f;
    my = my / 2.0f;
  }
  const float scale = (float)(1 << (4 + chroma_shift));
#if MM_ROUND_MODE
  float rx = packet ? roundeven_(mx * scale) : roundf_(mx * scale);
  float ry = packet ? roundeven_(my * scale) : roundf_(my * scale);
#else
  float rx = roundf_(mx * scale), ry = roundf_(my * scale);
#endif
  // cast<int>: x86 cvttss2si semantics for out-of-range values
  *fx = (fabsf_(rx) < 2147483648.0f) ? (int32_t)rx : (int32_t)0x80000000u;
  *fy = (fabsf_(ry) < 2147483648.0f) ? (int32_t)ry : (int32_t)0x80000000u;
}

}  // namespace mmmod
