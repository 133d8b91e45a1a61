// mm360_vtm.hpp -- C++ host shim over the C-ABI (include/mm360.h) with the call shape of the
// reference's MM path, so that DecoderLib / EncoderLib call sites change as little as possible.
//
//   mm360::Context             one decoder/encoder instance on one GPU (mm_create / mm_destroy)
//   mm360::MVReprojectionGPU   MVReprojection::init / isInitialized / subblockSize /
//                              reprojectMotionVectorSubblocks      (SRC/MVReprojection.h:32-58)
//   mm360::InterPredictionMM   xPredInterBlkMM + xWeightedAverage for a whole picture's PU list
//                              (SRC/InterPrediction.h:151-154, InterPrediction.cpp:1584-1679),
//                              per-list 14-bit predictions (xPredInterBlkMM bi = true), and the
//                              effective blocks of decoded PUs (motionCompensation's splits,
//                              SRC/InterPrediction.cpp:1681-1810)
//   mm360::EpipoleList         EpipoleList (SRC/EpipoleList.{h,cpp}) incl. derivePredictor
//   mm360::MMSyntax            the MM syntax of VLCReader / VLCWriter (SPS, PH) and of
//                              CABACReader / CABACWriter::motion_model, and the mm_seq_params a
//                              parsed SPS gives (DecLib.cpp:2013-2050's MM initialisation)
//
// Status codes become exceptions, like the reference's CHECK -> Exception (SRC/TypeDef.h:1120-1135).
// NaN reprojections (zero motion) and out-of-range sub-blocks (zero samples) are results, as in
// the reference, not errors.  SRC = source/Lib/CommonLib of FAU-LMS/vvc-extension-mm.
#pragma once
#include <cstdint>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../../include/mm360.h"

namespace mm360 {

class Exception : public std::runtime_error {
 public:
  Exception(int code, const std::string& what) : std::runtime_error(what), code_(code) {}
  int code() const { return code_; }

 private:
  int code_;
};

inline void check(mm_ctx* ctx, int rc, const char* call) {  // ctx may be null (host-only calls)
  if (rc != MM_OK)
    throw Exception(rc, std::string(call) + " failed (" + std::to_string(rc) + "): " +
                            (ctx ? mm_last_error(ctx) : "no context"));
}

// ---------------------------------------------------------------------------------------------
class Context {
 public:
  // SPS-derived parameters; the defaults are the reference's hard-coded MM settings
  // (EncApp.cpp:754-768): MMOffset4x4 code 1, GED flavour VISHWANATH_MODULATED.
  Context(const mm_seq_params& params, int device = 0) {
    int rc = mm_create(&params, device, &ctx_);
    if (rc != MM_OK) throw Exception(rc, "mm_create failed (no HIP device or invalid parameters)");
    params_ = params;
  }
  ~Context() {
    if (ctx_) mm_destroy(ctx_);
  }
  Context(const Context&) = delete;
  Context& operator=(const Context&) = delete;

  mm_ctx* get() const { return ctx_; }
  const mm_seq_params& params() const { return params_; }
  void setStream(void* hipStream) { check(ctx_, mm_set_stream(ctx_, hipStream), "mm_set_stream"); }
  void synchronize() { check(ctx_, mm_synchronize(ctx_), "mm_synchronize"); }

  // EpipoleList::addEpipole (EpipoleList.cpp:8-11), Q24 fixed point; -1 = wildcard POC
  void setEpipole(int curPOC, int refPOC, const int32_t q24[3]) {
    check(ctx_, mm_set_epipole(ctx_, curPOC, refPOC, q24), "mm_set_epipole");
  }
  // A reconstructed picture becomes a reference: unpadded planes, origin at (0, 0)
  void uploadReference(int poc, const int16_t* y, ptrdiff_t strideY, const int16_t* cb, const int16_t* cr,
                       ptrdiff_t strideC, bool onDevice) {
    check(ctx_, mm_upload_ref(ctx_, poc, y, strideY, cb, cr, strideC, onDevice ? 1 : 0), "mm_upload_ref");
  }
  void releaseReference(int poc) { check(ctx_, mm_release_ref(ctx_, poc), "mm_release_ref"); }

 private:
  mm_ctx* ctx_ = nullptr;
  mm_seq_params params_{};
};

// ---------------------------------------------------------------------------------------------
// EpipoleList (SRC/EpipoleList.h): a standalone list, or a view of a context's own list.
class EpipoleList {
 public:
  EpipoleList() : l_(mm_epipole_list_create()), owned_(true) {}
  explicit EpipoleList(Context& ctx) : l_(mm_get_epipole_list(ctx.get())), owned_(false) {}
  ~EpipoleList() {
    if (owned_) mm_epipole_list_destroy(l_);
  }
  EpipoleList(const EpipoleList&) = delete;
  EpipoleList& operator=(const EpipoleList&) = delete;

  void addEpipole(const int32_t q24[3], int curPOC = -1, int refPOC = -1, bool makeAvailable = false) {
    check(nullptr, mm_epipole_add(l_, curPOC, refPOC, q24, makeAvailable ? 1 : 0), "mm_epipole_add");
  }
  void makeAvailable(int curPOC) { mm_epipole_make_available(l_, curPOC); }
  bool hasEpipole(int curPOC, int refPOC) const { return mm_epipole_has(l_, curPOC, refPOC) != 0; }
  void findEpipoleFixed(int curPOC, int refPOC, int32_t q24[3]) const {
    check(nullptr, mm_epipole_find(l_, curPOC, refPOC, q24), "EpipoleList::findEpipole");
  }
  // derivePredictor + floatingToFixed, as DecLib does before adding the picture header's delta
  void derivePredictorFixed(int curPOC, int32_t q24[3]) const {
    check(nullptr, mm_epipole_derive_predictor(l_, curPOC, q24), "EpipoleList::derivePredictor");
  }
  int count() const { return mm_epipole_count(l_); }

 private:
  mm_epipole_list* l_;
  bool owned_;
};

// ---------------------------------------------------------------------------------------------
// ArrayXXFixedPtrPair analogue: X and Y fixed-point arrays, Eigen column-major (rows = h/sbh)
struct FixedPair {
  int rows = 0, cols = 0;
  std::vector<int32_t> x, y;
  int32_t X(int r, int c) const { return x[(size_t)c * rows + r]; }
  int32_t Y(int r, int c) const { return y[(size_t)c * rows + r]; }
};

class MVReprojectionGPU {
 public:
  // MVReprojection::init(projection, resolution, sps, epipoleList): the context already holds
  // the sequence parameters and builds the MPA frame caches on the device.
  void init(Context* ctx) { ctx_ = ctx; }
  bool isInitialized() const { return ctx_ != nullptr; }

  // MVReprojection::subblockSize (MVReprojection.cpp:73-78): 4x4 luma, 2x2 4:2:0 chroma
  static void subblockSize(int compID, int chromaFormat, int* w, int* h) {
    const bool sub = compID != 0 && chromaFormat == 1;
    *w = sub ? 2 : 4;
    *h = sub ? 2 : 4;
  }

  // reprojectMotionVectorSubblocks (MVReprojection.cpp:80-166); position/size in component units
  FixedPair reprojectMotionVectorSubblocks(int posX, int posY, int width, int height, int mvHor, int mvVer,
                                           int motionModelID, int compID, int curPOC, int refPOC) const {
    mm_block_desc b{posX, posY, width, height, mvHor, mvVer, motionModelID, compID, curPOC, refPOC};
    int sw, sh;
    subblockSize(compID, ctx_->params().chroma_format, &sw, &sh);
    FixedPair out;
    out.rows = height / sh;
    out.cols = width / sw;
    std::vector<int32_t> xy(2 * (size_t)out.rows * out.cols);
    check(ctx_->get(), mm_reproject(ctx_->get(), &b, 1, xy.data()), "mm_reproject");
    out.x.resize(xy.size() / 2);
    out.y.resize(xy.size() / 2);
    for (size_t i = 0; i < out.x.size(); i++) {
      out.x[i] = xy[2 * i];
      out.y[i] = xy[2 * i + 1];
    }
    return out;
  }

  // motionVectorInDesiredMotionModel (MVReprojection.cpp:168-217), same argument order; the
  // returned pair is the Mv (hor, ver).  For the call sites that convert one candidate at a time in
  // decoding order -- the spatial merge and AMVP candidates take the neighbour's final MV
  // (UnitTools.cpp:2930-2992, 3134-3167) -- on this host thread, with the library's own model
  // bodies (mm_mvp_convert_host); no device round trip.  The collocated (TMVP) candidates of a
  // whole picture (UnitTools.cpp:2267-2304) can instead be batched through mm_mvp_convert_device.
  std::pair<int32_t, int32_t> motionVectorInDesiredMotionModel(
      int posX, int posY, int32_t mvHor, int32_t mvVer, int modelOrig, int modelDesired, int shiftHor, int shiftVer,
      int curPOCOrig, int refPOCOrig, int curPOCDesired, int refPOCDesired, int candX, int candY, int candW, int candH,
      int curX, int curY, int curW, int curH) const {
    const mm_mvp_query q{posX,       posY,       mvHor,         mvVer,         modelOrig, modelDesired, shiftHor,
                         shiftVer,   curPOCOrig, refPOCOrig,    curPOCDesired, refPOCDesired, candX, candY,
                         candW,      candH,      curX,          curY,          curW,      curH};
    int32_t mv[2] = {0, 0};
    check(ctx_->get(),
          mm_mvp_convert_host(&ctx_->params(), mm_get_epipole_list(ctx_->get()), &q, 1, mv, nullptr),
          "motionVectorInDesiredMotionModel");
    return {mv[0], mv[1]};
  }

 private:
  Context* ctx_ = nullptr;
};

// ---------------------------------------------------------------------------------------------
// Batched MM motion compensation of one picture.  A decoder collects the MM PUs of a picture (or
// of a CTU row) while parsing -- after its own xSubPuMC / DMVR / BDOF-size splitting
// (InterPrediction.cpp:1737-1789) -- then predicts them in one call; the predictions land in
// device planes that the reconstruction reads.
class InterPredictionMM {
 public:
  explicit InterPredictionMM(Context* ctx) : ctx_(ctx) {}

  void clear() {
    pus_.clear();
    dmvr_.clear();
  }
  // One effective block: luma area, per list (mv in 1/16 luma, reference POC or -1, motion
  // model), the CU's BCW index
  void addPU(int x, int y, int w, int h, const int mv[2][2], const int refPOC[2], const int model[2],
             int bcwIdx = MM_BCW_DEFAULT) {
    mm_pu_desc d{};
    d.bcw_idx = bcwIdx;
    d.x = x;
    d.y = y;
    d.w = w;
    d.h = h;
    for (int l = 0; l < 2; l++) {
      d.mv[l][0] = mv[l][0];
      d.mv[l][1] = mv[l][1];
      d.ref_poc[l] = refPOC[l];
      d.model[l] = model[l];
    }
    pus_.push_back(d);
  }
  // One decoded PU as motionCompensation sees it: its effective blocks (16x16 BDOF-size
  // sub-PUs, merged SbTMVP strips, identical-motion uni L0) join the list, DMVR PUs the DMVR list
  void addDecodedPU(const mm_tool_flags& tools, const mm_pu_motion& pu, const mm_pu_desc* subMotion = nullptr) {
    const int cap = (pu.pu.w / 4) * (pu.pu.h / 4) + 1;
    std::vector<mm_pu_desc> mc(cap), dm(cap);
    int n_mc = 0, n_dm = 0;
    check(ctx_->get(),
          mm_derive_effective_blocks(&tools, &pu, 1, subMotion, mc.data(), cap, &n_mc, dm.data(), cap, &n_dm),
          "mm_derive_effective_blocks");
    pus_.insert(pus_.end(), mc.begin(), mc.begin() + n_mc);
    dmvr_.insert(dmvr_.end(), dm.begin(), dm.begin() + n_dm);
  }
  size_t size() const { return pus_.size(); }
  const std::vector<mm_pu_desc>& pus() const { return pus_; }
  const std::vector<mm_pu_desc>& dmvrPUs() const { return dmvr_; }

  // Synchronous: host PU list -> predicted device planes (bi: addAvg, uni: clipped).
  void predictPicture(int curPOC, int16_t* dstY, ptrdiff_t strideY, int16_t* dstCb, int16_t* dstCr,
                      ptrdiff_t strideC) {
    check(ctx_->get(),
          mm_pred(ctx_->get(), curPOC, pus_.data(), (int)pus_.size(), dstY, strideY, dstCb, dstCr, strideC),
          "mm_pred");
  }
  // DMVR PUs collected by addDecodedPU (xProcessDMVRProjected), synchronous
  void predictDmvr(int curPOC, int16_t* dstY, ptrdiff_t strideY, int16_t* dstCb, int16_t* dstCr, ptrdiff_t strideC) {
    if (dmvr_.empty()) return;
    check(ctx_->get(),
          mm_pred_dmvr(ctx_->get(), curPOC, dmvr_.data(), (int)dmvr_.size(), dstY, strideY, dstCb, dstCr, strideC,
                       nullptr),
          "mm_pred_dmvr");
  }
  // xPredInterBlkMM of one list of every collected PU: bi = true keeps the 14-bit intermediate
  // (GEO / CIIP / weighted-prediction blending happens in the caller), dstY or dstCb/dstCr may be
  // null for a per-component call.
  void predictList(int curPOC, int list, bool bi, int16_t* dstY, ptrdiff_t strideY, int16_t* dstCb, int16_t* dstCr,
                   ptrdiff_t strideC) {
    check(ctx_->get(),
          mm_pred_list(ctx_->get(), curPOC, pus_.data(), (int)pus_.size(), list, bi ? 1 : 0, dstY, strideY, dstCb,
                       dstCr, strideC),
          "mm_pred_list");
  }
  // Asynchronous on the context stream: PU list already in device memory (e.g. written by a GPU
  // parser); errors surface at Context::synchronize().
  void predictPictureDevice(int curPOC, const mm_pu_desc* devPUs, int n, int16_t* dstY, ptrdiff_t strideY,
                            int16_t* dstCb, int16_t* dstCr, ptrdiff_t strideC) {
    check(ctx_->get(), mm_pred_device(ctx_->get(), curPOC, devPUs, n, dstY, strideY, dstCb, dstCr, strideC),
          "mm_pred_device");
  }
  // Several pictures that do not reference each other (the leaves of one RA temporal layer) in one
  // launch chain, each with its own current POC, device PU list and destination planes; asynchronous
  // like predictPictureDevice.  At most MM_MAX_PICS pictures.
  void predictPicturesDevice(const std::vector<mm_pic_job>& pictures) {
    check(ctx_->get(), mm_pred_device_multi(ctx_->get(), pictures.data(), (int)pictures.size()),
          "mm_pred_device_multi");
  }

 private:
  Context* ctx_;
  std::vector<mm_pu_desc> pus_, dmvr_;
};

// ---------------------------------------------------------------------------------------------
// The bitstream side (host only).  Bit positions are MSB-first offsets into the caller's RBSP.
namespace MMSyntax {
inline mm_sps_mm readSPS(const uint8_t* rbsp, int64_t nbits, int64_t& bitPos) {
  mm_sps_mm s;
  check(nullptr, mm_sps_mm_read(rbsp, nbits, &bitPos, &s), "mm_sps_mm_read");
  return s;
}
// appends at bitPos, growing the buffer as needed
inline void writeSPS(const mm_sps_mm& s, std::vector<uint8_t>& rbsp, int64_t& bitPos) {
  if ((int64_t)rbsp.size() * 8 < bitPos + 2048) rbsp.resize((size_t)((bitPos + 2048 + 7) / 8), 0);
  check(nullptr, mm_sps_mm_write(&s, rbsp.data(), (int64_t)rbsp.size(), &bitPos), "mm_sps_mm_write");
}
inline void readEpipoleDelta(const mm_sps_mm& s, const uint8_t* rbsp, int64_t nbits, int64_t& bitPos, int32_t delta[3]) {
  check(nullptr, mm_ph_epipole_read(&s, rbsp, nbits, &bitPos, delta), "mm_ph_epipole_read");
}
// MMConfig::getActiveMotionModels order (the coding order of motion_model with m_mmPredType 0)
inline std::vector<int32_t> activeModels(const mm_sps_mm& s) {
  int32_t c[MM_NUM_MODEL_IDS];
  int32_t n = 0;
  check(nullptr, mm_motion_model_candidates(&s, 0, nullptr, 0, 0, 0, 0, 0, 0, 0, 0, 0, c, &n),
        "mm_motion_model_candidates");
  return std::vector<int32_t>(c, c + n);
}
// The sequence parameters of the MM path from a parsed SPS fragment plus the SPS's picture fields
// (DecLib.cpp:2013-2050 builds MVReprojection from the same values)
inline mm_seq_params seqParams(const mm_sps_mm& s, int width, int height, int chromaFormat, int bitDepth,
                               int maxCuWidth, int maxCuHeight) {
  uint32_t mask = 0;
  for (int32_t m : activeModels(s)) mask |= 1u << m;
  return mm_seq_params{width, height, chromaFormat, bitDepth, maxCuWidth, maxCuHeight, s.mm_offset_4x4,
                       s.ged_flavor, mask};
}
}  // namespace MMSyntax

}  // namespace mm360
