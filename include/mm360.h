/* mm360.h -- C-ABI of the MI355X-native 360-degree multi-model motion-compensation path.
 *
 * Drop-in boundary for the MM branch of VTM-17.2 + MM extension (FAU-LMS/vvc-extension-mm).
 * The reference has no plugin/FFI API; these entry points replace the C++ method surface
 * listed in SURVEY.md section 8(b).  Paths are relative to
 * /root/reference/source/Lib/CommonLib (SRC) or /root/reference/source/Lib.
 *
 *   mm_create        <- MVReprojection::init              SRC/MVReprojection.h:32
 *                       (+ EquirectangularProjection ctor SRC/Projection.h:127-130,
 *                          MMConfig active-model list     SRC/MMConfig.cpp:7-39)
 *   mm_set_epipole   <- EpipoleList::addEpipole           SRC/EpipoleList.cpp:8-11
 *   mm_upload_ref    <- Picture reconstruction planes     SRC/Picture.cpp:84-95 (+ extendPicBorder :988-1048)
 *   mm_reproject     <- MVReprojection::reprojectMotionVectorSubblocks
 *                                                         SRC/MVReprojection.h:54-58
 *   mm_pred          <- InterPrediction::xPredInterBlkMM  SRC/InterPrediction.h:151-154,
 *   mm_pred_device      batched over a picture's PU list together with the MM dispatch of
 *                       xPredInterUni (InterPrediction.cpp:455-533) and xWeightedAverage
 *                       (addAvg / addWeightedAvg (BCW) / copyClip)
 *                                                         SRC/InterPrediction.cpp:1584-1679,
 *                                                         SRC/Buffer.cpp:398-424, 551-658
 *   mm_pred_device_multi <- the same over several independent pictures in one launch chain
 *   mm_pred_list     <- InterPrediction::xPredInterBlkMM 1:1 per list: one reference list of every
 *                       PU, bi=true (14-bit, rndRes=false) or bi=false (clipped), InterPrediction.cpp:683-856
 *   mm_filter        <- InterpolationFilter::filterHor/filterVer  SRC/InterpolationFilter.h:123-128
 *   mm_pred_dmvr     <- InterPrediction::xProcessDMVRProjected  SRC/InterPrediction.cpp:2442-2634
 *   mm_mvp_convert   <- MVReprojection::motionVectorInDesiredMotionModel  SRC/MVReprojection.cpp:168-217
 *   mm_mvp_convert_host <- the same, per query on the host, at the spatial merge / AMVP call sites
 *                       (UnitTools.cpp:2930-2992, 3134-3167); device batches serve TMVP (:2267-2304)
 *   mm_sad_window    <- InterSearch::xMVReprojectionInterpolation + RdCost::xGetSAD per candidate
 *                       (EncoderLib/InterSearch.cpp:6277-6385, 363-443; SRC/RdCost.cpp:482-517)
 *   mm_sad_pattern   <- the same over the TZ / refinement candidate patterns (InterSearch.cpp:474-526,
 *                       6168-6249)
 *   mm_upload_org    <- the original picture (pcPatternKey) the encoder SAD compares against
 *   mm_destroy       <- (MVReprojection / InterPrediction destructors)
 *
 * Conventions: plain C, int status return (MM_OK = 0), one opaque context per
 * decoder instance, explicit HIP stream, no exceptions across the ABI.  Samples are `Pel`
 * (int16), planes are caller-owned; reprojection results are fixed-point sub-block origins
 * (1/16 pel luma, 1/32 pel 4:2:0 chroma) in Eigen column-major order (element (row, col) of the
 * reference's ArrayXXi at index col*rows + row).  NaN reprojections fall back to zero motion and
 * out-of-range sub-blocks predict zeros, exactly as the reference (these are results, not errors).
 */
#ifndef MM360_H
#define MM360_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MM_OK 0
#define MM_ERR_ARG 1        /* invalid argument (reference: CHECK -> Exception) */
#define MM_ERR_HIP 2        /* HIP runtime error */
#define MM_ERR_NOREF 3      /* reference POC not uploaded */
#define MM_ERR_NOEPIPOLE 4  /* no epipole for (curPOC, refPOC) -- EpipoleList.cpp:31 CHECK */
#define MM_ERR_MODEL 5      /* motion model not active / CLASSIC passed to reprojection */
#define MM_ERR_NODEV 6      /* no HIP device */
#define MM_ERR_BITSTREAM 7  /* malformed / truncated syntax (mm_*_read, mm_motion_model_decode) */

/* MotionModelID, SRC/TypeDef.h:865-879 */
enum mm_model_id {
  MM_CLASSIC = 0,
  MM_MPA_FRONT_BACK = 1,
  MM_MPA_LEFT_RIGHT = 2,
  MM_MPA_TOP_BOTTOM = 3,
  MM_TANGENTIAL = 4,
  MM_THREE_D_TRANSLATIONAL = 5,
  MM_ROTATIONAL = 6,
  MM_GEODESIC_X = 7,
  MM_GEODESIC_Y = 8,
  MM_GEODESIC_Z = 9,
  MM_GEODESIC_CAMPOSE = 10
};

/* Sequence parameters (SPS fields + hard-coded MM settings, EncApp.cpp:754-768) */
typedef struct mm_seq_params {
  int32_t width, height;       /* luma picture size of the ERP picture (multiples of 8, <= 16384) */
  int32_t chroma_format;       /* 0 = 4:0:0, 1 = 4:2:0 (ChromaFormat CHROMA_400 / CHROMA_420) */
  int32_t bit_depth;           /* internal bit depth (10 in the RA cfg) */
  int32_t max_cu_width;        /* SPS maxCUWidth (CTU size, 128) -- out-of-range rule */
  int32_t max_cu_height;
  int32_t mm_offset4x4;        /* SPS MMOffset4x4 code 0..4 (4 => 1.5), MVReprojection.cpp:10 */
  int32_t ged_flavor;          /* 0 VISHWANATH_ORIGINAL, 1 VISHWANATH_MODULATED */
  uint32_t active_models;      /* bit i set <=> MotionModelID i active (CLASSIC always) */
} mm_seq_params;

/* One reprojection request == one call of reprojectMotionVectorSubblocks */
typedef struct mm_block_desc {
  int32_t x, y, w, h;          /* block position/size in COMPONENT units (pu.blocks[compID]) */
  int32_t mv_hor, mv_ver;      /* Mv in 1/16 luma units (MV_FRACTIONAL_BITS_INTERNAL = 4) */
  int32_t model;               /* mm_model_id, not CLASSIC */
  int32_t comp;                /* 0 = luma, 1 = Cb, 2 = Cr */
  int32_t cur_poc, ref_poc;    /* for GEODESIC_CAMPOSE epipole selection */
} mm_block_desc;

/* BCW weight index (CU::bcwIdx): g_BcwWeights = {-2, 3, 4, 5, 10} (Rom.cpp:203), BCW_DEFAULT = 2
 * (CommonDef.h:348-349) is the plain addAvg.  Only bi PUs use it. */
#define MM_BCW_DEFAULT 2

/* mm_pu_desc.flags */
#define MM_PUF_DMVR 0x1u  /* bi PU that passed PU::checkDMVRCondition (UnitTools.cpp:1698-1726): mm_pred_device
                             runs xProcessDMVRProjected's search on its 16x16 sub-PUs before predicting them
                             (needs mm_set_dmvr(ctx, 1), the picture's DMVR enable) */

/* One prediction unit (or sub-PU after the host's xSubPuBio / DMVR / SbTMVP split; the helpers in
 * host/mm360_vtm.hpp derive these effective blocks).  64 bytes.  The PUs of one call must not
 * overlap (every luma sample is predicted by at most one PU, as in a decoded picture); the result
 * of an overlapping list is undefined, and a list whose PUs cover more sub-blocks than the
 * picture has is rejected with MM_ERR_ARG.
 * NOTE for zero-initialised descriptors: bcw_idx uses the reference encoding, in which 0 is the
 * (-2, 10) weight pair, not the plain average -- bi PUs must set bcw_idx = MM_BCW_DEFAULT (2).
 * flags bits other than MM_PUF_* and nonzero reserved words are rejected with MM_ERR_ARG (so a
 * stale 48-byte layout fails loudly instead of predicting garbage). */
typedef struct mm_pu_desc {
  int32_t x, y, w, h;          /* luma area */
  int32_t mv[2][2];            /* [list][hor, ver], 1/16 luma */
  int32_t ref_poc[2];          /* reference POC per list, -1 = list unused */
  int32_t model[2];            /* mm_model_id per list (non-CLASSIC for MM MC) */
  int32_t bcw_idx;             /* CU::bcwIdx 0..4 (bi PUs; MM_BCW_DEFAULT = addAvg); ignored for uni */
  uint32_t flags;              /* MM_PUF_* */
  int32_t reserved[2];         /* must be zero */
} mm_pu_desc;

/* ---- Effective blocks (host-side, no GPU) ----------------------------------------------------
 * The blocks InterPrediction::motionCompensation (SRC/InterPrediction.cpp:1681-1810) hands to
 * xPredInterBlkMM for one decoded PU: the BDOF pre-check's 16x16 split (xSubPuBio :361-453; the
 * reprojection block centre moves to the sub-PU), SbTMVP strip merging of identical MotionInfo
 * (xSubPuMC :283-359), xCheckIdenticalMotion (:248-281, bi -> uni L0) and the DMVR decision
 * (PU::checkDMVRCondition, UnitTools.cpp:1698-1726).  See csrc/mm_effective.h. */
#define MM_PU_MERGE 0x001u       /* pu.mergeFlag */
#define MM_PU_SUBPU 0x002u       /* mergeType == MRG_TYPE_SUBPU_ATMVP: motion per 8x8 in sub_motion */
#define MM_PU_CIIP 0x004u        /* pu.ciipFlag */
#define MM_PU_SMVD 0x008u        /* cu.smvdMode */
#define MM_PU_MMVD 0x010u        /* pu.mmvdMergeFlag || cu.mmvdSkip */
#define MM_PU_MVREFINE 0x020u    /* pu.mvRefine (DMVR requested) */
#define MM_PU_WEIGHTED 0x040u    /* explicit weighted prediction applies (WPScalingParam::isWeighted) */
#define MM_PU_LONGTERM 0x080u    /* a list references a long-term picture */
#define MM_PU_REF_SCALED 0x100u  /* a reference is scaled (RPR) */
#define MM_PU_MMVD_ENC2 0x200u   /* encoder: mmvdEncOptMode == 2 && mmvdMergeFlag */

typedef struct mm_tool_flags {  /* SPS / PPS / PH switches of the current picture */
  int32_t bdof;   /* sps BDOF enabled && !ph_bdof_disabled */
  int32_t dmvr;   /* sps DMVR enabled && !ph_dmvr_disabled */
  int32_t bcw;    /* sps BCW enabled */
  int32_t wp_bi;  /* pps weighted bi-prediction (xCheckIdenticalMotion) */
} mm_tool_flags;

typedef struct mm_pu_motion {
  mm_pu_desc pu;        /* the decoded PU: luma area, motion, CU bcwIdx */
  uint32_t flags;       /* MM_PU_* */
  int32_t cur_poc;
  int32_t sub_motion;   /* MM_PU_SUBPU: first of (w/8) x (h/8) raster mm_pu_desc motion records */
  int32_t reserved;
} mm_pu_motion;


/* One block of an encoder motion search (InterSearch::xMVReprojectionInterpolation call site,
 * EncoderLib/InterSearch.cpp:6189-6273): a window of candidate MVs around `mv` is evaluated. */
typedef struct mm_me_block {
  int32_t x, y, w, h;          /* luma block (PU) */
  int32_t mv_hor, mv_ver;      /* window centre, 1/16 luma (MV_PRECISION_INTERNAL) */
  int32_t model;               /* mm_model_id, not CLASSIC */
  int32_t ref_poc;
  int32_t sub_shift;           /* SAD row subsampling: 0 = every row, 1 = every other row
                                  (RdCost::setDistParam subShiftMode 2, RdCost.cpp:296-303) */
} mm_me_block;

/* One MM-MVP conversion: MVReprojection::motionVectorInDesiredMotionModel arguments
 * (MVReprojection.h:60-64, MVReprojection.cpp:168-217). */
typedef struct mm_mvp_query {
  int32_t pos_x, pos_y;                    /* position whose shift the MVs must agree on */
  int32_t mv_hor, mv_ver;                  /* candidate MV (shift_hor / shift_ver fractional bits) */
  int32_t model_orig, model_desired;       /* mm_model_id, CLASSIC allowed */
  int32_t shift_hor, shift_ver;
  int32_t cur_poc_orig, ref_poc_orig;      /* epipole of the candidate (GEODESIC_CAMPOSE) */
  int32_t cur_poc_desired, ref_poc_desired;
  int32_t cand_x, cand_y, cand_w, cand_h;  /* candidate block (MotionInfo::blockPos/blockSize) */
  int32_t cur_x, cur_y, cur_w, cur_h;      /* current block */
} mm_mvp_query;

typedef struct mm_ctx mm_ctx;

/* Lifecycle.  A context's device buffers come from the device's stream-ordered memory pool and are
 * freed in its own streams' order: growing them, mm_synchronize and mm_destroy never wait for other
 * contexts' or the application's queues.  mm_set_stream first waits for the work queued on the
 * context's previous stream. */
int mm_create(const mm_seq_params* params, int device, mm_ctx** out_ctx);
int mm_destroy(mm_ctx* ctx);
int mm_set_stream(mm_ctx* ctx, void* hip_stream);     /* hipStream_t; NULL = default stream */
int mm_synchronize(mm_ctx* ctx);                      /* also reports a deferred mm_pred_device status */
const char* mm_last_error(mm_ctx* ctx);
int mm_get_version(void);

/* Epipoles in Q24 fixed point (EPIPOLE_PRECISION_FIXED, CommonDef.h:441).  cur/ref POC -1 are
 * the wildcards of EpipoleList::findEpipoleFixed (exact pair, then (cur,-1), then (-1,-1)).
 * mm_set_epipole == EpipoleList::addEpipole(..., makeAvailable = true) on the context's list, as
 * the decoder adds them (DecLib.cpp:2048, 3141). */
int mm_set_epipole(mm_ctx* ctx, int cur_poc, int ref_poc, const int32_t q24[3]);

/* EpipoleList (SRC/EpipoleList.{h,cpp}) with its availability semantics.  A new list holds the
 * global (-1, -1) zero epipole, not available (EpipoleList.h:15-17); lookups only see available
 * entries.  Standalone lists need no GPU; mm_get_epipole_list returns the context's own list
 * (owned by the context, which uses it for every GEODESIC_CAMPOSE lookup). */
typedef struct mm_epipole_list mm_epipole_list;
mm_epipole_list* mm_epipole_list_create(void);
void mm_epipole_list_destroy(mm_epipole_list* list);        /* no-op on a context's list */
mm_epipole_list* mm_get_epipole_list(mm_ctx* ctx);
/* addEpipole (EpipoleList.cpp:8-11), Q24 in (the caller applies floatingToFixed) */
int mm_epipole_add(mm_epipole_list* list, int cur_poc, int ref_poc, const int32_t q24[3], int make_available);
int mm_epipole_make_available(mm_epipole_list* list, int cur_poc);           /* :91-99 */
int mm_epipole_has(mm_epipole_list* list, int cur_poc, int ref_poc);         /* :82-89, 1 / 0 */
int mm_epipole_find(mm_epipole_list* list, int cur_poc, int ref_poc, int32_t q24[3]); /* :19-36 */
/* derivePredictor (EpipoleList.cpp:38-80, incl. the `p0 + p1 / 2` tie rule as written) followed by
 * the decoder's floatingToFixed (DecLib.cpp:3138): the Q24 predictor the picture header's epipole
 * delta is added to.  MM_ERR_NOEPIPOLE if the global epipole is not available. */
int mm_epipole_derive_predictor(mm_epipole_list* list, int cur_poc, int32_t q24[3]);
int mm_epipole_count(mm_epipole_list* list);                                 /* EpipoleList::count */

/* Reference picture planes (reconstruction, unpadded, picture origin at plane[0]).  `src_is_device`
 * = 1 when the pointers are device memory.  The context keeps its own device copy with edge-
 * replicated margins of maxCU + the filter reach (extendPicBorder, Picture.cpp:988-1048), filled on
 * the device at upload; the caller's planes need no padding. */
int mm_upload_ref(mm_ctx* ctx, int poc, const int16_t* y, ptrdiff_t stride_y, const int16_t* cb,
                  const int16_t* cr, ptrdiff_t stride_c, int src_is_device);
int mm_release_ref(mm_ctx* ctx, int poc);

/* C4 transport (CTU-row stripes across GPUs, one all-gather per referenced picture): the packed
 * stripe-major picture.  The int16 stripe-major picture of `world` ranks (mm360/parallel.py
 * StripeLayout: segment r = the luma rows of stripe r, then its Cb rows, then its Cr rows, every
 * segment sized for the largest stripe of CTU rows of `ctu` luma rows: rows x W + 2 x (rows/2) x
 * (W/2) samples) is carried with K = 32 / bit_depth samples per dword (3 at 10 bits, so 2/3 of the
 * int16 bytes): sample j of a segment sits in bits (j % K) * bit_depth of dword j / K of the
 * segment's mm_stripe_packed_dwords(...) dwords.  Samples must lie in [0, 2^bit_depth) (predicted
 * samples do).  (No reference counterpart: the reference decodes on one CPU.)
 *   mm_stripe_packed_dwords: dwords per packed segment.
 *   mm_pack_samples: n int16 samples (device) -> ceil(n / K) dwords (device), on the context stream;
 *     a rank packs its own int16 segment into its packed segment before the all-gather.
 *   mm_upload_ref_packed: the gathered packed picture (device, world segments) becomes reference
 *     `poc`, unpacked straight into the context's padded reference copy -- margins included, as
 *     mm_upload_ref pads -- on the context stream.
 *   mm_upload_ref_stripes: the same from the int16 stripe-major picture (the unpacked transport). */
int64_t mm_stripe_packed_dwords(mm_ctx* ctx, int world, int ctu);
int mm_pack_samples(mm_ctx* ctx, const int16_t* d_src, int64_t n, uint32_t* d_dst);
int mm_upload_ref_packed(mm_ctx* ctx, int poc, const uint32_t* d_packed, int world, int ctu);
int mm_upload_ref_stripes(mm_ctx* ctx, int poc, const int16_t* d_stripes, int world, int ctu);

/* Parity API: n blocks, results written to out_xy (host memory) as int32 pairs
 * [X0, Y0, X1, Y1, ...] block after block, N_b = (w/sbw)*(h/sbh) pairs per block.  Blocks are at
 * most 128 x 128 in component units (VVC's MAX_CU_SIZE; MM_ERR_ARG beyond). */
int mm_reproject(mm_ctx* ctx, const mm_block_desc* blocks, int n, int32_t* out_xy);

/* Batched motion compensation of one picture's PU list (host descriptor array).
 * Writes the final prediction (bi: addAvg, or addWeightedAvg when bcw_idx != MM_BCW_DEFAULT, of
 * both lists' 14-bit predictions; uni: clipped prediction) of every PU into the destination planes
 * (device memory, picture-sized). */
int mm_pred(mm_ctx* ctx, int cur_poc, const mm_pu_desc* pus, int n, int16_t* dst_y,
            ptrdiff_t dst_stride_y, int16_t* dst_cb, int16_t* dst_cr, ptrdiff_t dst_stride_c);

/* The same with the PU list already in device memory: the whole per-picture path runs on the
 * device -- planning (PU classification, job bucketing, prefix offsets), per-block setup,
 * reprojection, interpolation and averaging -- as one asynchronous launch sequence on the
 * context stream, with no host synchronisation.  Descriptor validation (the reference's CHECKs:
 * geometry, model, reference, epipole) happens on the device; failing PUs are skipped and the
 * lowest failing PU's code is reported by mm_pred_status / mm_synchronize -- for the LAST
 * device-planned call: a decoder that wants every picture's status reads it before the next call. */
int mm_pred_device(mm_ctx* ctx, int cur_poc, const mm_pu_desc* d_pus, int n, int16_t* dst_y,
                   ptrdiff_t dst_stride_y, int16_t* dst_cb, int16_t* dst_cr,
                   ptrdiff_t dst_stride_c);

/* Several independent pictures in ONE launch chain: the pictures of one call must not reference
 * each other's output (the leaves of a random-access temporal layer, or the CTU-row stripes of
 * different pictures on one GPU, cfg/encoder_randomaccess_vtm.cfg:20-51).  Each picture has its
 * own current POC (GEODESIC_CAMPOSE epipoles of (cur_poc, ref)), device PU list and destination
 * planes; all read the context's resident references.  The planning, setup, reprojection and
 * interpolation of all pictures share their launches, so small pictures or stripes no longer pay
 * the per-call launch chain each.  Same semantics as mm_pred_device per picture (plan-ahead,
 * deferred status; the status's PU index counts through the pictures' lists in call order).
 * MM_PUF_DMVR PUs (mm_set_dmvr) are searched per picture inside the same chain -- the leaves of an
 * RA temporal layer are DMVR's usual bi PUs.  1 <= n_pics <= MM_MAX_PICS.  One launch chain holds
 * 16 distinct GEODESIC_CAMPOSE epipoles (over every (cur_poc, resident reference) pair of its
 * pictures); pictures beyond that are cut into consecutive runs of their own chain, and every run
 * but the last is then synchronised and its status read before the next is issued. */
#define MM_MAX_PICS 4
typedef struct mm_pic_job {
  int32_t cur_poc;
  const mm_pu_desc* d_pus;     /* device memory */
  int32_t n;
  int16_t* dst_y;
  ptrdiff_t dst_stride_y;
  int16_t* dst_cb;
  int16_t* dst_cr;
  ptrdiff_t dst_stride_c;
} mm_pic_job;
int mm_pred_device_multi(mm_ctx* ctx, const mm_pic_job* pics, int n_pics);

/* Waits for the context stream and returns the deferred status of the last device-planned
 * call (MM_OK or the code of the lowest failing PU, whose index goes to *first_bad_pu). */
int mm_pred_status(mm_ctx* ctx, int* first_bad_pu);

/* Split form for resident-input benchmarking: mm_pred_prepare copies the PU list into the
 * context's device buffer; mm_pred_run runs mm_pred_device on it (all device work, no host
 * synchronisation).  mm_pred == prepare + run + mm_pred_status. */
int mm_pred_prepare(mm_ctx* ctx, int cur_poc, const mm_pu_desc* pus, int n);
int mm_pred_run(mm_ctx* ctx, int16_t* dst_y, ptrdiff_t dst_stride_y, int16_t* dst_cb,
                int16_t* dst_cr, ptrdiff_t dst_stride_c);

/* Effective blocks of n decoded PUs (see MM_PU_*): out_mc receives the PUs for mm_pred (bi, uni,
 * identical-motion bi as uni L0, 16x16 sub-PUs, merged SbTMVP strips), out_dmvr those for
 * mm_pred_dmvr, each in motionCompensation's order.  n_mc / n_dmvr receive the counts; a count
 * beyond cap_* returns MM_ERR_ARG with the required counts.  Host code only: no context, no GPU. */
int mm_derive_effective_blocks(const mm_tool_flags* tools, const mm_pu_motion* pus, int n, const mm_pu_desc* sub_motion,
                               mm_pu_desc* out_mc, int cap_mc, int* n_mc, mm_pu_desc* out_dmvr, int cap_dmvr,
                               int* n_dmvr);

/* xPredInterBlkMM 1:1 per list (InterPrediction.h:151-154): the prediction of reference list
 * `list` (0/1) of every PU, exactly as InterPrediction::xPredInterBlkMM leaves it in its PelUnitBuf:
 * hp = 1 -> bi = true, 14-bit intermediate (rndRes = false, InterPrediction.cpp:697), as the
 * caller's GEO / BCW / CIIP blending consumes it (InterPrediction.cpp:637, 1651-1670); hp = 0 ->
 * bi = false, rounded and clipped.  Every PU must use `list` (ref_poc[list] >= 0), the other list is
 * ignored.  dst_y or dst_cb/dst_cr may be NULL to skip that component (per-component calls of the
 * reference).  Device-planned like mm_pred; host PU list; synchronous status. */
int mm_pred_list(mm_ctx* ctx, int cur_poc, const mm_pu_desc* pus, int n, int list, int hp, int16_t* dst_y,
                 ptrdiff_t dst_stride_y, int16_t* dst_cb, int16_t* dst_cr, ptrdiff_t dst_stride_c);

/* MM-DMVR (InterPrediction::xProcessDMVRProjected, InterPrediction.cpp:2442-2634): bi PUs that
 * pass PU::checkDMVRCondition (UnitTools.cpp:1698-1726; equal models, w, h >= 8, w*h >= 128 are
 * checked here, merge mode / POC distances / weights are the caller's decision).  Every
 * min(w,16) x min(h,16) sub-PU runs the 25-point mirrored integer search and the parabolic sub-pel
 * refinement on 14-bit luma predictions, then is predicted as a bi PU at the refined MVs (all
 * components, addAvg) into the destination planes (device memory).  mvd_out (host, optional):
 * the refined L0 delta (1/16 luma, pu.mvdL0SubPu) of every sub-PU, PU after PU, sub-PUs in raster
 * order.  Synchronous.  (The same device path as MM_PUF_DMVR PUs under mm_set_dmvr, with every PU
 * of the list flagged.) */
int mm_pred_dmvr(mm_ctx* ctx, int cur_poc, const mm_pu_desc* pus, int n, int16_t* dst_y,
                 ptrdiff_t dst_stride_y, int16_t* dst_cb, int16_t* dst_cr, ptrdiff_t dst_stride_c,
                 int32_t* mvd_out);

/* MM-MVP, batched: motionVectorInDesiredMotionModel for n queries (the candidate's modelMotion
 * at `pos` on a 1x1 array, then the desired model's motionVectorForEquivalentPixelShiftAt,
 * NaN -> zero MV, std::round to fixed point).  mv_out (host): 2 int32 per query.  Synchronous;
 * the first failing query's code is returned (MM_ERR_MODEL / MM_ERR_ARG / MM_ERR_NOEPIPOLE). */
int mm_mvp_convert(mm_ctx* ctx, const mm_mvp_query* queries, int n, int32_t* mv_out);

/* The same with queries and results in device memory: validation, GEODESIC_CAMPOSE epipole lookup
 * (a device copy of the context's EpipoleList, refreshed when the list changed) and both model
 * evaluations run on the device, stream-ordered on the context stream with no host
 * synchronisation.  Failures accumulate in one status word until the next mm_mvp_status /
 * mm_synchronize reads (and clears) it: that call reports a failing query of the conversions issued
 * since the previous read -- the lowest failing index among them -- so conversions issued
 * back to back lose no failure (the failing queries' result words are 0). */
int mm_mvp_convert_device(mm_ctx* ctx, const mm_mvp_query* d_queries, int n, int32_t* d_mv_out);
int mm_mvp_status(mm_ctx* ctx, int* first_bad_query);
/* The stream MM-MVP conversions run on (hipStream_t; NULL = the context stream, the default).  A
 * decoder that derives picture t+1's MVs while picture t is motion-compensated converts on its
 * own stream, so the conversions overlap the picture kernels; it orders the prediction of t+1
 * after them itself (an event on this stream).  Epipole-table refreshes (made on the context
 * stream) are ordered before the conversions that follow them, and after the conversions still
 * reading the table they replace (two tables alternate per EpipoleList version).  mm_mvp_status / mm_mvp_convert
 * wait for this stream; the call's device time (mm_last_timing) is recorded only while call
 * timing is on. */
int mm_set_mvp_stream(mm_ctx* ctx, void* hip_stream);

/* MM-MVP one query at a time on the calling host thread, for the candidates VTM converts in
 * decoding order: spatial merge and AMVP candidates take the neighbour's FINAL MV
 * (UnitTools.cpp:2930-2992 merge, 3134-3167 addMVPCandUnscaled), which the PUs decoded just before
 * produced, so they cannot wait for a device batch.  Replaces motionVectorInDesiredMotionModel
 * (MVReprojection.cpp:168-217) at those call sites with the same bodies as the device conversion
 * (csrc/mm_mvp.h) compiled for the host: results are identical to mm_mvp_convert_device's.  No
 * device work and no context: `params` are the sequence's (mm_create's), `epipoles` the
 * EpipoleList GEODESIC_CAMPOSE reads (a context's own list via mm_get_epipole_list, or NULL when
 * no query needs one).  Returns MM_OK or the lowest failing query's code (its result words 0);
 * first_bad (optional) = that query's index.  Re-entrant for distinct epipole lists; one thread
 * per list. */
int mm_mvp_convert_host(const mm_seq_params* params, mm_epipole_list* epipoles, const mm_mvp_query* queries, int n,
                        int32_t* mv_out, int* first_bad);

/* Single-block interpolation (InterpolationFilter::filterHor/filterVer on the device), for
 * parity tests of the integer pel pipeline.  comp 0 = luma 8-tap (16 phases), else chroma 4-tap
 * (32 phases).  `src` points at the block origin inside a host buffer; along the filtered axis
 * (columns for filterHor, rows for filterVer) the filter reads (taps/2 - 1) samples before the
 * block and taps/2 after it (luma 3 before / 4 after, chroma 1 / 2), nothing beyond the block on
 * the other axis; dst is host memory (w*h int16). */
int mm_filter(mm_ctx* ctx, int comp, int vertical, const int16_t* src, ptrdiff_t src_stride,
              int16_t* dst, ptrdiff_t dst_stride, int w, int h, int frac, int is_first,
              int is_last);

/* Original (source) luma picture of `poc` for the encoder SAD (the pcPatternKey / org buffer of
 * RdCost::xGetSAD); unpadded, picture origin at y[0]. */
int mm_upload_org(mm_ctx* ctx, int poc, const int16_t* y, ptrdiff_t stride_y, int src_is_device);

/* Encoder ME candidate evaluation (InterSearch::xMVReprojectionInterpolation + RdCost::xGetSAD,
 * EncoderLib/InterSearch.cpp:6277-6385, CommonLib/RdCost.cpp:482-517), batched:
 * for every block b and candidate (i, j) in [-range, range]^2 the block's luma is reprojected with
 * mv = (mv_hor + i*step, mv_ver + j*step) in its model, predicted as the reference does for the
 * encoder (rounded uni prediction, out-of-range margin 0) and compared with the original picture
 * of cur_poc.  sads (DEVICE memory, n * (2*range+1)^2 uint32) receives the SAD of candidate
 * c = (j + range) * (2*range + 1) + (i + range) at sads[b * (2*range+1)^2 + c].  step = 16 / 8 / 4
 * gives integer / half / quarter-pel windows.  Synchronous; the full SAD is returned where the
 * reference may stop early past its running best (same search decisions). */
int mm_sad_window(mm_ctx* ctx, int cur_poc, const mm_me_block* blocks, int n, int range, int step,
                  uint32_t* sads);
/* The same evaluation for a pattern of k candidate offsets shared by every block (1 <= k <= 64,
 * distinct, |offset| <= 4096 in 1/16 luma): candidate c of block b has
 * mv = (mv_hor + offsets[2c], mv_ver + offsets[2c+1]) and its SAD goes to sads[b * k + c] (DEVICE
 * memory).  The encoder's dependent steps -- xTZSearchHelp over the TZ 8-point square / diamond,
 * 2-point and star patterns (EncoderLib/InterSearch.cpp:474-526, xTZSearch :5350) and the 9-point
 * fractional refinements of xPatternRefinementProjected (:6168-6249) -- in one call per step for
 * all blocks: each block's setup work and each sub-block's MV-independent model head and original
 * samples are done once for its k candidates.  Same results as k range-0 mm_sad_window blocks. */
int mm_sad_pattern(mm_ctx* ctx, int cur_poc, const mm_me_block* blocks, int n, const int32_t* offsets, int k,
                   uint32_t* sads);

/* Device time of the last mm_pred_device / mm_pred_run / mm_sad_window / mm_mvp_convert_device
 * launch sequence (HIP events on the context stream around all of its launches), milliseconds.
 * MM_ERR_ARG if that sequence was a picture call made with call timing off. */
int mm_last_timing(mm_ctx* ctx, float* ms_total);

/* Call timing of the picture calls (mm_pred*, default on): the two events mm_last_timing reads.
 * Every event recorded on the context stream costs it ~4 us of a picture's ~0.2 ms, so a decoder
 * loop that does not read the time switches them off.  (No reference counterpart; the reference's
 * INTERPRED_PROFILING timers are compiled out by default.) */
int mm_set_call_timing(mm_ctx* ctx, int on);

/* Per-stage device time of the last launch sequence, recorded only while stage timing is on
 * (extra events between the launches): ms[0] planning (memset + k_plan_count + k_plan_place),
 * ms[1] k_setup, ms[2] k_reproj, ms[3] k_mc. */
int mm_set_stage_timing(mm_ctx* ctx, int on);
int mm_last_stage_timing(mm_ctx* ctx, float ms[4]);

/* Kernel timing of the interpolation kernel (k_mc_dev) inside an ordinary call sequence: while on,
 * every k_mc_dev launch is bracketed by a start / stop event pair bound to the dispatch itself
 * (no marker packets; under plan-ahead the stop event is also the plan slot's gate), so the
 * durations are those of the launches as they overlap the next picture's planning and
 * reprojection.  mm_kernel_times synchronises the context stream and returns the durations (ms)
 * of up to the last 256 launches since the timing was switched on or last read, oldest first, in
 * ms[0 .. *n); the count restarts.  (No reference counterpart; the bench's roofline reads it.) */
int mm_set_kernel_timing(mm_ctx* ctx, int on);
int mm_kernel_times(mm_ctx* ctx, float* ms, int cap, int* n);

/* Stripe pipelining of mm_pred_device / mm_pred_run (default 1, 1..64): the PU list is cut into
 * `stripes` contiguous ranges that are planned and predicted independently, alternating between
 * the context stream and an internal auxiliary stream that forks from and joins back into it, so
 * that one stripe's latency-bound planning kernels overlap another stripe's interpolation.  PUs
 * write disjoint samples: results do not depend on the setting.  Stage timing forces one stripe.
 * (No reference counterpart: the reference predicts PU by PU.) */
int mm_set_stripes(mm_ctx* ctx, int stripes);

/* The picture's DMVR enable (sps DMVR && !ph_dmvr_disabled; default off): with it on, PUs of an
 * mm_pred / mm_pred_device list flagged MM_PUF_DMVR run xProcessDMVRProjected's search (25-point
 * integer + parabolic sub-pel, InterPrediction.cpp:2442-2634) on their <= 16x16 sub-PUs inside the
 * same asynchronous launch sequence -- planning, search, decision, then the refined sub-PUs'
 * setup / reprojection / interpolation with the rest of the picture.  Forces one stripe.  With it
 * off, a flagged PU is rejected (MM_ERR_ARG).
 * Device memory: the DMVR work buffers are sized for the largest list the picture can hold, since
 * a device-resident list's DMVR share is unknown to the host -- per plan slot (two), about 310 bytes
 * per possible sub-PU (W*H/128 of them: the sub-PU record, its centre setups and centre terms, cost,
 * delta and survivor index): about 45 MB per slot, 90 MB per context at 6144x3072, allocated on the
 * first DMVR picture and kept until mm_destroy.  The 24 other offsets' setups, positions and costs of
 * a surviving sub-PU never leave the wave that searches it (round 4: 0.9 GB per context). */
int mm_set_dmvr(mm_ctx* ctx, int on);

/* Plan-ahead for mm_pred_device (default off): a picture's planning, setup and reprojection
 * kernels run on the internal auxiliary stream, gated only by the completion of the interpolation
 * kernel of the call TWO back (the last user of the plan buffers they overwrite), so they overlap
 * the previous picture's interpolation; the interpolation stays on the context stream, which waits
 * for them on the device, and a call returns without waiting for the GPU.  Contract while on: the
 * device PU list of call N is complete before call N is issued AND is not written by device work
 * that could still run after call N-2's interpolation -- i.e. it is written by the host, by device
 * work the caller has synchronised, or by work enqueued on the context stream before call N-2 was
 * issued.  A list written on the context stream between calls N-2 and N is NOT ordered before call
 * N's planning (synchronise first, or keep plan-ahead off).  mm_pred / mm_pred_prepare +
 * mm_pred_run copy and synchronise, so they always qualify.  Applies to one-stripe calls without
 * stage timing; results do not depend on the setting.  (No reference counterpart: VTM decodes a
 * picture's PUs inside its own CTU loop.) */
int mm_set_plan_ahead(mm_ctx* ctx, int on);

/* ---------------------------------------------------------------- bitstream side (host only)
 * The MM syntax a decoder parses around the hot path; bit-serial host code,
 * no context and no GPU.  Bit positions are MSB-first bit offsets into caller buffers, so the
 * fragments can be spliced into a caller's SPS / PH RBSP.
 *   mm_sps_mm_write / _read        <- VLCWriter.cpp:1110-1142 / VLCReader.cpp:1920-1980
 *                                     (sps_mpa_enabled_flag .. sps_global_epipole_i)
 *   mm_ph_epipole_write / _read    <- VLCWriter.cpp:2096-2109 / VLCReader.cpp:3354-3372
 *   mm_motion_model_candidates     <- the candidate order of CABACReader::motion_model
 *                                     (CABACReader.cpp:2179-2296, MMConfig.cpp:7-39)
 *   mm_motion_model_encode / _decode <- CABACWriter::motion_model / CABACReader::motion_model
 *                                     (CABACWriter.cpp:1984-2000, CABACReader.cpp:2300-2322) on
 *                                     VVC's CABAC engine (BinEncoder.cpp, BinDecoder.cpp) with the
 *                                     MotionModel contexts (Contexts.cpp:420-426) */
#define MM_MAX_CALIB_COEFFS 16   /* CALIBRATED_PROJECTION_MAX_NUM_COEFFS (CommonDef.h:442) */
#define MM_NUM_MODEL_IDS 11      /* MotionModelID CLASSIC .. GEODESIC_CAMPOSE (TypeDef.h:865-879) */

/* MMConfig's coded fields (CommonLib/MMConfig.h:15-30) */
typedef struct mm_sps_mm {
  int32_t mpa, t3d, tan, rot, ged, geda;  /* sps_{mpa,3dt,tan,rot,ged,geda}_enabled_flag */
  int32_t ged_flavor;                     /* sps_ged_flavor, coded iff ged || geda */
  int32_t mmmvp;                          /* sps_mmmvp_enabled_flag */
  int32_t mm_offset_4x4;                  /* sps_mm_offset_4x4, 0..4 */
  int32_t projection_fct;                 /* 0 EQUISOLID, 1 CALIBRATED, 2 EQUIRECTANGULAR */
  uint32_t focal_length_px, optical_center_x_px, optical_center_y_px;  /* EQUISOLID / CALIBRATED */
  uint32_t num_calibrated_coeffs;         /* CALIBRATED, <= MM_MAX_CALIB_COEFFS */
  int32_t calibrated_coeffs[MM_MAX_CALIB_COEFFS];  /* coded ue(v), stored int (VLCReader.cpp:1970) */
  int32_t global_epipole[3];              /* se(v), coded iff ged */
} mm_sps_mm;

/* Write the fragment at *bit_pos into buf (cap_bytes long; bits outside the fragment are left as
 * they are), advancing *bit_pos.  Every syntax element is written; when the multi-model flags are
 * all 0 only the six flags are.  MM_ERR_ARG: a value the reader rejects (mm_offset_4x4 outside
 * 0..4, projection_fct outside 0..2, more than 16 calibrated coefficients, a negative ue(v) field,
 * INT32_MIN epipole) or the buffer is too small. */
int mm_sps_mm_write(const mm_sps_mm* sps, uint8_t* buf, int64_t cap_bytes, int64_t* bit_pos);
/* Read the fragment at *bit_pos of a buffer holding nbits bits.  Fields not coded are 0 (the
 * MMConfig defaults).  MM_ERR_BITSTREAM on a range violation or truncation (*bit_pos unchanged). */
int mm_sps_mm_read(const uint8_t* buf, int64_t nbits, int64_t* bit_pos, mm_sps_mm* sps);
/* ph_signal_epipole_delta_flag (+ three se(v)), present iff the SPS enables multi-model AND GED;
 * the flag is 1 iff the delta is not {0, 0, 0}.  Nothing is written / read otherwise (delta = 0). */
int mm_ph_epipole_write(const mm_sps_mm* sps, const int32_t delta[3], uint8_t* buf, int64_t cap_bytes,
                        int64_t* bit_pos);
int mm_ph_epipole_read(const mm_sps_mm* sps, const uint8_t* buf, int64_t nbits, int64_t* bit_pos,
                       int32_t delta[3]);

/* The motion_model() candidate list of one PU, in coding order, into cand[MM_NUM_MODEL_IDS]; *n_cand
 * = the number of active models (getActiveMotionModels order: CLASSIC, MPA x3, 3DT, TAN, ROT,
 * GEODESIC_CAMPOSE, GEODESIC_X/Y/Z).  pred_type is CABACReader's m_mmPredType: 0 none (the
 * reference apps' setting, DecApp.cpp:895), 1 centre point, 2 voted, 3 sorted.  For 1-3,
 * col_models is the collocated picture's motion field on the 4x4 grid, [grid_h][grid_w][2] int8
 * (motionModel[list], -1 = INVALID), grid covering pic_w x pic_h; col_list = colFromL0Flag for
 * type 1 and eColRefPicList for 2 / 3 (CABACReader.cpp:2205); (x, y, w, h) the PU's luma area.
 * A predicted model the list does not hold leaves the order unchanged (the reference's
 * vector::erase(end()) is undefined there).  Ties: first maximum in model-id order (type 2), a
 * stable order (type 3).  MM_ERR_ARG on a bad argument or a field value outside -1..10. */
int mm_motion_model_candidates(const mm_sps_mm* sps, int pred_type, const int8_t* col_models, int grid_w,
                               int grid_h, int pic_w, int pic_h, int col_list, int x, int y, int w, int h,
                               int32_t* cand, int32_t* n_cand);

/* CABAC-code the motion_model() of n_pu PUs as one slice-data stream: the contexts initialised
 * for (slice_qp, init_type = slice type B 0 / P 1 / I 2 after the cabac_init_flag swap), the PUs'
 * bins in order, then end_of_slice_segment_flag (terminating bin 1), the arithmetic coder's flush
 * and rbsp trailing bits.  cand: n_pu rows of MM_NUM_MODEL_IDS (mm_motion_model_candidates output;
 * the first n_cand entries of each row are used), coding_depth = m_mmCodingDepth (the apps use 9).
 * affine (optional, n_pu bytes): affine PUs code nothing and must be CLASSIC (CABACWriter.cpp:1860).
 * With no multi-model flag set, no PU codes bins and every model must be CLASSIC.
 * encode: *nbytes = stream length; MM_ERR_ARG if a model is not in its PU's list or cap is short.
 * decode: models_out[n_pu]; MM_ERR_BITSTREAM if the stream is malformed, ends early, or does not
 * end with the terminating bin and the stop pattern exactly at its last byte (BinDecoder.cpp:85-91). */
int mm_motion_model_encode(const mm_sps_mm* sps, int slice_qp, int init_type, int coding_depth, int n_pu,
                           const int32_t* cand, const uint8_t* affine, const int32_t* models, uint8_t* out,
                           int64_t cap_bytes, int64_t* nbytes);
int mm_motion_model_decode(const mm_sps_mm* sps, int slice_qp, int init_type, int coding_depth, int n_pu,
                           const int32_t* cand, const uint8_t* affine, const uint8_t* in, int64_t nbytes,
                           int32_t* models_out);

#ifdef __cplusplus
}
#endif
#endif /* MM360_H */
