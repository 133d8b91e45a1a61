"""Python host interface of the MI355X 360-degree multi-model motion-compensation path.

Mirrors the reference's C++ call surface for this path:

    MVReprojection::init                          -> MMContext(...)          (mm_create)
    EpipoleList::addEpipole                       -> MMContext.set_epipole   (mm_set_epipole)
    Picture reconstruction planes                 -> MMContext.upload_ref    (mm_upload_ref)
    MVReprojection::reprojectMotionVectorSubblocks-> MMContext.reproject_motion_vector_subblocks
    InterPrediction::xPredInterBlkMM (+ addAvg / addWeightedAvg) -> MMContext.predict (mm_pred)
      same, PU list resident in HBM               -> MMContext.predict_device (mm_pred_device)
    InterPrediction::xPredInterBlkMM, one list    -> MMContext.predict_list  (mm_pred_list)
    InterpolationFilter::filterHor / filterVer    -> MMContext.filter_hor / filter_ver
    InterSearch::xMVReprojectionInterpolation + RdCost::xGetSAD (encoder)
                                                  -> MMContext.sad_window (dense windows) /
                                                     MMContext.sad_pattern (TZ / refinement steps)
    VLCReader / CABACReader MM syntax             -> mm360.syntax (host only)

Everything runs through the HIP C-ABI library ``lib/libmm360.so`` (include/mm360.h).  There is
no CPU fallback: constructing a context without the library or without a GPU raises.
Reference citations are into /root/reference/source/Lib/CommonLib.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, byref, c_int, c_int32, c_uint32, c_void_p, c_float
from typing import Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "lib", "libmm360.so")
# MM360_LIB: a diagnostic build of the same library (tools/race_probe.sh runs the GPU suite on the
# MM_RACE_PROBE variant); unset, the in-tree product library
if os.environ.get("MM360_LIB"):
    LIB_PATH = os.path.abspath(os.environ["MM360_LIB"])

# MotionModelID (TypeDef.h:865-879)
CLASSIC, MPA_FRONT_BACK, MPA_LEFT_RIGHT, MPA_TOP_BOTTOM = 0, 1, 2, 3
TANGENTIAL, THREE_D_TRANSLATIONAL, ROTATIONAL = 4, 5, 6
GEODESIC_X, GEODESIC_Y, GEODESIC_Z, GEODESIC_CAMPOSE = 7, 8, 9, 10
MODEL_NAMES = {
    CLASSIC: "CLASSIC", MPA_FRONT_BACK: "MPA_FRONT_BACK", MPA_LEFT_RIGHT: "MPA_LEFT_RIGHT",
    MPA_TOP_BOTTOM: "MPA_TOP_BOTTOM", TANGENTIAL: "TANGENTIAL",
    THREE_D_TRANSLATIONAL: "THREE_D_TRANSLATIONAL", ROTATIONAL: "ROTATIONAL",
    GEODESIC_X: "GEODESIC_X", GEODESIC_Y: "GEODESIC_Y", GEODESIC_Z: "GEODESIC_Z",
    GEODESIC_CAMPOSE: "GEODESIC_CAMPOSE",
}

MM_OK, MM_ERR_ARG, MM_ERR_HIP, MM_ERR_NOREF, MM_ERR_NOEPIPOLE, MM_ERR_MODEL, MM_ERR_NODEV, MM_ERR_BITSTREAM = range(8)
ERROR_NAMES = {
    MM_ERR_ARG: "MM_ERR_ARG", MM_ERR_HIP: "MM_ERR_HIP", MM_ERR_NOREF: "MM_ERR_NOREF",
    MM_ERR_NOEPIPOLE: "MM_ERR_NOEPIPOLE", MM_ERR_MODEL: "MM_ERR_MODEL", MM_ERR_NODEV: "MM_ERR_NODEV",
    MM_ERR_BITSTREAM: "MM_ERR_BITSTREAM",
}

# Every entry point declared in include/mm360.h (checked by the CPU test suite)
EXPORTED_SYMBOLS = (
    "mm_create", "mm_destroy", "mm_set_stream", "mm_synchronize", "mm_last_error", "mm_get_version",
    "mm_set_epipole", "mm_upload_ref", "mm_release_ref", "mm_reproject", "mm_pred",
    "mm_pred_device", "mm_pred_status", "mm_pred_prepare", "mm_pred_run", "mm_filter", "mm_last_timing", "mm_set_call_timing",
    "mm_set_stage_timing", "mm_last_stage_timing", "mm_upload_org", "mm_sad_window", "mm_pred_dmvr", "mm_mvp_convert",
    "mm_set_stripes", "mm_set_plan_ahead", "mm_pred_list", "mm_derive_effective_blocks", "mm_epipole_list_create",
    "mm_epipole_list_destroy", "mm_get_epipole_list", "mm_epipole_add", "mm_epipole_make_available", "mm_epipole_has",
    "mm_epipole_find", "mm_epipole_derive_predictor", "mm_epipole_count", "mm_mvp_convert_device", "mm_mvp_status", "mm_set_dmvr",
    "mm_set_mvp_stream", "mm_mvp_convert_host", "mm_pred_device_multi", "mm_set_kernel_timing", "mm_kernel_times",
    "mm_stripe_packed_dwords", "mm_pack_samples", "mm_upload_ref_packed", "mm_upload_ref_stripes",
    "mm_sad_pattern", "mm_sps_mm_write", "mm_sps_mm_read", "mm_ph_epipole_write", "mm_ph_epipole_read", "mm_motion_model_candidates",
    "mm_motion_model_encode", "mm_motion_model_decode",
)

BCW_DEFAULT = 2  # CommonDef.h:348-349; g_BcwWeights = {-2, 3, 4, 5, 10} (Rom.cpp:203)


class MMError(RuntimeError):
    """Status != MM_OK from the C-ABI (the reference would throw from CHECK, TypeDef.h:1120-1148)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERROR_NAMES.get(code, code)}: {msg}")
        self.code = code


class SeqParams(ctypes.Structure):
    _fields_ = [
        ("width", c_int32), ("height", c_int32), ("chroma_format", c_int32), ("bit_depth", c_int32),
        ("max_cu_width", c_int32), ("max_cu_height", c_int32), ("mm_offset4x4", c_int32),
        ("ged_flavor", c_int32), ("active_models", c_uint32),
    ]


# numpy views of mm_block_desc / mm_pu_desc (all int32, packed)
BLOCK_DTYPE = np.dtype([("x", "<i4"), ("y", "<i4"), ("w", "<i4"), ("h", "<i4"), ("mv_hor", "<i4"),
                        ("mv_ver", "<i4"), ("model", "<i4"), ("comp", "<i4"), ("cur_poc", "<i4"),
                        ("ref_poc", "<i4")])
PU_DTYPE = np.dtype([("x", "<i4"), ("y", "<i4"), ("w", "<i4"), ("h", "<i4"), ("mv", "<i4", (2, 2)),
                     ("ref_poc", "<i4", (2,)), ("model", "<i4", (2,)), ("bcw_idx", "<i4"),
                     ("flags", "<u4"), ("reserved", "<i4", (2,))])
ME_BLOCK_DTYPE = np.dtype([("x", "<i4"), ("y", "<i4"), ("w", "<i4"), ("h", "<i4"), ("mv_hor", "<i4"),
                           ("mv_ver", "<i4"), ("model", "<i4"), ("ref_poc", "<i4"), ("sub_shift", "<i4")])
MVP_QUERY_DTYPE = np.dtype([(n, "<i4") for n in (
    "pos_x", "pos_y", "mv_hor", "mv_ver", "model_orig", "model_desired", "shift_hor", "shift_ver", "cur_poc_orig",
    "ref_poc_orig", "cur_poc_desired", "ref_poc_desired", "cand_x", "cand_y", "cand_w", "cand_h", "cur_x", "cur_y",
    "cur_w", "cur_h")])
assert BLOCK_DTYPE.itemsize == 40 and PU_DTYPE.itemsize == 64 and ME_BLOCK_DTYPE.itemsize == 36
assert MVP_QUERY_DTYPE.itemsize == 80
# mm_pu_motion: a decoded PU for the effective-block derivation (mm_derive_effective_blocks)
PU_MOTION_DTYPE = np.dtype([("pu", PU_DTYPE), ("flags", "<u4"), ("cur_poc", "<i4"), ("sub_motion", "<i4"),
                            ("reserved", "<i4")])
assert PU_MOTION_DTYPE.itemsize == 80
# MM_PU_* flags (include/mm360.h)
PU_MERGE, PU_SUBPU, PU_CIIP, PU_SMVD, PU_MMVD, PU_MVREFINE = 0x1, 0x2, 0x4, 0x8, 0x10, 0x20
PU_WEIGHTED, PU_LONGTERM, PU_REF_SCALED, PU_MMVD_ENC2 = 0x40, 0x80, 0x100, 0x200
PUF_DMVR = 0x1  # mm_pu_desc.flags: MM_PUF_DMVR


MAX_PICS = 4  # MM_MAX_PICS: pictures per mm_pred_device_multi call


class PicJob(ctypes.Structure):
    """mm_pic_job: one picture of mm_pred_device_multi (device PU list and destination planes)."""
    _fields_ = [("cur_poc", c_int32), ("d_pus", c_void_p), ("n", c_int32), ("dst_y", c_void_p),
                ("dst_stride_y", ctypes.c_ssize_t), ("dst_cb", c_void_p), ("dst_cr", c_void_p),
                ("dst_stride_c", ctypes.c_ssize_t)]


class ToolFlags(ctypes.Structure):
    """mm_tool_flags: SPS / PPS / PH switches of the current picture."""
    _fields_ = [("bdof", c_int32), ("dmvr", c_int32), ("bcw", c_int32), ("wp_bi", c_int32)]


def new_pus(n: int) -> np.ndarray:
    """n zeroed mm_pu_desc records with bcw_idx = BCW_DEFAULT (plain addAvg for bi PUs)."""
    out = np.zeros(n, dtype=PU_DTYPE)
    out["bcw_idx"] = BCW_DEFAULT
    return out


def active_mask(models: Sequence[int]) -> int:
    """MMConfig active-model list as a bit mask; CLASSIC is always active (MMConfig.cpp:7-39)."""
    m = 1 << CLASSIC
    for x in models:
        m |= 1 << int(x)
    return m


def seq_params(width: int, height: int, models: Sequence[int], chroma_format: int = 1,
               bit_depth: int = 10, max_cu: int = 128, mm_offset4x4: int = 1,
               ged_flavor: int = 1) -> SeqParams:
    """Defaults are the reference's hard-coded MM settings (EncApp.cpp:754-768) and RA cfg."""
    return SeqParams(width, height, chroma_format, bit_depth, max_cu, max_cu, mm_offset4x4,
                     ged_flavor, active_mask(models))


_lib = None


def load_library() -> ctypes.CDLL:
    """Load the HIP library; raise if it has not been built (no fallback path exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise FileNotFoundError(f"{LIB_PATH} missing: build it with `make -C vvc-extension-mm_amd` "
                                "or __graft_entry__.build()")
    lib = ctypes.CDLL(LIB_PATH)
    vp = c_void_p
    sig = {
        "mm_create": (c_int, [POINTER(SeqParams), c_int, POINTER(vp)]),
        "mm_destroy": (c_int, [vp]),
        "mm_set_stream": (c_int, [vp, vp]),
        "mm_synchronize": (c_int, [vp]),
        "mm_last_error": (ctypes.c_char_p, [vp]),
        "mm_get_version": (c_int, []),
        "mm_set_epipole": (c_int, [vp, c_int, c_int, POINTER(c_int32)]),
        "mm_upload_ref": (c_int, [vp, c_int, vp, ctypes.c_ssize_t, vp, vp, ctypes.c_ssize_t, c_int]),
        "mm_release_ref": (c_int, [vp, c_int]),
        "mm_reproject": (c_int, [vp, vp, c_int, vp]),
        "mm_pred": (c_int, [vp, c_int, vp, c_int, vp, ctypes.c_ssize_t, vp, vp, ctypes.c_ssize_t]),
        "mm_pred_device": (c_int, [vp, c_int, vp, c_int, vp, ctypes.c_ssize_t, vp, vp, ctypes.c_ssize_t]),
        "mm_pred_status": (c_int, [vp, POINTER(c_int)]),
        "mm_pred_prepare": (c_int, [vp, c_int, vp, c_int]),
        "mm_pred_run": (c_int, [vp, vp, ctypes.c_ssize_t, vp, vp, ctypes.c_ssize_t]),
        "mm_filter": (c_int, [vp, c_int, c_int, vp, ctypes.c_ssize_t, vp, ctypes.c_ssize_t, c_int, c_int,
                              c_int, c_int, c_int]),
        "mm_last_timing": (c_int, [vp, POINTER(c_float)]),
        "mm_set_call_timing": (c_int, [vp, c_int]),
        "mm_set_stage_timing": (c_int, [vp, c_int]),
        "mm_upload_org": (c_int, [vp, c_int, vp, ctypes.c_ssize_t, c_int]),
        "mm_mvp_convert": (c_int, [vp, vp, c_int, vp]),
        "mm_mvp_convert_device": (c_int, [vp, vp, c_int, vp]),
        "mm_mvp_status": (c_int, [vp, POINTER(c_int)]),
        "mm_set_dmvr": (c_int, [vp, c_int]),
        "mm_set_mvp_stream": (c_int, [vp, vp]),
        "mm_pred_dmvr": (c_int, [vp, c_int, vp, c_int, vp, ctypes.c_ssize_t, vp, vp, ctypes.c_ssize_t, vp]),
        "mm_sad_window": (c_int, [vp, c_int, vp, c_int, c_int, c_int, vp]),
        "mm_sad_pattern": (c_int, [vp, c_int, vp, c_int, vp, c_int, vp]),
        "mm_last_stage_timing": (c_int, [vp, POINTER(c_float)]),
        "mm_set_kernel_timing": (c_int, [vp, c_int]),
        "mm_stripe_packed_dwords": (ctypes.c_int64, [vp, c_int, c_int]),
        "mm_pack_samples": (c_int, [vp, vp, ctypes.c_int64, vp]),
        "mm_upload_ref_packed": (c_int, [vp, c_int, vp, c_int, c_int]),
        "mm_upload_ref_stripes": (c_int, [vp, c_int, vp, c_int, c_int]),
        "mm_kernel_times": (c_int, [vp, POINTER(c_float), c_int, POINTER(c_int)]),
        "mm_set_stripes": (c_int, [vp, c_int]),
        "mm_set_plan_ahead": (c_int, [vp, c_int]),
        "mm_pred_list": (c_int, [vp, c_int, vp, c_int, c_int, c_int, vp, ctypes.c_ssize_t, vp, vp,
                                 ctypes.c_ssize_t]),
        "mm_derive_effective_blocks": (c_int, [POINTER(ToolFlags), vp, c_int, vp, vp, c_int, POINTER(c_int), vp,
                                               c_int, POINTER(c_int)]),
        "mm_epipole_list_create": (vp, []),
        "mm_epipole_list_destroy": (None, [vp]),
        "mm_get_epipole_list": (vp, [vp]),
        "mm_epipole_add": (c_int, [vp, c_int, c_int, POINTER(c_int32), c_int]),
        "mm_epipole_make_available": (c_int, [vp, c_int]),
        "mm_epipole_has": (c_int, [vp, c_int, c_int]),
        "mm_epipole_find": (c_int, [vp, c_int, c_int, POINTER(c_int32)]),
        "mm_epipole_derive_predictor": (c_int, [vp, c_int, POINTER(c_int32)]),
        "mm_epipole_count": (c_int, [vp]),
        "mm_mvp_convert_host": (c_int, [POINTER(SeqParams), vp, vp, c_int, vp, POINTER(c_int)]),
        "mm_pred_device_multi": (c_int, [vp, vp, c_int]),
        # bitstream side (mm360.syntax); the mm_sps_mm struct is passed as a pointer
        "mm_sps_mm_write": (c_int, [vp, vp, ctypes.c_int64, POINTER(ctypes.c_int64)]),
        "mm_sps_mm_read": (c_int, [vp, ctypes.c_int64, POINTER(ctypes.c_int64), vp]),
        "mm_ph_epipole_write": (c_int, [vp, POINTER(c_int32), vp, ctypes.c_int64, POINTER(ctypes.c_int64)]),
        "mm_ph_epipole_read": (c_int, [vp, vp, ctypes.c_int64, POINTER(ctypes.c_int64), POINTER(c_int32)]),
        "mm_motion_model_candidates": (c_int, [vp, c_int, vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                               c_int, POINTER(c_int32), POINTER(c_int32)]),
        "mm_motion_model_encode": (c_int, [vp, c_int, c_int, c_int, c_int, vp, vp, vp, vp, ctypes.c_int64,
                                           POINTER(ctypes.c_int64)]),
        "mm_motion_model_decode": (c_int, [vp, c_int, c_int, c_int, c_int, vp, vp, vp, ctypes.c_int64, vp]),
    }
    default_lib = os.path.abspath(LIB_PATH) == os.path.join(os.path.dirname(_HERE), "lib", "libmm360.so")
    for name, (res, args) in sig.items():
        if not default_lib and not hasattr(lib, name):
            continue  # an older A/B build (bench.py --lib) without a newer entry point
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def derive_effective_blocks(tools: ToolFlags, pus: np.ndarray, sub_motion: Optional[np.ndarray] = None):
    """InterPrediction::motionCompensation's effective blocks of decoded PUs (PU_MOTION_DTYPE):
    (PUs for mm_pred, PUs for mm_pred_dmvr), both PU_DTYPE.  Host code, no GPU."""
    lib = load_library()
    pus = np.ascontiguousarray(pus, dtype=PU_MOTION_DTYPE)
    sub = np.ascontiguousarray(sub_motion if sub_motion is not None else new_pus(0), dtype=PU_DTYPE)
    cap = int(((pus["pu"]["w"] // 4).astype(np.int64) * (pus["pu"]["h"] // 4)).sum()) + 1  # <= one per 4x4
    mc, dm = new_pus(cap), new_pus(cap)
    n_mc, n_dmvr = c_int(0), c_int(0)
    rc = lib.mm_derive_effective_blocks(byref(tools), c_void_p(pus.ctypes.data), len(pus),
                                        c_void_p(sub.ctypes.data) if len(sub) else None, c_void_p(mc.ctypes.data),
                                        cap, byref(n_mc), c_void_p(dm.ctypes.data), cap, byref(n_dmvr))
    if rc != MM_OK:
        raise MMError(rc, "mm_derive_effective_blocks: invalid PU")
    return mc[:n_mc.value], dm[:n_dmvr.value]


class EpipoleList:
    """EpipoleList (SRC/EpipoleList.{h,cpp}) through the C-ABI: Q24 epipoles keyed by
    (curPOC, refPOC) with -1 wildcards and availability.  Standalone (no GPU) or a context's own
    list (MMContext.epipole_list())."""

    def __init__(self, handle=None, owner=None):
        self.lib = load_library()
        self._owned = handle is None
        self.h = c_void_p(self.lib.mm_epipole_list_create()) if handle is None else c_void_p(handle)
        self._owner = owner  # keeps the context alive

    def __del__(self):
        try:
            if self._owned and self.h:
                self.lib.mm_epipole_list_destroy(self.h)
        except Exception:
            pass

    def add(self, cur_poc: int, ref_poc: int, q24: Sequence[int], make_available: bool = False):
        rc = self.lib.mm_epipole_add(self.h, cur_poc, ref_poc, (c_int32 * 3)(*[int(v) for v in q24]),
                                     int(make_available))
        if rc:
            raise MMError(rc, "mm_epipole_add")

    def make_available(self, cur_poc: int):
        self.lib.mm_epipole_make_available(self.h, cur_poc)

    def has(self, cur_poc: int, ref_poc: int) -> bool:
        return bool(self.lib.mm_epipole_has(self.h, cur_poc, ref_poc))

    def find(self, cur_poc: int, ref_poc: int):
        q = (c_int32 * 3)()
        rc = self.lib.mm_epipole_find(self.h, cur_poc, ref_poc, q)
        if rc:
            raise MMError(rc, f"no epipole for ({cur_poc}, {ref_poc})")
        return tuple(int(v) for v in q)

    def derive_predictor(self, cur_poc: int):
        q = (c_int32 * 3)()
        rc = self.lib.mm_epipole_derive_predictor(self.h, cur_poc, q)
        if rc:
            raise MMError(rc, "derivePredictor")
        return tuple(int(v) for v in q)

    def count(self) -> int:
        return int(self.lib.mm_epipole_count(self.h))


def mvp_convert_host(params: SeqParams, queries: np.ndarray, epipoles: Optional[EpipoleList] = None) -> np.ndarray:
    """mm_mvp_convert_host: motionVectorInDesiredMotionModel query by query on this host thread
    (the spatial merge / AMVP candidates VTM converts in decoding order, UnitTools.cpp:2930-2992,
    3134-3167), with the same bodies as the device conversion.  No GPU.  int32 [n, 2] MVs; raises
    MMError with the lowest failing query's code."""
    lib = load_library()
    q = np.ascontiguousarray(queries, dtype=MVP_QUERY_DTYPE)
    out = np.zeros((max(len(q), 1), 2), dtype=np.int32)
    bad = c_int(-1)
    rc = lib.mm_mvp_convert_host(byref(params), epipoles.h if epipoles is not None else None,
                                 c_void_p(q.ctypes.data), len(q), c_void_p(out.ctypes.data), byref(bad))
    if rc != MM_OK:
        raise MMError(rc, f"mm_mvp_convert_host: query {bad.value}")
    return out[:len(q)]


def _check_sad_out(out, n: int) -> None:
    """The SAD output the library writes n uint32 into: a contiguous 4-byte CUDA tensor that large
    (the C-ABI takes a bare device pointer and cannot check it)."""
    if not getattr(out, "is_cuda", False) or out.element_size() != 4 or not out.is_contiguous() or out.numel() < n:
        raise MMError(MM_ERR_ARG, f"SAD output must be a contiguous 4-byte CUDA tensor of >= {n} elements")


def _ptr(a) -> int:
    """Address of a numpy array or a torch tensor (host or device)."""
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return int(a.data_ptr())


def _is_device(a) -> bool:
    return not isinstance(a, np.ndarray) and getattr(a, "is_cuda", False)


def pus_to_device(pus: np.ndarray, device: int = 0):
    """Copy a PU_DTYPE array into device memory (int32 CUDA tensor of 16 words per PU)."""
    import torch
    pus = np.ascontiguousarray(pus, dtype=PU_DTYPE)
    words = pus.view(np.int32).reshape(len(pus), PU_DTYPE.itemsize // 4)
    return torch.from_numpy(words.copy()).to(f"cuda:{device}")


def queries_to_device(q: np.ndarray, device: int = 0):
    """Copy an MVP_QUERY_DTYPE array into device memory (int32 CUDA tensor, 20 words per query)."""
    import torch
    q = np.ascontiguousarray(q, dtype=MVP_QUERY_DTYPE)
    words = q.view(np.int32).reshape(len(q), MVP_QUERY_DTYPE.itemsize // 4)
    return torch.from_numpy(words.copy()).to(f"cuda:{device}")


def subblock_count(w: int, h: int, comp: int) -> int:
    sb = 2 if comp else 4
    return (w // sb) * (h // sb)


class MMContext:
    """One decoder instance's MM motion-compensation context on one GPU."""

    def __init__(self, params: SeqParams, device: int = 0):
        self.lib = load_library()
        self.params = params
        h = c_void_p()
        rc = self.lib.mm_create(byref(params), device, byref(h))
        if rc != MM_OK:
            raise MMError(rc, "mm_create failed (no HIP device, or invalid parameters)")
        self.h = h
        self.device = device

    # -- lifecycle ---------------------------------------------------------------------------
    def close(self):
        if getattr(self, "h", None):
            self.lib.mm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, rc: int):
        if rc != MM_OK:
            msg = self.lib.mm_last_error(self.h)
            raise MMError(rc, msg.decode() if msg else "")

    def set_stream(self, stream_handle: int):
        self._check(self.lib.mm_set_stream(self.h, c_void_p(stream_handle)))

    def synchronize(self):
        self._check(self.lib.mm_synchronize(self.h))

    # -- EpipoleList -------------------------------------------------------------------------
    def epipole_list(self) -> "EpipoleList":
        """The context's own EpipoleList (used for every GEODESIC_CAMPOSE lookup)."""
        return EpipoleList(self.lib.mm_get_epipole_list(self.h), owner=self)

    def set_epipole(self, cur_poc: int, ref_poc: int, q24: Sequence[int]):
        arr = (c_int32 * 3)(*[int(v) for v in q24])
        self._check(self.lib.mm_set_epipole(self.h, cur_poc, ref_poc, arr))

    # -- reference pictures ------------------------------------------------------------------
    def upload_ref(self, poc: int, y, cb=None, cr=None):
        """Planes: 2-D int16 numpy arrays (host) or torch int16 CUDA tensors (device)."""
        dev = _is_device(y)
        sy = y.strides[0] // 2 if isinstance(y, np.ndarray) else y.stride(0)
        sc = 0
        if cb is not None:
            sc = cb.strides[0] // 2 if isinstance(cb, np.ndarray) else cb.stride(0)
        self._check(self.lib.mm_upload_ref(self.h, poc, c_void_p(_ptr(y)), sy,
                                           c_void_p(_ptr(cb)) if cb is not None else None,
                                           c_void_p(_ptr(cr)) if cr is not None else None, sc, int(dev)))

    def release_ref(self, poc: int):
        self._check(self.lib.mm_release_ref(self.h, poc))

    # -- MVReprojection ----------------------------------------------------------------------
    def reproject(self, blocks: np.ndarray) -> np.ndarray:
        """Batched reprojectMotionVectorSubblocks: BLOCK_DTYPE array -> int32 [sum N_b, 2]."""
        blocks = np.ascontiguousarray(blocks, dtype=BLOCK_DTYPE)
        total = int(sum(subblock_count(int(b["w"]), int(b["h"]), int(b["comp"])) for b in blocks))
        out = np.zeros((max(total, 1), 2), dtype=np.int32)
        self._check(self.lib.mm_reproject(self.h, c_void_p(blocks.ctypes.data), len(blocks),
                                          c_void_p(out.ctypes.data)))
        return out[:total]

    def reproject_motion_vector_subblocks(self, position, size, mv, model, comp, cur_poc=0, ref_poc=0):
        """Single-call twin of MVReprojection::reprojectMotionVectorSubblocks
        (MVReprojection.h:54-58): returns the fixed-point X and Y arrays shaped (rows, cols) like
        the reference's Eigen::ArrayXXi pair."""
        b = np.zeros(1, dtype=BLOCK_DTYPE)
        b[0] = (position[0], position[1], size[0], size[1], mv[0], mv[1], model, comp, cur_poc, ref_poc)
        r = self.reproject(b)
        sb = 2 if comp else 4
        rows, cols = size[1] // sb, size[0] // sb
        return (r[:, 0].reshape(cols, rows).T.copy(), r[:, 1].reshape(cols, rows).T.copy())

    # -- InterPrediction ---------------------------------------------------------------------
    def predict(self, cur_poc: int, pus: np.ndarray, dst_y, dst_cb=None, dst_cr=None):
        """Batched xPredInterBlkMM + xWeightedAverage over a picture's PU list into device planes."""
        pus = np.ascontiguousarray(pus, dtype=PU_DTYPE)
        self._check(self.lib.mm_pred(self.h, cur_poc, c_void_p(pus.ctypes.data), len(pus),
                                     c_void_p(_ptr(dst_y)), dst_y.stride(0),
                                     c_void_p(_ptr(dst_cb)) if dst_cb is not None else None,
                                     c_void_p(_ptr(dst_cr)) if dst_cr is not None else None,
                                     dst_cb.stride(0) if dst_cb is not None else 0))

    def predict_list(self, cur_poc: int, pus: np.ndarray, list_: int, hp: bool, dst_y=None, dst_cb=None,
                     dst_cr=None):
        """xPredInterBlkMM of one reference list of every PU (mm_pred_list): hp=True gives the
        14-bit bi=true intermediate, hp=False the rounded and clipped prediction.  A plane left
        None is not predicted."""
        pus = np.ascontiguousarray(pus, dtype=PU_DTYPE)
        self._check(self.lib.mm_pred_list(self.h, cur_poc, c_void_p(pus.ctypes.data), len(pus), int(list_), int(hp),
                                          c_void_p(_ptr(dst_y)) if dst_y is not None else None,
                                          dst_y.stride(0) if dst_y is not None else 0,
                                          c_void_p(_ptr(dst_cb)) if dst_cb is not None else None,
                                          c_void_p(_ptr(dst_cr)) if dst_cr is not None else None,
                                          dst_cb.stride(0) if dst_cb is not None else 0))

    def mvp_convert(self, queries: np.ndarray) -> np.ndarray:
        """Batched MVReprojection::motionVectorInDesiredMotionModel: int32 [n, 2] MVs."""
        q = np.ascontiguousarray(queries, dtype=MVP_QUERY_DTYPE)
        out = np.zeros((max(len(q), 1), 2), dtype=np.int32)
        self._check(self.lib.mm_mvp_convert(self.h, c_void_p(q.ctypes.data), len(q), c_void_p(out.ctypes.data)))
        return out[:len(q)]

    def mvp_convert_device(self, d_queries, d_out):
        """mm_mvp_convert_device: `d_queries` a CUDA tensor of MVP_QUERY_DTYPE records (e.g.
        queries_to_device(q)), `d_out` an int32 CUDA tensor of 2 words per query.  Asynchronous on
        the context stream; errors surface at mvp_status() / synchronize()."""
        n = d_queries.numel() * d_queries.element_size() // MVP_QUERY_DTYPE.itemsize
        import torch
        assert d_out.numel() >= 2 * n and d_out.dtype == torch.int32
        self._check(self.lib.mm_mvp_convert_device(self.h, c_void_p(_ptr(d_queries)), n, c_void_p(_ptr(d_out))))

    def set_mvp_stream(self, stream_handle):
        """mm_set_mvp_stream: MM-MVP conversions on this HIP stream (None: the context stream)."""
        self._check(self.lib.mm_set_mvp_stream(self.h, c_void_p(stream_handle) if stream_handle else None))

    def mvp_status(self):
        """(code, first failing query) of the last mm_mvp_convert_device; raises MMError on failure."""
        bad = c_int(-1)
        self._check(self.lib.mm_mvp_status(self.h, ctypes.byref(bad)))

    def predict_dmvr(self, cur_poc: int, pus: np.ndarray, dst_y, dst_cb=None, dst_cr=None) -> np.ndarray:
        """MM-DMVR PUs (xProcessDMVRProjected): refined bi prediction into the device planes;
        returns the L0 MV delta (1/16 luma) of every <= 16x16 sub-PU, PU after PU, raster order."""
        pus = np.ascontiguousarray(pus, dtype=PU_DTYPE)
        nsub = int(sum(((int(u["w"]) + 15) // 16) * ((int(u["h"]) + 15) // 16) for u in pus))
        mvd = np.zeros((max(nsub, 1), 2), dtype=np.int32)
        self._check(self.lib.mm_pred_dmvr(self.h, cur_poc, c_void_p(pus.ctypes.data), len(pus),
                                          c_void_p(_ptr(dst_y)), dst_y.stride(0),
                                          c_void_p(_ptr(dst_cb)) if dst_cb is not None else None,
                                          c_void_p(_ptr(dst_cr)) if dst_cr is not None else None,
                                          dst_cb.stride(0) if dst_cb is not None else 0,
                                          c_void_p(mvd.ctypes.data)))
        return mvd[:nsub]

    def predict_device(self, cur_poc: int, d_pus, dst_y, dst_cb=None, dst_cr=None):
        """Whole picture path on the device from a device-resident PU list: `d_pus` is a CUDA
        tensor holding PU_DTYPE records (e.g. pus_to_device(pus)).  Asynchronous on the context
        stream; validation errors surface at status() / synchronize()."""
        n = d_pus.numel() * d_pus.element_size() // PU_DTYPE.itemsize
        self._check(self.lib.mm_pred_device(self.h, cur_poc, c_void_p(_ptr(d_pus)), n,
                                            c_void_p(_ptr(dst_y)), dst_y.stride(0),
                                            c_void_p(_ptr(dst_cb)) if dst_cb is not None else None,
                                            c_void_p(_ptr(dst_cr)) if dst_cr is not None else None,
                                            dst_cb.stride(0) if dst_cb is not None else 0))

    def predict_device_multi(self, pictures):
        """mm_pred_device_multi: independent pictures in one launch chain.  pictures = [(cur_poc,
        d_pus, dst_y, dst_cb, dst_cr)] (CUDA tensors / raw device addresses with strides given as
        (ptr, stride) pairs are not accepted here: tensors only), at most MAX_PICS."""
        assert 1 <= len(pictures) <= MAX_PICS
        jobs = (PicJob * len(pictures))()
        for q, (cur, d_pus, dy, dcb, dcr) in enumerate(pictures):
            jobs[q] = PicJob(cur, _ptr(d_pus), d_pus.numel() * d_pus.element_size() // PU_DTYPE.itemsize,
                             _ptr(dy), dy.stride(0), _ptr(dcb) if dcb is not None else None,
                             _ptr(dcr) if dcr is not None else None, dcb.stride(0) if dcb is not None else 0)
        self._check(self.lib.mm_pred_device_multi(self.h, jobs, len(pictures)))

    def predict_device_multi_raw(self, pictures):
        """mm_pred_device_multi into raw device addresses: pictures = [(cur_poc, d_pus, ptr_y, stride_y,
        ptr_cb, ptr_cr, stride_c)]."""
        assert 1 <= len(pictures) <= MAX_PICS
        jobs = (PicJob * len(pictures))()
        for q, (cur, d_pus, py, sy, pcb, pcr, sc) in enumerate(pictures):
            jobs[q] = PicJob(cur, _ptr(d_pus), d_pus.numel() * d_pus.element_size() // PU_DTYPE.itemsize,
                             py, sy, pcb, pcr, sc)
        self._check(self.lib.mm_pred_device_multi(self.h, jobs, len(pictures)))

    def status(self):
        """Deferred validation result of the last device-planned call: (code, first_bad_pu)."""
        bad = c_int(-1)
        rc = self.lib.mm_pred_status(self.h, byref(bad))
        return rc, int(bad.value)

    def prepare(self, cur_poc: int, pus: np.ndarray):
        pus = np.ascontiguousarray(pus, dtype=PU_DTYPE)
        self._check(self.lib.mm_pred_prepare(self.h, cur_poc, c_void_p(pus.ctypes.data), len(pus)))

    def run(self, dst_y, dst_cb=None, dst_cr=None):
        self._check(self.lib.mm_pred_run(self.h, c_void_p(_ptr(dst_y)), dst_y.stride(0),
                                         c_void_p(_ptr(dst_cb)) if dst_cb is not None else None,
                                         c_void_p(_ptr(dst_cr)) if dst_cr is not None else None,
                                         dst_cb.stride(0) if dst_cb is not None else 0))

    def run_raw(self, ptr_y: int, stride_y: int, ptr_cb: int, ptr_cr: int, stride_c: int):
        """mm_pred_run into raw device addresses (e.g. a rank's segment of a packed picture,
        parallel.StripeLayout.dst_pointers)."""
        self._check(self.lib.mm_pred_run(self.h, c_void_p(ptr_y), stride_y, c_void_p(ptr_cb), c_void_p(ptr_cr),
                                         stride_c))

    def predict_device_raw(self, cur_poc: int, d_pus, ptr_y: int, stride_y: int, ptr_cb: int, ptr_cr: int,
                           stride_c: int):
        """mm_pred_device into raw device addresses."""
        n = d_pus.numel() * d_pus.element_size() // PU_DTYPE.itemsize
        self._check(self.lib.mm_pred_device(self.h, cur_poc, c_void_p(_ptr(d_pus)), n, c_void_p(ptr_y), stride_y,
                                            c_void_p(ptr_cb), c_void_p(ptr_cr), stride_c))

    def set_call_timing(self, on: bool) -> None:
        """mm_set_call_timing: the events around every picture call (on by default)."""
        self._check(self.lib.mm_set_call_timing(self.h, 1 if on else 0))

    def last_timing_ms(self) -> float:
        ms = c_float()
        self._check(self.lib.mm_last_timing(self.h, byref(ms)))
        return float(ms.value)

    def set_dmvr(self, on: bool):
        """mm_set_dmvr: the picture's DMVR enable -- MM_PUF_DMVR PUs of mm_pred_device lists run
        the MM-DMVR search inside the launch sequence."""
        self._check(self.lib.mm_set_dmvr(self.h, int(on)))

    def set_stage_timing(self, on: bool):
        self._check(self.lib.mm_set_stage_timing(self.h, int(on)))

    def set_stripes(self, stripes: int):
        """Stripe pipelining of the device-planned path (mm_set_stripes)."""
        self._check(self.lib.mm_set_stripes(self.h, int(stripes)))

    def set_plan_ahead(self, on: bool):
        """Plan-ahead of the device-planned path (mm_set_plan_ahead): the device PU list of each
        predict_device call must be complete before the previous call is issued."""
        self._check(self.lib.mm_set_plan_ahead(self.h, int(on)))

    def last_stage_timing_ms(self):
        """(planning, k_setup, k_reproj, k_mc) device milliseconds of the last launch sequence."""
        ms = (c_float * 4)()
        self._check(self.lib.mm_last_stage_timing(self.h, ms))
        return tuple(float(v) for v in ms)

    # -- C4 transport (mm360.h: stripe-packed pictures) --------------------------------------
    def stripe_packed_dwords(self, world: int, ctu: int = 128) -> int:
        """mm_stripe_packed_dwords: dwords per packed segment of a `world`-rank stripe picture."""
        n = int(self.lib.mm_stripe_packed_dwords(self.h, world, ctu))
        if n < 0:
            raise MMError(MM_ERR_ARG, "mm_stripe_packed_dwords")
        return n

    def pack_samples(self, src, dst):
        """mm_pack_samples: the int16 CUDA tensor `src` (all of it) into the int32 CUDA tensor `dst`
        (ceil(numel / K) words, K = 32 // bit_depth), on the context stream."""
        self._check(self.lib.mm_pack_samples(self.h, c_void_p(_ptr(src)), src.numel(), c_void_p(_ptr(dst))))

    def upload_ref_packed(self, poc: int, packed, world: int, ctu: int = 128):
        """mm_upload_ref_packed: the gathered stripe-packed picture (int32 CUDA tensor, `world`
        segments) becomes reference `poc`, unpacked into the padded reference copy on the device."""
        self._check(self.lib.mm_upload_ref_packed(self.h, poc, c_void_p(_ptr(packed)), world, ctu))

    def upload_ref_stripes(self, poc: int, stripes, world: int, ctu: int = 128):
        """mm_upload_ref_stripes: the int16 stripe-major picture (CUDA tensor, StripeLayout.total
        samples) becomes reference `poc` (the unpacked C4 transport)."""
        self._check(self.lib.mm_upload_ref_stripes(self.h, poc, c_void_p(_ptr(stripes)), world, ctu))

    def set_kernel_timing(self, on: bool):
        """mm_set_kernel_timing: k_mc_dev launches bracketed by kernel-bound events while on."""
        self._check(self.lib.mm_set_kernel_timing(self.h, int(on)))

    def kernel_times_ms(self):
        """mm_kernel_times: k_mc_dev durations (ms) of the launches since the last read, oldest first."""
        ms = (c_float * 256)()
        n = c_int(0)
        self._check(self.lib.mm_kernel_times(self.h, ms, 256, ctypes.byref(n)))
        return [float(ms[i]) for i in range(n.value)]

    # -- encoder motion search (InterSearch::xMVReprojectionInterpolation + RdCost::xGetSAD) -
    def upload_org(self, poc: int, y):
        """Original luma picture of `poc` (numpy int16 host array or torch int16 CUDA tensor)."""
        sy = y.strides[0] // 2 if isinstance(y, np.ndarray) else y.stride(0)
        self._check(self.lib.mm_upload_org(self.h, poc, c_void_p(_ptr(y)), sy, int(_is_device(y))))

    def sad_window(self, cur_poc: int, blocks: np.ndarray, range_: int, step: int = 16, out=None):
        """SADs of every candidate of every block's window: a torch uint32-as-int32 CUDA tensor
        [n_blocks, (2*range+1)**2] (candidate c = (j+range)*(2*range+1) + (i+range))."""
        import torch
        blocks = np.ascontiguousarray(blocks, dtype=ME_BLOCK_DTYPE)
        C = (2 * range_ + 1) ** 2
        if out is None:
            out = torch.zeros((len(blocks), C), dtype=torch.int32, device=f"cuda:{self.device}")
        _check_sad_out(out, len(blocks) * C)
        self._check(self.lib.mm_sad_window(self.h, cur_poc, c_void_p(blocks.ctypes.data), len(blocks), range_, step,
                                           c_void_p(_ptr(out))))
        return out

    def sad_pattern(self, cur_poc: int, blocks: np.ndarray, offsets, out=None):
        """SADs of every block at mv + offsets[c] (1/16 luma, shared pattern of k candidates): a torch
        uint32-as-int32 CUDA tensor [n_blocks, k] (mm_sad_pattern)."""
        import torch
        blocks = np.ascontiguousarray(blocks, dtype=ME_BLOCK_DTYPE)
        off = np.ascontiguousarray(np.asarray(offsets, dtype=np.int32).reshape(-1, 2))
        if out is None:
            out = torch.zeros((len(blocks), len(off)), dtype=torch.int32, device=f"cuda:{self.device}")
        _check_sad_out(out, len(blocks) * len(off))
        self._check(self.lib.mm_sad_pattern(self.h, cur_poc, c_void_p(blocks.ctypes.data), len(blocks),
                                            c_void_p(off.ctypes.data), len(off), c_void_p(_ptr(out))))
        return out

    # -- InterpolationFilter -----------------------------------------------------------------
    def _filter(self, comp, vertical, src, x0, y0, w, h, frac, is_first, is_last):
        src = np.ascontiguousarray(src, dtype=np.int16)
        dst = np.zeros((h, w), dtype=np.int16)
        base = src.ctypes.data + (y0 * src.shape[1] + x0) * 2
        self._check(self.lib.mm_filter(self.h, comp, vertical, c_void_p(base), src.shape[1],
                                       c_void_p(dst.ctypes.data), w, w, h, frac, int(is_first),
                                       int(is_last)))
        return dst

    def filter_hor(self, comp, src, x0, y0, w, h, frac, is_last):
        """InterpolationFilter::filterHor (always isFirst, InterpolationFilter.cpp:658)."""
        return self._filter(comp, 0, src, x0, y0, w, h, frac, True, is_last)

    def filter_ver(self, comp, src, x0, y0, w, h, frac, is_first, is_last):
        """InterpolationFilter::filterVer."""
        return self._filter(comp, 1, src, x0, y0, w, h, frac, is_first, is_last)
