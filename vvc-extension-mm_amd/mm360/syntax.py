"""Bitstream side of the MM extension over the C-ABI (include/mm360.h, csrc/mm_syntax.h).

Mirrors the reference's parsing / writing entry points for the MM syntax:

    VLCWriter / VLCReader SPS fragment (VLCWriter.cpp:1110-1142, VLCReader.cpp:1920-1980)
                                            -> write_sps_mm / read_sps_mm
    picture header epipole delta (VLCWriter.cpp:2096-2109, VLCReader.cpp:3354-3372)
                                            -> write_ph_epipole / read_ph_epipole
    CABACReader::motion_model candidate order (CABACReader.cpp:2179-2296)
                                            -> motion_model_candidates
    CABACWriter::motion_model / CABACReader::motion_model (CABACWriter.cpp:1984-2000,
    CABACReader.cpp:2300-2322)               -> encode_motion_models / decode_motion_models

Host code only (no context, no GPU); errors raise MMError as the rest of the package does.
"""
from __future__ import annotations

import ctypes
from ctypes import byref, c_int32, c_int64, c_uint32, c_void_p
from typing import Optional, Sequence, Tuple

import numpy as np

from . import MM_ERR_ARG, MM_OK, MMError, load_library

MAX_CALIB_COEFFS = 16  # MM_MAX_CALIB_COEFFS
NUM_MODEL_IDS = 11     # MM_NUM_MODEL_IDS
EQUISOLID, CALIBRATED, EQUIRECTANGULAR = 0, 1, 2  # ProjectionID (Projection.h:12-17)
B_SLICE, P_SLICE, I_SLICE = 0, 1, 2                # SliceType (TypeDef.h:367-373)
PRED_NONE, PRED_CENTRE, PRED_VOTED, PRED_SORTED = 0, 1, 2, 3  # m_mmPredType
APP_CODING_DEPTH = 9  # m_mmCodingDepth set by DecApp.cpp:894 / EncApp.cpp:759


class SpsMM(ctypes.Structure):
    """mm_sps_mm: MMConfig's coded fields (MMConfig.h:15-30)."""
    _fields_ = [("mpa", c_int32), ("t3d", c_int32), ("tan", c_int32), ("rot", c_int32), ("ged", c_int32),
                ("geda", c_int32), ("ged_flavor", c_int32), ("mmmvp", c_int32), ("mm_offset_4x4", c_int32),
                ("projection_fct", c_int32), ("focal_length_px", c_uint32), ("optical_center_x_px", c_uint32),
                ("optical_center_y_px", c_uint32), ("num_calibrated_coeffs", c_uint32),
                ("calibrated_coeffs", c_int32 * MAX_CALIB_COEFFS), ("global_epipole", c_int32 * 3)]

    def as_dict(self) -> dict:
        d = {f: getattr(self, f) for f, _ in self._fields_ if f not in ("calibrated_coeffs", "global_epipole")}
        d["calibrated_coeffs"] = list(self.calibrated_coeffs)[: min(int(self.num_calibrated_coeffs), MAX_CALIB_COEFFS)]
        d["global_epipole"] = list(self.global_epipole)
        return d


def sps_mm(**kw) -> SpsMM:
    """An SpsMM from keyword fields (calibrated_coeffs / global_epipole as sequences)."""
    s = SpsMM()
    for k, v in kw.items():
        if k == "calibrated_coeffs":
            for i, c in enumerate(v):
                s.calibrated_coeffs[i] = int(c)
            if "num_calibrated_coeffs" not in kw:
                s.num_calibrated_coeffs = len(v)
        elif k == "global_epipole":
            for i in range(3):
                s.global_epipole[i] = int(v[i])
        else:
            setattr(s, k, int(v))
    return s


def _buf(a: np.ndarray) -> c_void_p:
    return c_void_p(a.ctypes.data)


def write_sps_mm(sps: SpsMM, buf: Optional[np.ndarray] = None, bit_pos: int = 0) -> Tuple[np.ndarray, int]:
    """Write the SPS MM fragment at bit_pos; returns (buffer, new bit position)."""
    lib = load_library()
    if buf is None:
        buf = np.zeros(256, np.uint8)
    pos = c_int64(bit_pos)
    rc = lib.mm_sps_mm_write(byref(sps), _buf(buf), buf.nbytes, byref(pos))
    if rc != MM_OK:
        raise MMError(rc, "mm_sps_mm_write")
    return buf, pos.value


def read_sps_mm(buf: np.ndarray, nbits: Optional[int] = None, bit_pos: int = 0) -> Tuple[SpsMM, int]:
    lib = load_library()
    buf = np.ascontiguousarray(buf, np.uint8)
    pos, s = c_int64(bit_pos), SpsMM()
    rc = lib.mm_sps_mm_read(_buf(buf), buf.nbytes * 8 if nbits is None else nbits, byref(pos), byref(s))
    if rc != MM_OK:
        raise MMError(rc, "mm_sps_mm_read")
    return s, pos.value


def write_ph_epipole(sps: SpsMM, delta: Sequence[int], buf: Optional[np.ndarray] = None,
                     bit_pos: int = 0) -> Tuple[np.ndarray, int]:
    lib = load_library()
    if buf is None:
        buf = np.zeros(64, np.uint8)
    d, pos = (c_int32 * 3)(*[int(v) for v in delta]), c_int64(bit_pos)
    rc = lib.mm_ph_epipole_write(byref(sps), d, _buf(buf), buf.nbytes, byref(pos))
    if rc != MM_OK:
        raise MMError(rc, "mm_ph_epipole_write")
    return buf, pos.value


def read_ph_epipole(sps: SpsMM, buf: np.ndarray, nbits: Optional[int] = None, bit_pos: int = 0):
    lib = load_library()
    buf = np.ascontiguousarray(buf, np.uint8)
    d, pos = (c_int32 * 3)(), c_int64(bit_pos)
    rc = lib.mm_ph_epipole_read(byref(sps), _buf(buf), buf.nbytes * 8 if nbits is None else nbits, byref(pos), d)
    if rc != MM_OK:
        raise MMError(rc, "mm_ph_epipole_read")
    return [d[0], d[1], d[2]], pos.value


def motion_model_candidates(sps: SpsMM, pred_type: int = PRED_NONE, col_models: Optional[np.ndarray] = None,
                            pic_w: int = 0, pic_h: int = 0, col_list: int = 0, x: int = 0, y: int = 0, w: int = 0,
                            h: int = 0) -> list:
    """The PU's motion_model() candidates in coding order.  col_models: int8 [grid_h, grid_w, 2]."""
    lib = load_library()
    cand, n = (c_int32 * NUM_MODEL_IDS)(), c_int32(0)
    if col_models is not None:
        col_models = np.ascontiguousarray(col_models, np.int8)
        gh, gw = col_models.shape[:2]
        ptr = _buf(col_models)
    else:
        gh = gw = 0
        ptr = None
    rc = lib.mm_motion_model_candidates(byref(sps), pred_type, ptr, gw, gh, pic_w, pic_h, col_list, x, y, w, h,
                                        cand, byref(n))
    if rc != MM_OK:
        raise MMError(rc, "mm_motion_model_candidates")
    return list(cand)[: n.value]


def _cand_rows(cand, n_pu: int) -> np.ndarray:
    rows = np.full((n_pu, NUM_MODEL_IDS), -1, np.int32)
    for i, c in enumerate(cand):
        rows[i, : len(c)] = c
    return rows


def encode_motion_models(sps: SpsMM, models: Sequence[int], cand, slice_qp: int = 32, init_type: int = B_SLICE,
                         coding_depth: int = APP_CODING_DEPTH, affine: Optional[Sequence[int]] = None) -> bytes:
    """CABAC stream of the PUs' motion_model() (+ end_of_slice, flush, trailing bits).
    cand: one candidate list per PU (motion_model_candidates)."""
    lib = load_library()
    n = len(models)
    rows = _cand_rows(cand, n)
    m = np.ascontiguousarray(models, np.int32)
    aff = np.ascontiguousarray(affine, np.uint8) if affine is not None else None
    cap = 64 + 4 * n
    out, nbytes = np.zeros(cap, np.uint8), c_int64(0)
    rc = lib.mm_motion_model_encode(byref(sps), slice_qp, init_type, coding_depth, n, _buf(rows),
                                    _buf(aff) if aff is not None else None, _buf(m), _buf(out), cap, byref(nbytes))
    if rc != MM_OK:
        raise MMError(rc, "mm_motion_model_encode")
    return out[: nbytes.value].tobytes()


def decode_motion_models(sps: SpsMM, stream: bytes, cand, slice_qp: int = 32, init_type: int = B_SLICE,
                         coding_depth: int = APP_CODING_DEPTH, affine: Optional[Sequence[int]] = None) -> list:
    lib = load_library()
    n = len(cand)
    rows = _cand_rows(cand, n)
    data = np.frombuffer(bytes(stream) or b"\0", np.uint8).copy()
    aff = np.ascontiguousarray(affine, np.uint8) if affine is not None else None
    out = np.zeros(max(n, 1), np.int32)
    rc = lib.mm_motion_model_decode(byref(sps), slice_qp, init_type, coding_depth, n, _buf(rows),
                                    _buf(aff) if aff is not None else None, _buf(data), len(stream), _buf(out))
    if rc != MM_OK:
        raise MMError(rc, "mm_motion_model_decode")
    return [int(v) for v in out[:n]]


__all__ = ["SpsMM", "sps_mm", "write_sps_mm", "read_sps_mm", "write_ph_epipole", "read_ph_epipole",
           "motion_model_candidates", "encode_motion_models", "decode_motion_models", "MM_ERR_ARG"]
