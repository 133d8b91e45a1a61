"""ctypes binding of the CPU oracle (oracle/mm_oracle.c) -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module; the
product (vvc-extension-mm_amd/) never does.  Parity status: UNPINNED (see mm_oracle.c header).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, c_int, c_int32, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libmmoracle.so")


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def load(variant=None):
    """The oracle library; variant = a numerics-mode build ("round", "prod3", "tanc", "psqrt")."""
    path = LIB if variant is None else os.path.join(HERE, "_build", f"libmmoracle_{variant}.so")
    if not os.path.exists(path):
        subprocess.check_call(["make", "-s", "-C", HERE] + ([] if variant is None else ["variants"]))
    lib = ctypes.CDLL(path)
    lib.orc_create.restype = c_void_p
    lib.orc_create.argtypes = [c_void_p]
    lib.orc_destroy.argtypes = [c_void_p]
    lib.orc_set_epipole.argtypes = [c_void_p, c_int, c_int, POINTER(c_int32)]
    lib.orc_reproject.argtypes = [c_void_p, c_void_p, c_int, c_void_p]
    lib.orc_pred.argtypes = [c_void_p, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                             ctypes.c_ssize_t, ctypes.c_ssize_t, c_void_p, ctypes.c_ssize_t, c_void_p, c_void_p,
                             ctypes.c_ssize_t]
    lib.orc_pred_list.argtypes = [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                                  c_void_p, c_void_p, ctypes.c_ssize_t, ctypes.c_ssize_t, c_void_p,
                                  ctypes.c_ssize_t, c_void_p, c_void_p, ctypes.c_ssize_t]
    lib.orc_effective.argtypes = [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, POINTER(c_int), c_void_p,
                                  c_int, POINTER(c_int)]
    lib.orc_epi_create.restype = c_void_p
    lib.orc_epi_destroy.argtypes = [c_void_p]
    lib.orc_epi_add.argtypes = [c_void_p, c_int, c_int, POINTER(c_int32), c_int]
    lib.orc_epi_find.argtypes = [c_void_p, c_int, c_int, POINTER(c_int32)]
    lib.orc_epi_has.argtypes = [c_void_p, c_int, c_int]
    lib.orc_epi_make_available.argtypes = [c_void_p, c_int]
    lib.orc_epi_predictor.argtypes = [c_void_p, c_int, POINTER(c_int32)]
    lib.orc_epi_count.argtypes = [c_void_p]
    lib.orc_refs_create.restype = c_void_p
    lib.orc_refs_create.argtypes = [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_ssize_t,
                                    ctypes.c_ssize_t]
    lib.orc_refs_destroy.argtypes = [c_void_p]
    lib.orc_pred_padded.argtypes = [c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p, ctypes.c_ssize_t, c_void_p,
                                    c_void_p, ctypes.c_ssize_t, c_int]
    lib.orc_filter.argtypes = [c_int, c_int, c_int, c_void_p, ctypes.c_ssize_t, c_void_p, ctypes.c_ssize_t, c_int,
                               c_int, c_int, c_int, c_int]
    lib.orc_pred_dmvr.argtypes = [c_void_p, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                  ctypes.c_ssize_t, ctypes.c_ssize_t, c_void_p, ctypes.c_ssize_t, c_void_p, c_void_p,
                                  ctypes.c_ssize_t, c_void_p]
    lib.orc_pred_dmvr_trace.argtypes = lib.orc_pred_dmvr.argtypes + [c_void_p]
    lib.orc_mvp.argtypes = [c_void_p, c_void_p, c_int, c_void_p]
    lib.orc_sad_window.argtypes = [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                                   ctypes.c_ssize_t, c_void_p, ctypes.c_ssize_t, c_void_p]
    return lib


def _ptr_array(arrs):
    return (c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])


class _PaddedRefs:
    def __init__(self, lib, h):
        self.lib, self.h = lib, c_void_p(h)

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.orc_refs_destroy(self.h)
            self.h = None


class Oracle:
    """CPU restatement of MVReprojection / xPredInterBlkMM for one sequence."""

    def __init__(self, params, epipoles=(), variant=None):
        self.lib = load(variant)
        self.params = params
        self.h = self.lib.orc_create(ctypes.byref(params))
        for (cur, ref, q) in epipoles:
            self.set_epipole(cur, ref, q)

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.orc_destroy(self.h)
            self.h = None

    def set_epipole(self, cur, ref, q):
        self.lib.orc_set_epipole(self.h, cur, ref, (c_int32 * 3)(*q))

    def reproject(self, blocks):
        blocks = np.ascontiguousarray(blocks)
        sb = np.where(blocks["comp"] != 0, 2, 4)
        total = int(((blocks["w"] // sb) * (blocks["h"] // sb)).sum())
        out = np.zeros((max(total, 1), 2), dtype=np.int32)
        rc = self.lib.orc_reproject(self.h, c_void_p(blocks.ctypes.data), len(blocks), c_void_p(out.ctypes.data))
        if rc:
            raise RuntimeError(f"oracle reproject failed: {rc}")
        return out[:total]

    def predict(self, cur_poc, pus, refs, W, H):
        """refs: dict poc -> (Y, Cb, Cr) int16 arrays.  Returns (Y, Cb, Cr) predicted planes
        (zero where no PU)."""
        pus = np.ascontiguousarray(pus)
        pocs = sorted(refs)
        ys = [np.ascontiguousarray(refs[p][0]) for p in pocs]
        cbs = [np.ascontiguousarray(refs[p][1]) for p in pocs]
        crs = [np.ascontiguousarray(refs[p][2]) for p in pocs]
        dy = np.zeros((H, W), dtype=np.int16)
        dcb = np.zeros((H // 2, W // 2), dtype=np.int16)
        dcr = np.zeros((H // 2, W // 2), dtype=np.int16)
        pa = np.array(pocs, dtype=np.int32)
        rc = self.lib.orc_pred(self.h, cur_poc, c_void_p(pus.ctypes.data), len(pus), len(pocs),
                               c_void_p(pa.ctypes.data), _ptr_array(ys), _ptr_array(cbs), _ptr_array(crs),
                               ys[0].shape[1], cbs[0].shape[1], c_void_p(dy.ctypes.data), W,
                               c_void_p(dcb.ctypes.data), c_void_p(dcr.ctypes.data), W // 2)
        if rc:
            raise RuntimeError(f"oracle predict failed: {rc}")
        return dy, dcb, dcr

    def padded_refs(self, refs):
        """Pad the reference pictures once (Picture::extendPicBorder layout) for predict_padded."""
        pocs = sorted(refs)
        ys = [np.ascontiguousarray(refs[p][0]) for p in pocs]
        cbs = [np.ascontiguousarray(refs[p][1]) for p in pocs]
        crs = [np.ascontiguousarray(refs[p][2]) for p in pocs]
        pa = np.array(pocs, dtype=np.int32)
        h = self.lib.orc_refs_create(self.h, len(pocs), c_void_p(pa.ctypes.data), _ptr_array(ys), _ptr_array(cbs),
                                     _ptr_array(crs), ys[0].shape[1], cbs[0].shape[1])
        return _PaddedRefs(self.lib, h)

    def predict_padded(self, prefs, cur_poc, pus, W, H, threads=1):
        """predict() on pre-padded references, PU-parallel on `threads` host threads."""
        pus = np.ascontiguousarray(pus)
        dy = np.zeros((H, W), dtype=np.int16)
        dcb = np.zeros((H // 2, W // 2), dtype=np.int16)
        dcr = np.zeros((H // 2, W // 2), dtype=np.int16)
        rc = self.lib.orc_pred_padded(self.h, prefs.h, cur_poc, c_void_p(pus.ctypes.data), len(pus),
                                      c_void_p(dy.ctypes.data), W, c_void_p(dcb.ctypes.data),
                                      c_void_p(dcr.ctypes.data), W // 2, int(threads))
        if rc:
            raise RuntimeError(f"oracle predict_padded failed: {rc}")
        return dy, dcb, dcr

    def predict_list(self, cur_poc, pus, list_, hp, refs, W, H):
        """xPredInterBlkMM of reference list `list_` of every PU: 14-bit (hp) or clipped planes."""
        pus = np.ascontiguousarray(pus)
        pocs = sorted(refs)
        ys = [np.ascontiguousarray(refs[p][0]) for p in pocs]
        cbs = [np.ascontiguousarray(refs[p][1]) for p in pocs]
        crs = [np.ascontiguousarray(refs[p][2]) for p in pocs]
        dy = np.zeros((H, W), dtype=np.int16)
        dcb = np.zeros((H // 2, W // 2), dtype=np.int16)
        dcr = np.zeros((H // 2, W // 2), dtype=np.int16)
        pa = np.array(pocs, dtype=np.int32)
        rc = self.lib.orc_pred_list(self.h, cur_poc, c_void_p(pus.ctypes.data), len(pus), int(list_), int(hp),
                                    len(pocs), c_void_p(pa.ctypes.data), _ptr_array(ys), _ptr_array(cbs),
                                    _ptr_array(crs), ys[0].shape[1], cbs[0].shape[1], c_void_p(dy.ctypes.data), W,
                                    c_void_p(dcb.ctypes.data), c_void_p(dcr.ctypes.data), W // 2)
        if rc:
            raise RuntimeError(f"oracle predict_list failed: {rc}")
        return dy, dcb, dcr

    def predict_dmvr(self, cur_poc, pus, refs, W, H, out=None, trace=False):
        """MM-DMVR PUs (xProcessDMVRProjected): predicted planes and the per-sub-PU L0 deltas.
        out: (Y, Cb, Cr) planes to predict into (only the PUs' samples are written).
        trace: also return the per-sub-PU branch words (mm_oracle.c DMVR_TR_*, dmvr_branches)."""
        pus = np.ascontiguousarray(pus)
        pocs = sorted(refs)
        ys = [np.ascontiguousarray(refs[p][0]) for p in pocs]
        cbs = [np.ascontiguousarray(refs[p][1]) for p in pocs]
        crs = [np.ascontiguousarray(refs[p][2]) for p in pocs]
        if out is None:
            dy = np.zeros((H, W), dtype=np.int16)
            dcb = np.zeros((H // 2, W // 2), dtype=np.int16)
            dcr = np.zeros((H // 2, W // 2), dtype=np.int16)
        else:
            dy, dcb, dcr = out
        nsub = int(sum(((int(u["w"]) + 15) // 16) * ((int(u["h"]) + 15) // 16) for u in pus))
        mvd = np.zeros((max(nsub, 1), 2), dtype=np.int32)
        pa = np.array(pocs, dtype=np.int32)
        tr = np.zeros(max(nsub, 1), dtype=np.int32)
        rc = self.lib.orc_pred_dmvr_trace(self.h, cur_poc, c_void_p(pus.ctypes.data), len(pus), len(pocs),
                                          c_void_p(pa.ctypes.data), _ptr_array(ys), _ptr_array(cbs), _ptr_array(crs),
                                          ys[0].shape[1], cbs[0].shape[1], c_void_p(dy.ctypes.data), W,
                                          c_void_p(dcb.ctypes.data), c_void_p(dcr.ctypes.data), W // 2,
                                          c_void_p(mvd.ctypes.data), c_void_p(tr.ctypes.data))
        if rc:
            raise RuntimeError(f"oracle predict_dmvr failed: {rc}")
        if trace:
            return (dy, dcb, dcr), mvd[:nsub], tr[:nsub]
        return (dy, dcb, dcr), mvd[:nsub]

    def predict_mixed(self, cur_poc, pus, refs, W, H, prefs=None, threads=1):
        """A picture list in which PUs flagged MM_PUF_DMVR (flags bit 0) run MM-DMVR: the other PUs
        through predict (predict_padded when prefs is given), then the flagged ones through
        predict_dmvr into the same planes (PUs do not overlap)."""
        dm = (np.asarray(pus["flags"]) & 1) != 0
        rest = np.ascontiguousarray(pus[~dm])
        if prefs is not None:
            planes = self.predict_padded(prefs, cur_poc, rest, W, H, threads)
        else:
            planes = self.predict(cur_poc, rest, refs, W, H)
        if dm.any():
            d = np.ascontiguousarray(pus[dm]).copy()
            d["flags"] = 0
            self.predict_dmvr(cur_poc, d, refs, W, H, out=planes)
        return planes

    def mvp(self, queries):
        """MM-MVP conversions: int32 [n, 2]."""
        q = np.ascontiguousarray(queries)
        out = np.zeros((max(len(q), 1), 2), dtype=np.int32)
        rc = self.lib.orc_mvp(self.h, c_void_p(q.ctypes.data), len(q), c_void_p(out.ctypes.data))
        if rc:
            raise RuntimeError(f"oracle mvp failed: {rc}")
        return out[:len(q)]

    def sad_window(self, cur_poc, blocks, range_, step, refs, org):
        """Encoder candidate windows: uint32 SADs [n_blocks, (2*range+1)**2].  refs: poc -> luma."""
        blocks = np.ascontiguousarray(blocks)
        pocs = sorted(refs)
        ys = [np.ascontiguousarray(refs[p]) for p in pocs]
        org = np.ascontiguousarray(org, dtype=np.int16)
        C = (2 * range_ + 1) ** 2
        out = np.zeros((len(blocks), C), dtype=np.uint32)
        pa = np.array(pocs, dtype=np.int32)
        rc = self.lib.orc_sad_window(self.h, cur_poc, c_void_p(blocks.ctypes.data), len(blocks), range_, step,
                                     len(pocs), c_void_p(pa.ctypes.data), _ptr_array(ys), ys[0].shape[1],
                                     c_void_p(org.ctypes.data), org.shape[1], c_void_p(out.ctypes.data))
        if rc:
            raise RuntimeError(f"oracle sad_window failed: {rc}")
        return out

    def filter(self, comp, vertical, bd, src, x0, y0, w, h, frac, first, last):
        src = np.ascontiguousarray(src, dtype=np.int16)
        dst = np.zeros((h, w), dtype=np.int16)
        base = src.ctypes.data + (y0 * src.shape[1] + x0) * 2
        rc = self.lib.orc_filter(comp, vertical, bd, c_void_p(base), src.shape[1], c_void_p(dst.ctypes.data), w, w,
                                 h, frac, int(first), int(last))
        if rc:
            raise RuntimeError(f"oracle filter failed: {rc}")
        return dst


def dmvr_branches(trace):
    """Counts of the MM-DMVR decision branches in an orc_pred_dmvr_trace word array
    (InterPrediction.cpp:2516-2531 early exit, :2567-2580 border best, xSubPelErrorSrfc :1996-2048)."""
    t = np.asarray(trace, dtype=np.int64)
    searched = (t & 1) == 0
    surf = searched & ((t & 64) == 0)
    out = {"sub_pus": int(len(t)), "early_exit": int((~searched).sum()), "searched": int(searched.sum()),
           "border_best": int((searched & ((t & 64) != 0)).sum()),
           "centre_best": int((searched & (((t >> 1) & 31) == 12)).sum())}
    for axis, sh in (("h", 8), ("v", 10)):
        case = (t >> sh) & 3
        for k, name in enumerate(("den0", "div", "tie_minus", "tie_plus")):
            out[f"{axis}_{name}"] = int((surf & (case == k)).sum())
    return out


def effective_blocks(tools, pus, sub_motion, pu_dtype, cap=1 << 16):
    """Oracle restatement of motionCompensation's effective blocks: (mc, dmvr) PU arrays."""
    lib = load()
    pus = np.ascontiguousarray(pus)
    sub = np.ascontiguousarray(sub_motion)
    mc = np.zeros(cap, dtype=pu_dtype)
    dm = np.zeros(cap, dtype=pu_dtype)
    n_mc, n_dm = c_int(0), c_int(0)
    rc = lib.orc_effective(ctypes.addressof(tools), c_void_p(pus.ctypes.data), len(pus),
                           c_void_p(sub.ctypes.data) if len(sub) else None, c_void_p(mc.ctypes.data), cap,
                           ctypes.byref(n_mc), c_void_p(dm.ctypes.data), cap, ctypes.byref(n_dm))
    if rc:
        raise RuntimeError(f"oracle effective blocks failed: {rc}")
    return mc[:n_mc.value], dm[:n_dm.value]


class OracleEpipoleList:
    """Oracle restatement of EpipoleList (SRC/EpipoleList.cpp)."""

    def __init__(self):
        self.lib = load()
        self.h = c_void_p(self.lib.orc_epi_create())

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.orc_epi_destroy(self.h)
            self.h = None

    def add(self, cur, ref, q, make_available=False):
        self.lib.orc_epi_add(self.h, cur, ref, (c_int32 * 3)(*q), int(make_available))

    def make_available(self, cur):
        self.lib.orc_epi_make_available(self.h, cur)

    def has(self, cur, ref):
        return bool(self.lib.orc_epi_has(self.h, cur, ref))

    def find(self, cur, ref):
        q = (c_int32 * 3)()
        rc = self.lib.orc_epi_find(self.h, cur, ref, q)
        return None if rc else tuple(q)

    def derive_predictor(self, cur):
        q = (c_int32 * 3)()
        rc = self.lib.orc_epi_predictor(self.h, cur, q)
        return rc, (tuple(q) if rc == 0 else None)

    def count(self):
        return int(self.lib.orc_epi_count(self.h))
