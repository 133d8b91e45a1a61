"""ctypes binding of the CPU twin (tests/native/host_twin.cpp) -- test utility."""
import ctypes
import os
import subprocess
from ctypes import c_int, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libhosttwin.so")


_VARIANT = [None]  # numerics-mode build in use (None = default; "round", "prod3", "tanc", "psqrt")


def use_variant(name):
    """Route the following calls to a numerics-mode build (make -C tests/native variants)."""
    _VARIANT[0] = name


def load():
    path = LIB if _VARIANT[0] is None else os.path.join(HERE, "_build", f"libhosttwin_{_VARIANT[0]}.so")
    if not os.path.exists(path):
        subprocess.check_call(["make", "-s", "-C", HERE] + ([] if _VARIANT[0] is None else ["variants"]))
    lib = ctypes.CDLL(path)
    lib.twin_reproject.argtypes = [c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p]
    lib.twin_pred.argtypes = [c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p,
                              c_void_p, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p, c_int]
    lib.twin_pred_dmvr.argtypes = [c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p,
                                   c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p, c_int,
                                   c_void_p]
    lib.twin_mvp.argtypes = [c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p]
    lib.twin_pred_mixed.argtypes = [c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p,
                                    c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p, c_int]
    lib.twin_pred_list1.argtypes = [c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_void_p,
                                    c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p,
                                    c_int]
    lib.twin_sad_window.argtypes = [c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_void_p,
                                    c_void_p, c_int, c_void_p, c_int, c_void_p]
    lib.twin_sad_pattern.argtypes = [c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_int,
                                     c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p]
    lib.twin_pred_multi.argtypes = [c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                                    c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p,
                                    c_int, c_int]
    lib.twin_mc_subblock.argtypes = [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                                     c_int, c_void_p, c_void_p, c_void_p]
    return lib


def _epi(epipoles):
    a = np.array([[c, r, q[0], q[1], q[2]] for (c, r, q) in epipoles] or [[0] * 5], dtype=np.int32)
    return len(epipoles), a


def reproject(params, blocks, epipoles=()):
    lib = load()
    blocks = np.ascontiguousarray(blocks)
    sb = np.where(blocks["comp"] != 0, 2, 4)
    total = int(((blocks["w"] // sb) * (blocks["h"] // sb)).sum())
    out = np.zeros((max(total, 1), 2), dtype=np.int32)
    n_epi, ea = _epi(epipoles)
    rc = lib.twin_reproject(ctypes.addressof(params), n_epi, c_void_p(ea.ctypes.data), c_void_p(blocks.ctypes.data),
                            len(blocks), c_void_p(out.ctypes.data))
    if rc:
        raise RuntimeError(f"twin reproject failed: {rc}")
    return out[:total]


def predict(params, cur_poc, pus, refs, W, H, epipoles=(), dmvr=False):
    """mm_pred_device twin; dmvr: mm_set_dmvr on (MM_PUF_DMVR PUs run the search)."""
    lib = load()
    pus = np.ascontiguousarray(pus)
    pocs = sorted(refs)
    arrs = [[np.ascontiguousarray(refs[p][k]) for p in pocs] for k in range(3)]
    ptrs = [(c_void_p * len(pocs))(*[a.ctypes.data for a in arrs[k]]) for k in range(3)]
    dy = np.zeros((H, W), dtype=np.int16)
    dcb = np.zeros((H // 2, W // 2), dtype=np.int16)
    dcr = np.zeros((H // 2, W // 2), dtype=np.int16)
    pa = np.array(pocs, dtype=np.int32)
    n_epi, ea = _epi(epipoles)
    fn = lib.twin_pred_mixed if dmvr else lib.twin_pred
    rc = fn(ctypes.addressof(params), n_epi, c_void_p(ea.ctypes.data), cur_poc, c_void_p(pus.ctypes.data),
            len(pus), len(pocs), c_void_p(pa.ctypes.data), ptrs[0], ptrs[1], ptrs[2], arrs[0][0].shape[1],
            arrs[1][0].shape[1], c_void_p(dy.ctypes.data), W, c_void_p(dcb.ctypes.data),
            c_void_p(dcr.ctypes.data), W // 2)
    if rc:
        raise RuntimeError(f"twin predict failed: {rc}")
    return dy, dcb, dcr


def predict_multi(params, pictures, refs, W, H, epipoles=(), dmvr=False):
    """mm_pred_device_multi twin: pictures = [(cur_poc, pus)], predicted as one list; planes per picture;
    dmvr: mm_set_dmvr (MM_PUF_DMVR PUs run the search)."""
    lib = load()
    allp = np.ascontiguousarray(np.concatenate([p for _, p in pictures]))
    base = np.cumsum([0] + [len(p) for _, p in pictures]).astype(np.int32)
    cur = np.array([c for c, _ in pictures], dtype=np.int32)
    pocs = sorted(refs)
    arrs = [[np.ascontiguousarray(refs[p][k]) for p in pocs] for k in range(3)]
    ptrs = [(c_void_p * len(pocs))(*[a.ctypes.data for a in arrs[k]]) for k in range(3)]
    outs = [(np.zeros((H, W), np.int16), np.zeros((H // 2, W // 2), np.int16), np.zeros((H // 2, W // 2), np.int16))
            for _ in pictures]
    dp = [(c_void_p * len(outs))(*[o[k].ctypes.data for o in outs]) for k in range(3)]
    pa = np.array(pocs, dtype=np.int32)
    n_epi, ea = _epi(epipoles)
    rc = lib.twin_pred_multi(ctypes.addressof(params), n_epi, c_void_p(ea.ctypes.data), len(pictures),
                             c_void_p(cur.ctypes.data), c_void_p(allp.ctypes.data), c_void_p(base.ctypes.data),
                             len(pocs), c_void_p(pa.ctypes.data), ptrs[0], ptrs[1], ptrs[2], arrs[0][0].shape[1],
                             arrs[1][0].shape[1], dp[0], W, dp[1], dp[2], W // 2, int(dmvr))
    if rc:
        raise RuntimeError(f"twin predict_multi failed: {rc}")
    return outs


def predict_list(params, cur_poc, pus, list_, hp, refs, W, H, epipoles=()):
    """mm_pred_list twin: list `list_` of every PU, 14-bit (hp) or clipped."""
    lib = load()
    pus = np.ascontiguousarray(pus)
    pocs = sorted(refs)
    arrs = [[np.ascontiguousarray(refs[p][k]) for p in pocs] for k in range(3)]
    ptrs = [(c_void_p * len(pocs))(*[a.ctypes.data for a in arrs[k]]) for k in range(3)]
    dy = np.zeros((H, W), dtype=np.int16)
    dcb = np.zeros((H // 2, W // 2), dtype=np.int16)
    dcr = np.zeros((H // 2, W // 2), dtype=np.int16)
    pa = np.array(pocs, dtype=np.int32)
    n_epi, ea = _epi(epipoles)
    rc = lib.twin_pred_list1(ctypes.addressof(params), n_epi, c_void_p(ea.ctypes.data), cur_poc,
                             c_void_p(pus.ctypes.data), len(pus), int(list_), int(hp), len(pocs),
                             c_void_p(pa.ctypes.data), ptrs[0], ptrs[1], ptrs[2], arrs[0][0].shape[1],
                             arrs[1][0].shape[1], c_void_p(dy.ctypes.data), W, c_void_p(dcb.ctypes.data),
                             c_void_p(dcr.ctypes.data), W // 2)
    if rc:
        raise RuntimeError(f"twin predict_list failed: {rc}")
    return dy, dcb, dcr


def sad_window(params, cur_poc, blocks, range_, step, refs, org, epipoles=()):
    """refs: poc -> luma plane.  uint32 SADs [n_blocks, (2*range+1)**2]."""
    lib = load()
    blocks = np.ascontiguousarray(blocks)
    pocs = sorted(refs)
    ys = [np.ascontiguousarray(refs[p]) for p in pocs]
    ptrs = (c_void_p * len(pocs))(*[a.ctypes.data for a in ys])
    org = np.ascontiguousarray(org, dtype=np.int16)
    C = (2 * range_ + 1) ** 2
    out = np.zeros((len(blocks), C), dtype=np.uint32)
    pa = np.array(pocs, dtype=np.int32)
    n_epi, ea = _epi(epipoles)
    rc = lib.twin_sad_window(ctypes.addressof(params), n_epi, c_void_p(ea.ctypes.data), cur_poc,
                             c_void_p(blocks.ctypes.data), len(blocks), range_, step, len(pocs),
                             c_void_p(pa.ctypes.data), ptrs, ys[0].shape[1], c_void_p(org.ctypes.data), org.shape[1],
                             c_void_p(out.ctypes.data))
    if rc:
        raise RuntimeError(f"twin sad_window failed: {rc}")
    return out


def sad_pattern(params, cur_poc, blocks, offsets, refs, org, epipoles=()):
    """mm_sad_pattern's host twin: uint32 SADs [n_blocks, k] at mv + offsets[c]."""
    lib = load()
    blocks = np.ascontiguousarray(blocks)
    off = np.ascontiguousarray(np.asarray(offsets, dtype=np.int32).reshape(-1, 2))
    pocs = sorted(refs)
    ys = [np.ascontiguousarray(refs[p]) for p in pocs]
    ptrs = (c_void_p * len(pocs))(*[a.ctypes.data for a in ys])
    org = np.ascontiguousarray(org, dtype=np.int16)
    out = np.zeros((len(blocks), len(off)), dtype=np.uint32)
    pa = np.array(pocs, dtype=np.int32)
    n_epi, ea = _epi(epipoles)
    rc = lib.twin_sad_pattern(ctypes.addressof(params), n_epi, c_void_p(ea.ctypes.data), cur_poc,
                              c_void_p(blocks.ctypes.data), len(blocks), c_void_p(off.ctypes.data), len(off), len(pocs),
                              c_void_p(pa.ctypes.data), ptrs, ys[0].shape[1], c_void_p(org.ctypes.data), org.shape[1],
                              c_void_p(out.ctypes.data))
    if rc:
        raise RuntimeError(f"twin sad_pattern failed: {rc}")
    return out


def predict_dmvr(params, cur_poc, pus, refs, W, H, epipoles=()):
    lib = load()
    pus = np.ascontiguousarray(pus)
    pocs = sorted(refs)
    arrs = [[np.ascontiguousarray(refs[p][k]) for p in pocs] for k in range(3)]
    ptrs = [(c_void_p * len(pocs))(*[a.ctypes.data for a in arrs[k]]) for k in range(3)]
    dy = np.zeros((H, W), dtype=np.int16)
    dcb = np.zeros((H // 2, W // 2), dtype=np.int16)
    dcr = np.zeros((H // 2, W // 2), dtype=np.int16)
    nsub = int(sum(((int(u["w"]) + 15) // 16) * ((int(u["h"]) + 15) // 16) for u in pus))
    mvd = np.zeros((max(nsub, 1), 2), dtype=np.int32)
    pa = np.array(pocs, dtype=np.int32)
    n_epi, ea = _epi(epipoles)
    rc = lib.twin_pred_dmvr(ctypes.addressof(params), n_epi, c_void_p(ea.ctypes.data), cur_poc,
                            c_void_p(pus.ctypes.data), len(pus), len(pocs), c_void_p(pa.ctypes.data), ptrs[0], ptrs[1],
                            ptrs[2], arrs[0][0].shape[1], arrs[1][0].shape[1], c_void_p(dy.ctypes.data), W,
                            c_void_p(dcb.ctypes.data), c_void_p(dcr.ctypes.data), W // 2, c_void_p(mvd.ctypes.data))
    if rc:
        raise RuntimeError(f"twin predict_dmvr failed: {rc}")
    return (dy, dcb, dcr), mvd[:nsub]


def mvp(params, queries, epipoles=()):
    lib = load()
    q = np.ascontiguousarray(queries)
    out = np.zeros((max(len(q), 1), 2), dtype=np.int32)
    n_epi, ea = _epi(epipoles)
    rc = lib.twin_mvp(ctypes.addressof(params), n_epi, c_void_p(ea.ctypes.data), c_void_p(q.ctypes.data), len(q),
                      c_void_p(out.ctypes.data))
    if rc:
        raise RuntimeError(f"twin mvp failed: {rc}")
    return out[:len(q)]


def mc_subblock(params, use, bcw, hp, pos, planes):
    """One sub-block through the interpolation body at explicit positions (no reprojection).
    pos: int32 [2, 4] = per list (luma x, y in 1/16, chroma x, y in 1/32); planes: (y, cb, cr) of
    the one reference both lists read.  Returns (4x4 luma, 2x2 cb, 2x2 cr)."""
    lib = load()
    pos = np.ascontiguousarray(pos, dtype=np.int32)
    y, cb, cr = (np.ascontiguousarray(a, dtype=np.int16) for a in planes)
    oy = np.zeros((4, 4), dtype=np.int16)
    ocb = np.zeros((2, 2), dtype=np.int16)
    ocr = np.zeros((2, 2), dtype=np.int16)
    lib.twin_mc_subblock(ctypes.addressof(params), int(use), int(bcw), int(hp), c_void_p(pos.ctypes.data),
                         c_void_p(y.ctypes.data), c_void_p(cb.ctypes.data), c_void_p(cr.ctypes.data), y.shape[1],
                         cb.shape[1], c_void_p(oy.ctypes.data), c_void_p(ocb.ctypes.data), c_void_p(ocr.ctypes.data))
    return oy, ocb, ocr
