"""Multi-GPU partitioning of the MM motion-compensation path.

Given the reference pictures, PUs are independent: MC reads only the references plus the PU's
own descriptor.  A picture therefore shards by contiguous CTU-row stripes (PU -> rank owning
the CTU row of its top-left sample); the references stay replicated on every GPU because MM
motion can fetch anywhere in the picture (it wraps across the ERP seam, Projection.cpp:235, and is
bounded only by the +-maxCU zeroing rule, InterPrediction.cpp:780).  After MC, ONE all-gather of
the predicted stripes (RCCL over xGMI with the "nccl" backend; gloo on CPU) gives every rank the
whole picture again, as a decoder needs for the next reference.

The all-gather moves the picture in a stripe-major packed layout (StripeLayout): rank r's segment
holds its luma rows, then its Cb rows, then its Cr rows, so one in-place all_gather_into_tensor of
equal segments carries Y + Cb + Cr together and no staging copy exists -- each rank's kernels
write their stripe straight into their own segment (the destination pointers are offset so that
picture row y0 of the stripe lands at the segment start).
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np


def stripe_rows(height: int, world: int, rank: int, ctu: int = 128) -> Tuple[int, int]:
    """Luma row range [y0, y1) of `rank`'s CTU-row stripe."""
    n_ctu = (height + ctu - 1) // ctu
    a = (n_ctu * rank) // world
    b = (n_ctu * (rank + 1)) // world
    return min(a * ctu, height), min(b * ctu, height)


def shard_pus(pus: np.ndarray, height: int, world: int, rank: int, ctu: int = 128) -> np.ndarray:
    """PUs whose top-left CTU row falls into `rank`'s stripe (PUs never cross CTU rows)."""
    y0, y1 = stripe_rows(height, world, rank, ctu)
    sel = (pus["y"] >= y0) & (pus["y"] < y1)
    return pus[sel]


def max_stripe_rows(height: int, world: int, ctu: int = 128) -> int:
    return max(b - a for a, b in (stripe_rows(height, world, r, ctu) for r in range(world)))


class StripeLayout:
    """Stripe-major packed 4:2:0 picture (int16 samples): segment r = Y rows of stripe r
    (rows x W), then its Cb rows ((rows / 2) x W/2), then its Cr rows; every segment is sized for
    the largest stripe so that the all-gather exchanges equal chunks."""

    def __init__(self, width: int, height: int, world: int, ctu: int = 128):
        self.W, self.H, self.world, self.ctu = width, height, world, ctu
        self.rows = max_stripe_rows(height, world, ctu)
        self.luma = self.rows * width
        self.chroma = (self.rows // 2) * (width // 2)
        self.seg = self.luma + 2 * self.chroma  # int16 elements per segment
        self.total = self.seg * world

    def dst_pointers(self, base_ptr: int, rank: int):
        """(ptr_y, stride_y, ptr_cb, ptr_cr, stride_c) for rank's kernels writing into a packed
        buffer at device address base_ptr: picture row y of the stripe maps to segment row
        y - y0.  Only rows inside the stripe are ever written."""
        y0, _ = stripe_rows(self.H, self.world, rank, self.ctu)
        seg = base_ptr + 2 * rank * self.seg
        py = seg - 2 * y0 * self.W
        pcb = seg + 2 * self.luma - 2 * (y0 // 2) * (self.W // 2)
        pcr = pcb + 2 * self.chroma
        return py, self.W, pcb, pcr, self.W // 2

    def pack(self, planes, rank: int, out: np.ndarray) -> None:
        """Host helper: copy rank's stripe of full planes (Y, Cb, Cr) into its segment of `out`."""
        y0, y1 = stripe_rows(self.H, self.world, rank, self.ctu)
        s = out[rank * self.seg:(rank + 1) * self.seg]
        s[: (y1 - y0) * self.W] = planes[0][y0:y1].reshape(-1)
        c0, c1, wc = y0 // 2, y1 // 2, self.W // 2
        s[self.luma:self.luma + (c1 - c0) * wc] = planes[1][c0:c1].reshape(-1)
        s[self.luma + self.chroma:self.luma + self.chroma + (c1 - c0) * wc] = planes[2][c0:c1].reshape(-1)

    def unpack(self, buf: np.ndarray):
        """Full (Y, Cb, Cr) planes from a packed picture (host int16 array of `total` elements)."""
        W, wc = self.W, self.W // 2
        y = np.zeros((self.H, W), dtype=np.int16)
        cb = np.zeros((self.H // 2, wc), dtype=np.int16)
        cr = np.zeros_like(cb)
        for r in range(self.world):
            y0, y1 = stripe_rows(self.H, self.world, r, self.ctu)
            s = buf[r * self.seg:(r + 1) * self.seg]
            y[y0:y1] = s[: (y1 - y0) * W].reshape(y1 - y0, W)
            c0, c1 = y0 // 2, y1 // 2
            cb[c0:c1] = s[self.luma:self.luma + (c1 - c0) * wc].reshape(c1 - c0, wc)
            cr[c0:c1] = s[self.luma + self.chroma:self.luma + self.chroma + (c1 - c0) * wc].reshape(c1 - c0, wc)
        return y, cb, cr


def samples_per_word(bit_depth: int) -> int:
    """K of the packed C4 transport (include/mm360.h): bit_depth-bit samples per 32-bit word."""
    return 32 // bit_depth


def packed_words(layout: StripeLayout, bit_depth: int) -> int:
    """32-bit words per packed segment (mm_stripe_packed_dwords)."""
    k = samples_per_word(bit_depth)
    return (layout.seg + k - 1) // k


def pack_samples(samples: np.ndarray, bit_depth: int) -> np.ndarray:
    """Host restatement of mm_pack_samples (the format's definition, used by the CPU tests and the
    gloo rehearsal): sample j in bits (j % K) * bit_depth of word j // K, K = 32 // bit_depth."""
    k = samples_per_word(bit_depth)
    v = samples.astype(np.int64).ravel() & ((1 << bit_depth) - 1)
    v = np.concatenate([v, np.zeros((-len(v)) % k, dtype=np.int64)]).reshape(-1, k)
    w = np.zeros(len(v), dtype=np.uint64)
    for i in range(k):
        w |= (v[:, i].astype(np.uint64) << np.uint64(i * bit_depth))
    return w.astype(np.uint32)


def unpack_samples(words: np.ndarray, n: int, bit_depth: int) -> np.ndarray:
    """The inverse: the first n samples of packed words, as int16."""
    k = samples_per_word(bit_depth)
    w = words.astype(np.uint64).ravel()
    cols = [((w >> np.uint64(i * bit_depth)) & np.uint64((1 << bit_depth) - 1)) for i in range(k)]
    return np.stack(cols, axis=1).ravel()[:n].astype(np.int16)


def pack_segment(buf: np.ndarray, layout: StripeLayout, rank: int, bit_depth: int, out: np.ndarray) -> None:
    """Pack rank's int16 segment of the stripe-major picture into its segment of the packed buffer
    `out` (uint32, world x packed_words)."""
    nw = packed_words(layout, bit_depth)
    out[rank * nw:(rank + 1) * nw] = pack_samples(buf[rank * layout.seg:(rank + 1) * layout.seg], bit_depth)


def unpack_picture(words: np.ndarray, layout: StripeLayout, bit_depth: int):
    """Full (Y, Cb, Cr) planes of a gathered packed picture (what mm_upload_ref_packed reads)."""
    nw = packed_words(layout, bit_depth)
    buf = np.concatenate([unpack_samples(words[r * nw:(r + 1) * nw], layout.seg, bit_depth)
                          for r in range(layout.world)])
    return layout.unpack(buf)


def allgather_packed(buf, layout: StripeLayout, group=None, async_op: bool = False):
    """In place: the one collective of a sharded picture.  `buf` (torch int16, layout.total
    elements -- or the packed form, int32, world x packed_words) holds this rank's segment;
    afterwards every rank holds every segment.  The samples travel bit-exactly as bytes (RCCL and
    gloo have no int16 type)."""
    import torch
    import torch.distributed as dist

    rank = dist.get_rank(group)
    b8 = buf.view(-1).view(torch.uint8)
    seg = b8.numel() // layout.world
    return dist.all_gather_into_tensor(b8, b8[rank * seg:(rank + 1) * seg], group=group, async_op=async_op)
