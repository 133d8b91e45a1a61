"""Random-access decode order and reference structure, for the multi-GPU (C4) picture loop.

Two GOPs:
  * "ra32": the reference's own RA configuration (cfg/encoder_randomaccess_vtm.cfg:15-51, GOPSize
    32): decode order, temporal id and the ACTIVE reference pictures of every picture (the first
    #ref_pics_active deltas of each list, POC_ref = POC - delta);
  * "ra8": a dyadic hierarchical-B GOP of 8 (decode order 8 4 2 1 3 6 5 7): each picture
    references the two ends of the interval it bisects, the key picture the previous key picture.

The C4 loop uses it to be honest about reference dependencies: picture k is motion-compensated
only after the all-gather of every picture it references has landed on every rank, so a
picture's all-gather can only overlap the prediction of pictures that do not reference it (in
practice: pictures of the same temporal layer)."""
from __future__ import annotations

from typing import Dict, List, Tuple

# (POC within the GOP, temporal id, active L0 deltas, active L1 deltas), decode order.
# Frame1..Frame32 of the reference's RA cfg (data, not code).
RA_GOP32: Tuple[Tuple[int, int, Tuple[int, ...], Tuple[int, ...]], ...] = (
    (32, 0, (32, 64), (32,)),
    (16, 1, (16, 32, 48), (-16,)),
    (8, 2, (8, 24, 16, 40), (-8, -24)),
    (4, 3, (4, 8, 20), (-4, -12, -28)),
    (2, 4, (2, 6, 18), (-2, -6, -14, -30)),
    (1, 5, (1,), (-1, -3)),
    (3, 5, (1, 3), (-1, -5)),
    (6, 4, (2, 4, 6), (-2, -10, -26)),
    (5, 5, (1, 5), (-1, -3)),
    (7, 5, (1, 3), (-1, -9)),
    (12, 3, (4, 8, 12), (-4, -20)),
    (10, 4, (2, 4, 6, 10), (-2, -6, -22)),
    (9, 5, (1, 5), (-1, -3)),
    (11, 5, (1, 3), (-1, -5)),
    (14, 4, (2, 4, 6, 14), (-2, -18)),
    (13, 5, (1, 5), (-1, -3)),
    (15, 5, (1, 3), (-1, -17)),
    (24, 2, (8, 16, 24), (-8,)),
    (20, 3, (4, 12, 20), (-4, -12)),
    (18, 4, (2, 10, 18), (-2, -6, -14)),
    (17, 5, (1, 9), (-1, -3)),
    (19, 5, (1, 3), (-1, -5)),
    (22, 4, (2, 6, 22), (-2, -10, 4)),
    (21, 5, (1, 5), (-1, -3)),
    (23, 5, (1, 3), (-1, -9)),
    (28, 3, (4, 8, 12), (-4,)),
    (26, 4, (2, 6, 10, 26), (-2, -6)),
    (25, 5, (1, 5), (-1, -3)),
    (27, 5, (1, 3), (-1, -5)),
    (30, 4, (2, 6, 14, 30), (-2,)),
    (29, 5, (1, 5), (-1, -3)),
    (31, 5, (1, 3), (-1,)),
)


def dyadic_gop(size: int):
    """(POC, temporal id, L0 deltas, L1 deltas) in decode order of a dyadic hierarchical-B GOP."""
    out = [(size, 0, (size,), ())]

    def split(lo, hi, tid):
        if hi - lo < 2:
            return
        mid = (lo + hi) // 2
        out.append((mid, tid, (mid - lo,), (mid - hi,)))
        split(lo, mid, tid + 1)
        split(mid, hi, tid + 1)

    split(0, size, 1)
    return tuple(out)


GOPS = {"ra32": RA_GOP32, "ra8": dyadic_gop(8)}


def decode_sequence(n_pictures: int, gop: str = "ra32", start: int = 0) -> List[Tuple[int, int, List[int]]]:
    """(absolute POC, temporal id, absolute POCs of its active references) of decode-order
    pictures start .. start + n - 1, GOP after GOP (references below POC 0 belong to a GOP
    decoded before the sequence and count as available)."""
    table = GOPS[gop]
    size = len(table)
    out = []
    for k in range(start, start + n_pictures):
        g, i = divmod(k, size)
        poc, tid, l0, l1 = table[i]
        cur = g * size + poc
        out.append((cur, tid, sorted({cur - d for d in l0 + l1})))
    return out


def is_referenced(poc: int, gop: str = "ra32") -> bool:
    """Whether any picture of the GOP structure references `poc` (periodic: by POC modulo the GOP
    size).  The highest temporal layer -- half the pictures, the odd POCs -- is never referenced:
    those pictures are output only, so the sharded decoder never needs them whole on every GPU."""
    table = GOPS[gop]
    size = len(table)
    residues = {(p - d) % size for p, _, l0, l1 in table for d in l0 + l1}
    return poc % size in residues


def schedule(n_pictures: int, mc_ms: float, allgather_ms: float, gop: str = "ra32",
             gather_all: bool = False, batch_ms: Dict[int, float] = None) -> Dict[str, float]:
    """Modelled per-picture time of the CTU-row-sharded C4 loop: picture k's MC starts when the
    GPUs are free (picture k-1's MC is done) and the all-gathers of all its references have
    landed; a referenced picture (every picture with gather_all) is all-gathered after its MC, one
    all-gather at a time on the links (RCCL's stream serialises them).  batch_ms {k: ms per picture}
    (k >= 2): consecutive decode-order pictures none of which references another (DependencyLoop.
    next_batch, up to max(batch_ms) of them) are predicted together at that per-picture time, once
    all their references have landed.  n_pictures should be a whole number of GOPs."""
    seq = decode_sequence(n_pictures, gop)
    max_pics = max(batch_ms) if batch_ms else 1
    landed: Dict[int, float] = {}
    t_mc = 0.0
    link = 0.0
    stall = 0.0
    i = 0
    while i < len(seq):
        batch = [seq[i]]
        while (len(batch) < max_pics and i + len(batch) < len(seq)
               and not any(r == p for r in seq[i + len(batch)][2] for p, _, _ in batch)):
            batch.append(seq[i + len(batch)])
        k = len(batch)
        per = mc_ms if k == 1 else batch_ms[k]
        ready = max([t_mc] + [landed.get(r, 0.0) for _, _, refs in batch for r in refs])
        stall += ready - t_mc
        t_mc = ready + k * per
        for poc, _, _ in batch:
            if gather_all or is_referenced(poc, gop):
                link = max(t_mc, link) + allgather_ms
                landed[poc] = link
        i += k
    total = max(t_mc, link)
    return {"ms_per_picture": total / n_pictures, "stall_ms_per_picture": stall / n_pictures}


class DependencyLoop:
    """Drives the picture loop of one rank in decode order: before picture k is predicted, the
    all-gathers of its references are waited for (`wait(handle)`, a stream wait for RCCL); then
    `predict(k, poc, refs, buf)` writes the rank's stripe and, for a picture that later pictures
    reference (every picture with gather_all), `gather(buf)` starts its all-gather and returns its
    handle; an unreferenced picture stays sharded (each rank outputs its own stripe).  Picture
    buffers rotate over `n_bufs`; a buffer is reused only after its previous picture's all-gather
    is done.  A None handle (a synchronous all-gather) is never waited for.  ref_waits False drops
    the reference waits (the dependency-free upper bound)."""

    def __init__(self, gop: str, n_bufs: int, predict, gather, wait, start: int = 0, ref_waits: bool = True,
                 gather_all: bool = False):
        self.gop, self.n_bufs, self.ref_waits, self.gather_all = gop, n_bufs, ref_waits, gather_all
        self.gathered: List[int] = []  # POCs all-gathered, in decode order
        self.predict, self.gather, self.wait = predict, gather, wait
        self.k = start
        self.handles: Dict[int, object] = {}
        self.buf_handle: List[object] = [None] * n_bufs
        self.trace: List[Tuple[int, List[int]]] = []  # (POC, references waited for)

    def step(self) -> int:
        (poc, _, refs), = decode_sequence(1, self.gop, self.k)
        waited = []
        for r in refs if self.ref_waits else ():
            h = self.handles.get(r)
            if h is not None:
                self.wait(h)
                waited.append(r)
        b = self.k % self.n_bufs
        if self.buf_handle[b] is not None:
            self.wait(self.buf_handle[b])
        self.predict(self.k, poc, refs, b)
        h = None
        if self.gather_all or is_referenced(poc, self.gop):
            h = self.gather(b)
            self.gathered.append(poc)
            self.handles[poc] = h
        self.buf_handle[b] = h
        for old in [p for p in self.handles if p < poc - 2 * len(GOPS[self.gop])]:
            del self.handles[old]
        self.trace.append((poc, waited))
        self.k += 1
        return poc

    def next_batch(self, max_pics: int) -> List[Tuple[int, int, List[int]]]:
        """The pictures from decode position k on that can be predicted together (at most max_pics):
        none of them references another picture of the batch.  In RA order these are the runs of
        highest-temporal-layer leaves (GOP-32: 1 3, 5 7, 9 11, ...), which nothing references."""
        batch: List[Tuple[int, int, List[int]]] = []
        k = self.k
        while len(batch) < max_pics:
            (poc, tid, refs), = decode_sequence(1, self.gop, k)
            if any(r == p for r in refs for p, _, _ in batch):
                break
            batch.append((poc, tid, refs))
            k += 1
        return batch

    def step_batch(self, max_pics: int, predict_batch) -> List[int]:
        """step() for a batch of independent pictures (next_batch): the reference all-gathers of
        every picture of the batch are waited for, then predict_batch([(k, poc, refs, buf), ...])
        predicts them together (one launch chain), then each referenced one is all-gathered."""
        batch = self.next_batch(max_pics)
        assert len(batch) <= self.n_bufs
        items = []
        seen = set()
        for i, (poc, _, refs) in enumerate(batch):
            waited = []
            for r in refs if self.ref_waits else ():
                h = self.handles.get(r)
                if h is not None:
                    if r not in seen:
                        self.wait(h)
                        seen.add(r)
                    waited.append(r)
            b = (self.k + i) % self.n_bufs
            if self.buf_handle[b] is not None:
                self.wait(self.buf_handle[b])
            items.append((self.k + i, poc, refs, b))
            self.trace.append((poc, waited))
        predict_batch(items)
        for k, poc, _, b in items:
            h = None
            if self.gather_all or is_referenced(poc, self.gop):
                h = self.gather(b)
                self.gathered.append(poc)
                self.handles[poc] = h
            self.buf_handle[b] = h
        for old in [p for p in self.handles if p < items[-1][1] - 2 * len(GOPS[self.gop])]:
            del self.handles[old]
        self.k += len(items)
        return [poc for _, poc, _, _ in items]
