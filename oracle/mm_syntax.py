"""CPU restatement of the MM bitstream syntax -- TEST INFRASTRUCTURE ONLY.

Only tests/ import this module; the product (vvc-extension-mm_amd/csrc/mm_syntax.h behind the
C-ABI) never does.  Parity status: UNPINNED -- the reference ships no MM bitstream and its coder
cannot be built here (Eigen), so no reference-produced bits exist to pin against.  What pins it
instead is independence of formulation:

* the arithmetic coder here is the H.266 specification's bit-serial formulation (9-bit ivlOffset,
  RenormD one bit at a time, 10-bit ivlLow with bitsOutstanding / PutBit on the encoder side,
  EncodeFlush writing the stop bit), with the probability state as the spec's pStateIdx0 (10 bit)
  / pStateIdx1 (14 bit) pair -- while the product restates VTM's byte-oriented engine
  (BinEncoder.cpp:94-390, BinDecoder.cpp:73-362) over its 15-bit packed states (Contexts.h:87-155);
  the two must agree bit for bit;
* Exp-Golomb codes are built as bit strings from their definition (H.266 9.2), not from the
  VLCWriter / VLCReader loops the product follows.

Syntax order and conditions follow VLCReader.cpp:1920-1980 (SPS), :3354-3372 (PH) and
CABACReader.cpp:2170-2322 (motion_model) -- cited per function below.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

CLASSIC, MPA_FB, MPA_LR, MPA_TB, TAN, T3D, ROT, GED_X, GED_Y, GED_Z, GED_CAMPOSE = range(11)
INVALID = -1
EQUISOLID, CALIBRATED, EQUIRECTANGULAR = 0, 1, 2
MAX_CALIB = 16

SPS_FIELDS = ("mpa", "t3d", "tan", "rot", "ged", "geda", "ged_flavor", "mmmvp", "mm_offset_4x4",
              "projection_fct", "focal_length_px", "optical_center_x_px", "optical_center_y_px",
              "num_calibrated_coeffs", "calibrated_coeffs", "global_epipole")


class SyntaxError_(ValueError):
    pass


# ------------------------------------------------------------------------------- bit strings
def ue_bits(v: int) -> str:
    """ue(v): k leading zeros, then (v + 1) in k + 1 bits (H.266 9.2.1)."""
    if not 0 <= v <= 0xFFFFFFFE:
        raise SyntaxError_("ue(v) out of range")
    b = bin(v + 1)[2:]
    return "0" * (len(b) - 1) + b


def se_bits(v: int) -> str:
    """se(v): k > 0 -> 2k - 1, k <= 0 -> -2k (H.266 Table 9-3)."""
    if not -(2 ** 31 - 1) <= v <= 2 ** 31 - 1:
        raise SyntaxError_("se(v) out of range")
    return ue_bits(2 * v - 1 if v > 0 else -2 * v)


class Bits:
    def __init__(self, s: str, pos: int = 0):
        self.s, self.pos = s, pos

    def u(self, n: int) -> int:
        if self.pos + n > len(self.s):
            raise SyntaxError_("truncated")
        v = int(self.s[self.pos:self.pos + n] or "0", 2)
        self.pos += n
        return v

    def ue(self) -> int:
        k = 0
        while self.u(1) == 0:
            k += 1
            if k > 31:
                raise SyntaxError_("ue(v) prefix too long")
        return (1 << k) - 1 + self.u(k)

    def se(self) -> int:
        k = self.ue()
        return (k + 1) // 2 if k & 1 else -(k // 2)


def bytes_to_bits(b: bytes) -> str:
    return "".join(f"{x:08b}" for x in b)


def bits_to_bytes(s: str) -> bytes:
    s = s + "0" * (-len(s) % 8)
    return bytes(int(s[i:i + 8], 2) for i in range(0, len(s), 8))


# -------------------------------------------------------------------------------- SPS and PH
def multi_model(sps: dict) -> bool:  # MMConfig.h:32
    return any(sps.get(k, 0) for k in ("mpa", "t3d", "tan", "rot", "ged", "geda"))


def sps_bits(sps: dict) -> str:
    """VLCWriter.cpp:1110-1142 (the order VLCReader.cpp:1920-1980 parses)."""
    f = lambda k: str(int(bool(sps.get(k, 0))))  # noqa: E731
    out = "".join(f(k) for k in ("mpa", "t3d", "tan", "rot", "ged", "geda"))
    if not multi_model(sps):
        return out
    if not 0 <= sps.get("mm_offset_4x4", 0) <= 4 or not 0 <= sps.get("projection_fct", 0) <= 2:
        raise SyntaxError_("range")
    if sps.get("ged") or sps.get("geda"):
        out += ue_bits(sps.get("ged_flavor", 0))
    out += f("mmmvp") + ue_bits(sps.get("mm_offset_4x4", 0)) + ue_bits(sps.get("projection_fct", 0))
    proj = sps.get("projection_fct", 0)
    if proj in (EQUISOLID, CALIBRATED):
        out += "".join(ue_bits(sps.get(k, 0)) for k in ("focal_length_px", "optical_center_x_px",
                                                       "optical_center_y_px"))
    if proj == CALIBRATED:
        n = sps.get("num_calibrated_coeffs", 0)
        if n > MAX_CALIB:
            raise SyntaxError_("range")
        out += ue_bits(n) + "".join(ue_bits(c & 0xFFFFFFFF) for c in sps.get("calibrated_coeffs", [])[:n])
    if sps.get("ged"):
        out += "".join(se_bits(v) for v in sps.get("global_epipole", (0, 0, 0)))
    return out


def parse_sps(r: Bits) -> dict:
    """VLCReader.cpp:1920-1980; uncoded fields are the MMConfig defaults (MMConfig.h:15-30)."""
    s = {k: 0 for k in SPS_FIELDS}
    s["calibrated_coeffs"], s["global_epipole"] = [], [0, 0, 0]
    for k in ("mpa", "t3d", "tan", "rot", "ged", "geda"):
        s[k] = r.u(1)
    if not multi_model(s):
        return s
    if s["ged"] or s["geda"]:
        s["ged_flavor"] = r.ue()
    s["mmmvp"] = r.u(1)
    s["mm_offset_4x4"] = r.ue()
    if s["mm_offset_4x4"] > 4:
        raise SyntaxError_("sps_mm_offset_4x4")
    s["projection_fct"] = r.ue()
    if s["projection_fct"] >= 3:
        raise SyntaxError_("sps_projection_fct")
    if s["projection_fct"] in (EQUISOLID, CALIBRATED):
        for k in ("focal_length_px", "optical_center_x_px", "optical_center_y_px"):
            s[k] = r.ue()
    if s["projection_fct"] == CALIBRATED:
        s["num_calibrated_coeffs"] = r.ue()
        if s["num_calibrated_coeffs"] > MAX_CALIB:
            raise SyntaxError_("sps_num_calibrated_coeffs")
        s["calibrated_coeffs"] = [(lambda v: v - (1 << 32) if v >= 1 << 31 else v)(r.ue())
                                  for _ in range(s["num_calibrated_coeffs"])]
    if s["ged"]:
        s["global_epipole"] = [r.se() for _ in range(3)]
    return s


def ph_bits(sps: dict, delta: Sequence[int]) -> str:
    """VLCWriter.cpp:2096-2109."""
    if not (multi_model(sps) and sps.get("ged")):
        return ""
    if not any(delta):
        return "0"
    return "1" + "".join(se_bits(v) for v in delta)


def parse_ph(r: Bits, sps: dict) -> List[int]:
    """VLCReader.cpp:3354-3372."""
    if not (multi_model(sps) and sps.get("ged")):
        return [0, 0, 0]
    return [r.se() for _ in range(3)] if r.u(1) else [0, 0, 0]


# -------------------------------------------------------------- arithmetic coding (spec form)
class Ctx:
    """H.266 9.3.2.2: pStateIdx0 / pStateIdx1 from initValue; shiftIdx -> shift0 / shift1."""

    def __init__(self, qp: int, init_value: int = 35, shift_idx: int = 1):
        m, n = (init_value >> 3) - 4, (init_value & 7) * 18 + 1
        pre = min(max(((m * (min(max(qp, 0), 63) - 16)) >> 1) + n, 1), 127)
        self.p0, self.p1 = pre << 3, pre << 7
        self.sh0 = (shift_idx >> 2) + 2
        self.sh1 = (shift_idx & 3) + 3 + self.sh0

    def lps(self, rng: int):
        p = self.p1 + 16 * self.p0
        mps = p >> 14
        return ((rng >> 5) * ((32767 - p if mps else p) >> 9) >> 1) + 4, mps

    def update(self, b: int):
        self.p0 = self.p0 - (self.p0 >> self.sh0) + ((1023 * b) >> self.sh0)
        self.p1 = self.p1 - (self.p1 >> self.sh1) + ((16383 * b) >> self.sh1)


class SpecEncoder:
    """The spec's informative encoder: ivlLow 10 bits, PutBit with bitsOutstanding."""

    def __init__(self):
        self.low, self.rng, self.first, self.outstanding, self.out = 0, 510, True, 0, []

    def _put(self, b: int):
        if self.first:
            self.first = False
        else:
            self.out.append(b)
        while self.outstanding:
            self.out.append(1 - b)
            self.outstanding -= 1

    def _renorm(self):
        while self.rng < 256:
            if self.low < 256:
                self._put(0)
            elif self.low >= 512:
                self.low -= 512
                self._put(1)
            else:
                self.low -= 256
                self.outstanding += 1
            self.rng <<= 1
            self.low <<= 1

    def decision(self, ctx: Ctx, b: int):
        lps, mps = ctx.lps(self.rng)
        self.rng -= lps
        if b != mps:
            self.low += self.rng
            self.rng = lps
        ctx.update(b)
        self._renorm()

    def bypass(self, b: int):
        self.low <<= 1
        if b:
            self.low += self.rng
        if self.low >= 1024:
            self._put(1)
            self.low -= 1024
        elif self.low < 512:
            self._put(0)
        else:
            self.low -= 512
            self.outstanding += 1

    def terminate(self, b: int):
        self.rng -= 2
        if b:
            self.low += self.rng
            self.rng = 2  # EncodeFlush
            self._renorm()
            self._put((self.low >> 9) & 1)
            v = ((self.low >> 7) & 3) | 1  # the last bit is rbsp_stop_one_bit
            self.out += [v >> 1, v & 1]
        else:
            self._renorm()

    def data(self) -> bytes:
        return bits_to_bytes("".join(map(str, self.out)))


class SpecDecoder:
    """H.266 9.3.4.3: ivlOffset read 9 bits at init and one bit per renormalisation step."""

    def __init__(self, data: bytes):
        self.r = Bits(bytes_to_bits(data))
        self.rng, self.off = 510, self.r.u(9)

    def decision(self, ctx: Ctx) -> int:
        lps, mps = ctx.lps(self.rng)
        self.rng -= lps
        if self.off >= self.rng:
            b = 1 - mps
            self.off -= self.rng
            self.rng = lps
        else:
            b = mps
        ctx.update(b)
        while self.rng < 256:
            self.rng <<= 1
            self.off = (self.off << 1) | self.r.u(1)
        return b

    def bypass(self) -> int:
        self.off = (self.off << 1) | self.r.u(1)
        if self.off >= self.rng:
            self.off -= self.rng
            return 1
        return 0

    def terminate(self) -> int:
        self.rng -= 2
        if self.off >= self.rng:
            return 1
        while self.rng < 256:
            self.rng <<= 1
            self.off = (self.off << 1) | self.r.u(1)
        return 0

    def end(self) -> None:
        """After end_of_slice_segment_flag = 1: the last bit inserted into ivlOffset is the
        rbsp_stop_one_bit (the last bit EncodeFlush writes); only alignment zeros may follow."""
        if self.r.s[self.r.pos - 1] != "1":
            raise SyntaxError_("rbsp_stop_one_bit")
        rest = self.r.s[self.r.pos:]
        if len(rest) >= 8 or "1" in rest:
            raise SyntaxError_("trailing data")


# ------------------------------------------------------------------ motion_model() syntax
def active_models(sps: dict) -> List[int]:
    """MMConfig::getActiveMotionModels (MMConfig.cpp:7-39)."""
    out = [CLASSIC]
    if sps.get("mpa"):
        out += [MPA_FB, MPA_LR, MPA_TB]
    if sps.get("t3d"):
        out.append(T3D)
    if sps.get("tan"):
        out.append(TAN)
    if sps.get("rot"):
        out.append(ROT)
    if sps.get("ged"):
        out.append(GED_CAMPOSE)
    if sps.get("geda"):
        out += [GED_X, GED_Y, GED_Z]
    return out


def candidates(sps: dict, pred_type: int = 0, col=None, pic_w: int = 0, pic_h: int = 0, col_list: int = 0,
               x: int = 0, y: int = 0, w: int = 0, h: int = 0) -> List[int]:
    """CABACReader.cpp:2179-2296.  col: nested lists / array [gh][gw][2] of model ids (-1 INVALID)."""
    cand = active_models(sps)
    if pred_type == 0:
        return cand

    def front(p):
        if p in cand:  # erase(end()) is undefined in the reference; the product keeps the order
            cand.remove(p)
            cand.insert(0, p)

    if pred_type == 1:
        cx, cy = x + w // 2, y + h // 2
        front(int(col[cy >> 2][cx >> 2][col_list]))
        return cand
    vx, vy, vw, vh = x, y, w, h
    if pred_type == 3:
        if vw < 32:
            vx -= (32 - vw) >> 1
            vw = 32
            if vx < 0:
                vw, vx = vw + vx, 0
            if vx + vw > pic_w:
                vw -= vx + vw - pic_w
        if vh < 32:
            vy -= (32 - vh) >> 1
            vh = 32
            if vy < 0:
                vh, vy = vh + vy, 0
            if vy + vh > pic_h:
                vh -= vy + vh - pic_h
    votes = {}
    for yy in range(vy >> 2, (vy >> 2) + (vh >> 2)):
        for xx in range(vx >> 2, (vx >> 2) + (vw >> 2)):
            m = int(col[yy][xx][col_list])
            if m == INVALID:
                m = int(col[yy][xx][1 - col_list])
            votes[m] = votes.get(m, 0) + 1
    if pred_type == 2:
        best, mx = INVALID, 0
        for k in sorted(votes):
            if votes[k] > mx:
                best, mx = k, votes[k]
        front(best)
        return cand
    return sorted(cand, key=lambda m: -votes.get(m, 0))  # Python's sort is stable


def _binarise(cand: Sequence[int], depth: int, model: int):
    """(context bins [(ctx id, bin)], (bypass value, bypass bins) or None): CABACWriter.cpp:1984-2000."""
    n = len(cand)
    k = list(cand).index(model)
    ctx_bins = []
    for i in range(min(k + 1, n - 1, depth)):
        ctx_bins.append((cand[i], int(i == k)))
    if k >= depth and depth < n - 1:
        return ctx_bins, (k - depth, n - depth)
    return ctx_bins, None


def encode_models(sps: dict, models: Sequence[int], cands: Sequence[Sequence[int]], qp: int = 32, depth: int = 9,
                  affine: Optional[Sequence[int]] = None) -> bytes:
    ctxs = {m: Ctx(qp) for m in range(11)}
    e = SpecEncoder()
    for p, model in enumerate(models):
        if not multi_model(sps) or (affine is not None and affine[p]):
            if model != CLASSIC:
                raise SyntaxError_("non-CLASSIC model without MM bins")
            continue
        ctx_bins, ep = _binarise(cands[p], depth, model)
        for c, b in ctx_bins:
            e.decision(ctxs[c], b)
        if ep is not None:
            v, nb = ep
            for i in range(nb - 1, -1, -1):
                e.bypass((v >> i) & 1)
    e.terminate(1)
    return e.data()


def decode_models(sps: dict, data: bytes, cands: Sequence[Sequence[int]], qp: int = 32, depth: int = 9,
                  affine: Optional[Sequence[int]] = None) -> List[int]:
    """CABACReader.cpp:2300-2322 over the spec decoder."""
    ctxs = {m: Ctx(qp) for m in range(11)}
    d = SpecDecoder(data)
    out = []
    for p, cand in enumerate(cands):
        if not multi_model(sps) or (affine is not None and affine[p]):
            out.append(CLASSIC)
            continue
        n, got = len(cand), None
        for i in range(n):
            if i == n - 1:
                got = cand[i]
                break
            if i < depth:
                if d.decision(ctxs[cand[i]]):
                    got = cand[i]
                    break
            else:
                idx = 0
                for _ in range(n - depth):
                    idx = (idx << 1) | d.bypass()
                if idx >= n - depth:
                    raise SyntaxError_("bypass index past the list")
                got = cand[depth + idx]
                break
        out.append(got)
    if d.terminate() != 1:
        raise SyntaxError_("end_of_slice_segment_flag")
    d.end()
    return out
