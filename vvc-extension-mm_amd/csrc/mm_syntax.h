// mm_syntax.h -- the bitstream side of the MM extension, host code.
//
// What a decoder needs besides the reprojection / MC hot path to read an MM bitstream:
//   * the SPS fragment that switches the motion models on and carries the camera parameters
//     (DecoderLib/VLCReader.cpp:1920-1980, written by EncoderLib/VLCWriter.cpp:1110-1142),
//   * the picture header's epipole delta (VLCReader.cpp:3354-3372, VLCWriter.cpp:2096-2109),
//   * the per-PU motion_model() syntax element, CABAC coded (DecoderLib/CABACReader.cpp:2170-2322,
//     EncoderLib/CABACWriter.cpp:1854-2000) with its candidate ordering from the collocated picture
//     and the MotionModel context set (CommonLib/Contexts.cpp:420-426: init value 35 in every slice
//     type, window-size code 1).
// The CABAC engine is VVC's (BinEncoder.cpp:94-390, BinDecoder.cpp:73-362, the dual-window
// probability model Contexts.h:87-155 / Contexts.cpp:123-132 and m_RenormTable_32 Contexts.cpp:45).
// Everything here is bit-serial host work (a few bins per PU); it has no GPU part by design.
#pragma once
#include <algorithm>
#include <climits>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/mm360.h"

namespace mmsyn {

// MotionModelID (CommonLib/TypeDef.h:865-879)
enum { CLASSIC = 0, MPA_FB = 1, MPA_LR = 2, MPA_TB = 3, TAN = 4, T3D = 5, ROT = 6, GED_X = 7, GED_Y = 8,
       GED_Z = 9, GED_CAMPOSE = 10, NUM_MODELS = 11, INVALID = -1 };
// ProjectionID (CommonLib/Projection.h:12-17)
enum { EQUISOLID = 0, CALIBRATED = 1, EQUIRECTANGULAR = 2, NUM_PROJECTIONS = 3 };
constexpr int MAX_CALIB = MM_MAX_CALIB_COEFFS;

// ---------------------------------------------------------------- fixed-length / Exp-Golomb bits
// MSB-first bit writer into a caller buffer (OutputBitstream::write semantics); `bad` on overflow.
struct BitWriter {
  uint8_t* buf;
  int64_t cap_bits, pos;
  bool bad = false;
  void put(uint32_t v, int n) {  // n <= 32, the low n bits of v, MSB first
    if (n <= 0) return;
    if (pos + n > cap_bits) {
      bad = true;
      return;
    }
    for (int i = n - 1; i >= 0; --i, ++pos) {
      const uint8_t m = uint8_t(0x80u >> (pos & 7));
      if ((v >> i) & 1u)
        buf[pos >> 3] |= m;
      else
        buf[pos >> 3] &= uint8_t(~m);
    }
  }
  // VLCWriter::xWriteUvlc (VLCWriter.cpp:131-146): length = 2*floor(log2(v+1)) + 1
  void ue(uint32_t v) {
    const uint32_t code = v + 1;
    if (code == 0) {  // CHECK(!temp, "Integer overflow")
      bad = true;
      return;
    }
    int len = 1;
    for (uint32_t t = code; t != 1; t >>= 1) len += 2;
    put(0, len >> 1);
    put(code, (len + 1) >> 1);
  }
  // VLCWriter::xWriteSvlc (VLCWriter.cpp:148-152)
  void se(int32_t v) {
    if (v == INT32_MIN) {  // (-iCode) << 1 does not fit
      bad = true;
      return;
    }
    ue(v <= 0 ? uint32_t(-int64_t(v)) << 1 : (uint32_t(v) << 1) - 1);
  }
};

struct BitReader {
  const uint8_t* buf;
  int64_t nbits, pos;
  bool bad = false;
  uint32_t get(int n) {
    if (n <= 0) return 0;
    if (pos + n > nbits) {
      bad = true;
      pos = nbits;
      return 0;
    }
    uint32_t v = 0;
    for (int i = 0; i < n; ++i, ++pos) v = (v << 1) | ((buf[pos >> 3] >> (7 - (pos & 7))) & 1u);
    return v;
  }
  // VLCReader::xReadUvlc (VLCReader.cpp:145-180).  More than 31 leading zeros is not a uint32
  // code (the reference's `1 << length` would overflow): flagged as malformed.
  uint32_t ue() {
    if (get(1)) return 0;
    int len = 0;  // leading zeros
    for (;;) {
      const uint32_t b = get(1);
      if (bad) return 0;
      ++len;
      if (b) break;
    }
    if (len > 31) {
      bad = true;
      return 0;
    }
    const uint32_t suffix = get(len);
    return suffix + ((1u << len) - 1u);
  }
  // VLCReader::xReadSvlc (VLCReader.cpp:183-215): odd codes positive
  int32_t se() {
    const uint32_t c = ue();
    const int64_t m = (int64_t(c) + 1) >> 1;
    return (c & 1u) ? int32_t(m) : int32_t(-m);
  }
};

// ----------------------------------------------------------------------------- SPS / PH syntax
using SpsMM = mm_sps_mm;  // include/mm360.h
inline bool use_multi_model(const SpsMM& s) {  // MMConfig::getUseMultiModel (MMConfig.h:32)
  return s.mpa || s.t3d || s.tan || s.rot || s.ged || s.geda;
}
// MMConfig::getActiveMotionModels (MMConfig.cpp:7-39) -- the CABAC candidate order, NOT id order
inline int active_models(const SpsMM& s, int32_t* out) {
  int n = 0;
  out[n++] = CLASSIC;
  if (s.mpa) out[n++] = MPA_FB, out[n++] = MPA_LR, out[n++] = MPA_TB;
  if (s.t3d) out[n++] = T3D;
  if (s.tan) out[n++] = TAN;
  if (s.rot) out[n++] = ROT;
  if (s.ged) out[n++] = GED_CAMPOSE;
  if (s.geda) out[n++] = GED_X, out[n++] = GED_Y, out[n++] = GED_Z;
  return n;
}

// The range rules both sides hold: the reader's CHECKs (VLCReader.cpp:1948-1954) plus the array
// bound of calibratedCoeffsPx, which the reader does not check (it would write past the array).
inline bool sps_valid(const SpsMM& s) {
  if (!use_multi_model(s)) return true;
  return s.mm_offset_4x4 >= 0 && s.mm_offset_4x4 <= 4 && s.projection_fct >= 0 && s.projection_fct < NUM_PROJECTIONS &&
         ((!s.ged && !s.geda) || s.ged_flavor >= 0) &&
         (s.projection_fct != CALIBRATED || s.num_calibrated_coeffs <= uint32_t(MAX_CALIB));
}

// VLCWriter.cpp:1110-1142
inline void write_sps_mm(BitWriter& w, const SpsMM& s) {
  w.put(s.mpa != 0, 1);
  w.put(s.t3d != 0, 1);
  w.put(s.tan != 0, 1);
  w.put(s.rot != 0, 1);
  w.put(s.ged != 0, 1);
  w.put(s.geda != 0, 1);
  if (!use_multi_model(s)) return;
  if (s.ged || s.geda) w.ue(uint32_t(s.ged_flavor));
  w.put(s.mmmvp != 0, 1);
  w.ue(uint32_t(s.mm_offset_4x4));
  w.ue(uint32_t(s.projection_fct));
  if (s.projection_fct == EQUISOLID || s.projection_fct == CALIBRATED) {
    w.ue(s.focal_length_px);
    w.ue(s.optical_center_x_px);
    w.ue(s.optical_center_y_px);
  }
  if (s.projection_fct == CALIBRATED) {
    w.ue(s.num_calibrated_coeffs);
    for (uint32_t i = 0; i < s.num_calibrated_coeffs; ++i) w.ue(uint32_t(s.calibrated_coeffs[i]));
  }
  if (s.ged)
    for (int i = 0; i < 3; ++i) w.se(s.global_epipole[i]);
}

// VLCReader.cpp:1920-1980; fields the bitstream does not carry keep the MMConfig defaults (0).
// Returns false on a range violation or a truncated fragment.
inline bool read_sps_mm(BitReader& r, SpsMM& s) {
  std::memset(&s, 0, sizeof s);
  s.mpa = int32_t(r.get(1));
  s.t3d = int32_t(r.get(1));
  s.tan = int32_t(r.get(1));
  s.rot = int32_t(r.get(1));
  s.ged = int32_t(r.get(1));
  s.geda = int32_t(r.get(1));
  if (r.bad) return false;
  if (!use_multi_model(s)) return true;
  if (s.ged || s.geda) s.ged_flavor = int32_t(r.ue());
  s.mmmvp = int32_t(r.get(1));
  const uint32_t off = r.ue();
  if (r.bad || off > 4) return false;  // VLCReader.cpp:1948
  s.mm_offset_4x4 = int32_t(off);
  const uint32_t proj = r.ue();
  if (r.bad || proj >= uint32_t(NUM_PROJECTIONS)) return false;  // VLCReader.cpp:1952
  s.projection_fct = int32_t(proj);
  if (proj == EQUISOLID || proj == CALIBRATED) {
    s.focal_length_px = r.ue();
    s.optical_center_x_px = r.ue();
    s.optical_center_y_px = r.ue();
  }
  if (proj == CALIBRATED) {
    s.num_calibrated_coeffs = r.ue();
    if (r.bad || s.num_calibrated_coeffs > uint32_t(MAX_CALIB)) return false;
    for (uint32_t i = 0; i < s.num_calibrated_coeffs; ++i) s.calibrated_coeffs[i] = int32_t(r.ue());
  }
  if (s.ged)
    for (int i = 0; i < 3; ++i) s.global_epipole[i] = r.se();
  return !r.bad;
}

// VLCWriter.cpp:2096-2109: present iff multi-model and GED; the flag is "delta is not zero"
inline void write_ph_epipole(BitWriter& w, const SpsMM& s, const int32_t d[3]) {
  if (!(use_multi_model(s) && s.ged)) return;
  const bool signal = d[0] || d[1] || d[2];
  w.put(signal, 1);
  if (signal)
    for (int i = 0; i < 3; ++i) w.se(d[i]);
}
// VLCReader.cpp:3354-3372 (absent -> {0, 0, 0})
inline bool read_ph_epipole(BitReader& r, const SpsMM& s, int32_t d[3]) {
  d[0] = d[1] = d[2] = 0;
  if (!(use_multi_model(s) && s.ged)) return true;
  if (r.get(1))
    for (int i = 0; i < 3; ++i) d[i] = r.se();
  return !r.bad;
}

// ---------------------------------------------------------------------------------- CABAC engine
// BinProbModel_Std (Contexts.h:87-155): two probability estimates of 10 and 14 bits inside 15-bit
// words, adapted with window sizes rate0 / rate1.
constexpr int PROB_MASK_0 = 0x7fe0;  // ~(~0u << 10) << 5
constexpr int PROB_MASK_1 = 0x7ffe;  // ~(~0u << 14) << 1
struct ProbModel {
  uint16_t s0 = 1u << 14, s1 = 1u << 14;
  uint8_t rate = 8;
  // BinProbModel_Std::init (Contexts.cpp:123-132) + setLog2WindowSize (Contexts.h:113-119)
  void init(int qp, int init_id, int win_code) {
    const int slope = (init_id >> 3) - 4, offset = ((init_id & 7) * 18) + 1;
    int st = ((slope * (qp - 16)) >> 1) + offset;
    st = st < 1 ? 1 : st > 127 ? 127 : st;
    const int p1 = st << 8;
    s0 = uint16_t(p1 & PROB_MASK_0);
    s1 = uint16_t(p1 & PROB_MASK_1);
    const int r0 = 2 + ((win_code >> 2) & 3), r1 = 3 + r0 + (win_code & 3);
    rate = uint8_t(16 * r0 + r1);
  }
  unsigned state() const { return unsigned(s0 + s1) >> 8; }
  unsigned mps() const { return state() >> 7; }
  unsigned lps(unsigned range) const {
    unsigned q = state();
    if (q & 0x80) q ^= 0xff;
    return ((q >> 2) * (range >> 5) >> 1) + 4;
  }
  void update(unsigned bin) {
    const int r0 = rate >> 4, r1 = rate & 15;
    s0 = uint16_t(s0 - ((s0 >> r0) & PROB_MASK_0));
    s1 = uint16_t(s1 - ((s1 >> r1) & PROB_MASK_1));
    if (bin) {
      s0 = uint16_t(s0 + ((0x7fffu >> r0) & PROB_MASK_0));
      s1 = uint16_t(s1 + ((0x7fffu >> r1) & PROB_MASK_1));
    }
  }
};
// m_RenormTable_32 (Contexts.cpp:45-55), indexed by LPS >> 3
inline unsigned renorm_lps(unsigned lps) {
  static const uint8_t t[32] = {6, 5, 4, 4, 3, 3, 3, 3, 2, 2, 2, 2, 2, 2, 2, 2,
                                1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1};
  return t[lps >> 3];
}

// BinEncoderBase / TBinEncoder (BinEncoder.cpp:94-390) over a growable bit buffer
struct CabacEncoder {
  std::vector<uint8_t> out;
  int64_t nbits = 0;
  uint32_t low = 0, range = 510, buffered = 0xff, nbuffered = 0;
  int bits_left = 23;
  void put(uint32_t v, int n) {
    for (int i = n - 1; i >= 0; --i, ++nbits) {
      if ((nbits & 7) == 0) out.push_back(0);
      if ((v >> i) & 1u) out.back() |= uint8_t(0x80u >> (nbits & 7));
    }
  }
  void write_out() {  // BinEncoder.cpp:313-345
    const uint32_t lead = low >> (24 - bits_left);
    bits_left += 8;
    low &= 0xffffffffu >> bits_left;
    if (lead == 0xff) {
      nbuffered++;
    } else if (nbuffered > 0) {
      const uint32_t carry = lead >> 8;
      put(buffered + carry, 8);
      buffered = lead & 0xff;
      const uint32_t fill = (0xff + carry) & 0xff;
      for (; nbuffered > 1; --nbuffered) put(fill, 8);
    } else {
      nbuffered = 1;
      buffered = lead;
    }
  }
  void bin(unsigned b, ProbModel& m) {  // TBinEncoder::encodeBin (BinEncoder.cpp:354-390)
    const uint32_t l = m.lps(range);
    range -= l;
    if (b != m.mps()) {
      const int nb = int(renorm_lps(l));
      bits_left -= nb;
      low += range;
      low <<= nb;
      range = l << nb;
      if (bits_left < 12) write_out();
    } else if (range < 256) {  // getRenormBitsRange == 1
      bits_left -= 1;
      low <<= 1;
      range <<= 1;
      if (bits_left < 12) write_out();
    }
    m.update(b);
  }
  void bins_ep(uint32_t bins, unsigned n) {  // BinEncoder.cpp:173-206 (+ aligned 276-311)
    if (range == 256) {
      for (unsigned rem = n; rem > 0;) {
        const unsigned k = std::min(rem, 8u);
        const uint32_t nb = (bins >> (rem - k)) & ((1u << k) - 1);
        low = (low << k) + (nb << 8);
        rem -= k;
        bits_left -= int(k);
        if (bits_left < 12) write_out();
      }
      return;
    }
    while (n > 8) {
      n -= 8;
      const uint32_t pat = bins >> n;
      low <<= 8;
      low += range * pat;
      bins -= pat << n;
      bits_left -= 8;
      if (bits_left < 12) write_out();
    }
    low <<= n;
    low += range * bins;
    bits_left -= int(n);
    if (bits_left < 12) write_out();
  }
  void bin_trm(unsigned b) {  // BinEncoder.cpp:246-270
    range -= 2;
    if (b) {
      low += range;
      low <<= 7;
      range = 2 << 7;
      bits_left -= 7;
    } else if (range >= 256) {
      return;
    } else {
      low <<= 1;
      range <<= 1;
      bits_left--;
    }
    if (bits_left < 12) write_out();
  }
  void finish() {  // BinEncoder.cpp:105-130
    if (low >> (32 - bits_left)) {
      put(buffered + 1, 8);
      for (; nbuffered > 1; --nbuffered) put(0x00, 8);
      low -= 1u << (32 - bits_left);
    } else {
      if (nbuffered > 0) put(buffered, 8);
      for (; nbuffered > 1; --nbuffered) put(0xff, 8);
    }
    put(low >> 8, 24 - bits_left);
  }
  // end_of_slice_segment_flag = 1, finish, rbsp_trailing_bits (stop bit + alignment zeros)
  void end_of_slice() {
    bin_trm(1);
    finish();
    put(1, 1);
    while (nbits & 7) put(0, 1);
  }
};

// BinDecoderBase / TBinDecoder (BinDecoder.cpp:73-362); reading past the end sets `bad`
struct CabacDecoder {
  const uint8_t* in;
  int64_t n, pos = 0;
  uint32_t range = 510, value = 0;
  int bits_needed = -8;
  bool bad = false;
  uint32_t byte() {
    if (pos >= n) {
      bad = true;
      return 0;
    }
    return in[pos++];
  }
  void start() {
    value = byte() << 8;
    value += byte();
    range = 510;
    bits_needed = -8;
  }
  unsigned bin(ProbModel& m) {
    unsigned b = m.mps();
    const uint32_t l = m.lps(range);
    range -= l;
    const uint32_t sr = range << 7;
    if (value < sr) {
      if (range < 256) {
        range <<= 1;
        value <<= 1;
        if (++bits_needed >= 0) {
          value += byte() << bits_needed;
          bits_needed -= 8;
        }
      }
    } else {
      b = 1 - b;
      const int nb = int(renorm_lps(l));
      value = (value - sr) << nb;
      range = l << nb;
      bits_needed += nb;
      if (bits_needed >= 0) {
        value += byte() << bits_needed;
        bits_needed -= 8;
      }
    }
    m.update(b);
    return b;
  }
  uint32_t bins_ep(unsigned num) {
    uint32_t bins = 0;
    if (range == 256) {  // decodeAlignedBinsEP (BinDecoder.cpp:260-300)
      for (unsigned rem = num; rem > 0;) {
        const unsigned k = std::min(rem, 8u);
        bins = (bins << k) | ((value >> (15 - k)) & ((1u << k) - 1));
        value = (value << k) & 0x7fff;
        rem -= k;
        bits_needed += int(k);
        if (bits_needed >= 0) {
          value |= byte() << bits_needed;
          bits_needed -= 8;
        }
      }
      return bins;
    }
    unsigned rem = num;
    while (rem > 8) {
      value = (value << 8) + (byte() << (8 + bits_needed));
      uint32_t sr = range << 15;
      for (int i = 0; i < 8; ++i) {
        bins += bins;
        sr >>= 1;
        if (value >= sr) {
          bins++;
          value -= sr;
        }
      }
      rem -= 8;
    }
    bits_needed += int(rem);
    value <<= rem;
    if (bits_needed >= 0) {
      value += byte() << bits_needed;
      bits_needed -= 8;
    }
    uint32_t sr = range << (rem + 7);
    for (unsigned i = 0; i < rem; ++i) {
      bins += bins;
      sr >>= 1;
      if (value >= sr) {
        bins++;
        value -= sr;
      }
    }
    return bins;
  }
  unsigned bin_trm() {  // BinDecoder.cpp:217-246
    range -= 2;
    const uint32_t sr = range << 7;
    if (value >= sr) return 1;
    if (range < 256) {
      range += range;
      value += value;
      if (++bits_needed == 0) {
        value += byte();
        bits_needed = -8;
      }
    }
    return 0;
  }
  // BinDecoderBase::finish (BinDecoder.cpp:85-91): the last byte read holds the stop bit; and the
  // stream must end there (only alignment zeros follow the stop bit inside that byte)
  bool finish() const {
    if (bad || pos == 0) return false;
    const uint32_t last = in[pos - 1];
    return ((last << (8 + bits_needed)) & 0xff) == 0x80 && pos == n;
  }
};

// MotionModel context set: one context per MotionModelID, initId 35 in B / P / I, window code 1
// (Contexts.cpp:420-426).  init_type is the CtxStore table index: the slice type (B 0, P 1, I 2)
// after the cabac_init_flag swap (CABACReader.cpp:66-86).
struct MotionModelCtx {
  ProbModel m[NUM_MODELS];
  void init(int slice_qp, int init_type) {
    (void)init_type;  // every table holds 35 (CNU = 35, Contexts.cpp:176)
    const int qp = slice_qp < 0 ? 0 : slice_qp > 63 ? 63 : slice_qp;  // Clip3(0, MAX_QP, qp)
    for (auto& c : m) c.init(qp, 35, 1);
  }
};

// ------------------------------------------------------------------ motion_model() candidates
// col_models: the collocated picture's motion field on the 4x4 grid, [grid_h][grid_w][2] int8
// (MotionInfo::motionModel[list], -1 = INVALID).  Candidate order per CABACReader.cpp:2179-2296
// (identical in CABACWriter.cpp:1863-1980).  Returns false on a bad argument.
struct ColField {
  const int8_t* m;
  int gw, gh;
  int at(int x4, int y4, int list) const { return m[(size_t(y4) * gw + x4) * 2 + list]; }
};

// votes[0] counts INVALID, votes[1 + id] model id; std::map<MotionModelID, int> key order
inline void vote(const ColField& f, int x4, int y4, int w4, int h4, int list, int32_t votes[NUM_MODELS + 1]) {
  for (int i = 0; i <= NUM_MODELS; ++i) votes[i] = 0;
  for (int x = 0; x < w4; ++x)
    for (int y = 0; y < h4; ++y) {
      int mm = f.at(x4 + x, y4 + y, list);
      if (mm == INVALID) mm = f.at(x4 + x, y4 + y, 1 - list);
      votes[mm + 1]++;
    }
}

// pred_type 0 none, 1 centre point (list = colFromL0Flag), 2 voted, 3 sorted (list = the
// eColRefPicList of CABACReader.cpp:2205 / 2240); x, y, w, h the PU's luma area.
inline bool order_candidates(const SpsMM& s, int pred_type, const ColField* f, int pic_w, int pic_h, int list, int x,
                             int y, int w, int h, int32_t* cand, int* n_cand) {
  int n = active_models(s, cand);
  *n_cand = n;
  if (pred_type == 0) return true;
  if (!f || !f->m || list < 0 || list > 1 || pred_type < 0 || pred_type > 3 || w <= 0 || h <= 0 || x < 0 || y < 0 ||
      x + w > pic_w || y + h > pic_h || f->gw * 4 < pic_w || f->gh * 4 < pic_h)
    return false;
  auto check_field = [&](int x4, int y4, int w4, int h4) {
    for (int yy = y4; yy < y4 + h4; ++yy)
      for (int xx = x4; xx < x4 + w4; ++xx)
        for (int l = 0; l < 2; ++l) {
          const int v = f->at(xx, yy, l);
          if (v < INVALID || v >= NUM_MODELS) return false;
        }
    return true;
  };
  // the predicted model to the front; erase(find(...)) of a model the list does not hold is
  // undefined in the reference (vector::erase(end())) -- here the order then stays as it is
  auto to_front = [&](int pred) {
    int* it = std::find(cand, cand + n, pred);
    if (it == cand + n) return;
    std::rotate(cand, it, it + 1);
  };
  if (pred_type == 1) {  // getMotionInfo(blockCenter).motionModel[colFromL0Flag] (:2187-2196)
    const int cx = x + w / 2, cy = y + h / 2;
    if (!check_field(cx >> 2, cy >> 2, 1, 1)) return false;
    to_front(f->at(cx >> 2, cy >> 2, list));
    return true;
  }
  int vx = x, vy = y, vw = w, vh = h;
  if (pred_type == 3) {  // minimum 32x32 voting area, clipped to the picture (:2242-2265)
    if (vw < 32) {
      vx -= (32 - vw) >> 1;
      vw = 32;
      if (vx < 0) {
        vw += vx;
        vx = 0;
      }
      if (vx + vw > pic_w) vw -= (vx + vw) - pic_w;
    }
    if (vh < 32) {
      vy -= (32 - vh) >> 1;
      vh = 32;
      if (vy < 0) {
        vh += vy;
        vy = 0;
      }
      if (vy + vh > pic_h) vh -= (vy + vh) - pic_h;
    }
  }
  // CodingStructure::getMotionBuf: g_miScaling.scale of position and size (>> 2 each)
  const int x4 = vx >> 2, y4 = vy >> 2, w4 = vw >> 2, h4 = vh >> 2;
  if (!check_field(x4, y4, w4, h4)) return false;
  int32_t votes[NUM_MODELS + 1];
  vote(*f, x4, y4, w4, h4, list, votes);
  if (pred_type == 2) {  // first maximum in key order (:2222-2232)
    int best = INVALID, max_votes = 0;
    for (int k = 0; k <= NUM_MODELS; ++k)
      if (votes[k] > max_votes) max_votes = votes[k], best = k - 1;
    to_front(best);
    return true;
  }
  // std::sort by votes, descending: libstdc++ sorts <= 16 elements by insertion sort, which keeps
  // equal-vote candidates in list order -- a stable sort
  std::stable_sort(cand, cand + n, [&](int32_t a, int32_t b) { return votes[a + 1] > votes[b + 1]; });
  return true;
}

// CABACWriter::motion_model (CABACWriter.cpp:1984-2000): context bins "is it this one" for the
// first coding_depth candidates, then the rest as a fixed-length bypass index of
// (n - coding_depth) bins.
inline bool encode_motion_model(CabacEncoder& e, MotionModelCtx& ctx, const int32_t* cand, int n, int depth,
                                int model) {
  const int* it = std::find(cand, cand + n, model);
  if (it == cand + n) return false;
  for (int i = 0; i < n; ++i) {
    const int mm = cand[i];
    if (i != n - 1) {
      if (i < depth) {
        e.bin(model == mm, ctx.m[mm]);
      } else {
        e.bins_ep(uint32_t(it - cand - depth), unsigned(n - depth));
        break;
      }
    }
    if (model == mm) break;
  }
  return true;
}
// CABACReader::motion_model (CABACReader.cpp:2300-2322).  The bypass index can point past the
// list for an index of (n - depth) bins; the reference then reads out of bounds -- malformed here.
inline int decode_motion_model(CabacDecoder& d, MotionModelCtx& ctx, const int32_t* cand, int n, int depth) {
  for (int i = 0; i < n; ++i) {
    if (i == n - 1) return cand[i];
    if (i < depth) {
      if (d.bin(ctx.m[cand[i]])) return cand[i];
    } else {
      const uint32_t idx = d.bins_ep(unsigned(n - depth));
      if (idx >= uint32_t(n - depth)) return INVALID;
      return cand[depth + int(idx)];
    }
  }
  return INVALID;
}

}  // namespace mmsyn
