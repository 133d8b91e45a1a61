// mm_epipole.h -- EpipoleList of the GED camera-pose model (host C++).
//
// Restates SRC/EpipoleList.{h,cpp} (SRC = source/Lib/CommonLib): epipoles in Q24 fixed point
// (EPIPOLE_PRECISION_FIXED, CommonDef.h:441) keyed by (curPOC, refPOC) with the -1 wildcards, an
// availability bit per entry, the three-step lookup, and the decoder's epipole predictor.  The
// context of the C-ABI owns one list (mm_get_epipole_list); standalone lists serve hosts that keep
// the decoder-side bookkeeping (DecLib.cpp:2048, 3136-3142) apart from a GPU context.
#pragma once
#include <array>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <map>
#include <utility>

#include "../../include/mm360.h"

namespace mmepi {

constexpr int EPIPOLE_PRECISION_FIXED = 24;  // CommonDef.h:441
using Q3 = std::array<int32_t, 3>;

// FloatingFixedConversion::fixedToFloating (Coordinate.cpp:70-78), TCoord = float
inline float fixed_to_floating(int32_t v, int precision) {
  return (float)(v >> precision) + (float)(v & ((1 << precision) - 1)) / (float)(1 << precision);
}
// FloatingFixedConversion::floatingToFixed (Coordinate.cpp:86-92): std::round (ties away), cast
inline int32_t floating_to_fixed(float f, int precision) {
  return (int32_t)std::round(f * (float)(1 << precision));
}

class EpipoleList {
 public:
  struct Entry {
    Q3 q{0, 0, 0};
    bool available = false;
  };

  // EpipoleList() adds the global (-1, -1) zero epipole, not available (EpipoleList.h:15-17)
  EpipoleList() { add({0, 0, 0}, -1, -1, false); }

  // addEpipole (EpipoleList.cpp:8-11): insert or replace; the caller converts to Q24
  void add(const Q3& q, int cur, int ref, bool make_available) {
    m_[{cur, ref}] = Entry{q, make_available};
    version_++;
  }

  // findEpipoleFixed (EpipoleList.cpp:19-36): (cur, ref), then (cur, -1), then (-1, -1), available
  // entries only; false where the reference CHECKs "No epipole for given (curPOC, refPOC)"
  bool find(int cur, int ref, Q3* out) const {
    const std::pair<int, int> keys[3] = {{cur, ref}, {cur, -1}, {-1, -1}};
    for (const auto& k : keys) {
      auto it = m_.find(k);
      if (it != m_.end() && it->second.available) {
        *out = it->second.q;
        return true;
      }
    }
    return false;
  }

  // hasEpipole (EpipoleList.cpp:82-89): the exact key, available
  bool has(int cur, int ref) const {
    auto it = m_.find({cur, ref});
    return it != m_.end() && it->second.available;
  }

  // makeAvailable (EpipoleList.cpp:91-99): every entry whose curPOC matches
  void make_available(int cur) {
    for (auto& kv : m_)
      if (kv.first.first == cur) kv.second.available = true;
    version_++;
  }

  // count() (EpipoleList.h:21-24): entries, not counting a zero global epipole
  int count() const {
    auto it = m_.find({-1, -1});
    const bool global_default = it != m_.end() && it->second.q == Q3{0, 0, 0};
    return (int)m_.size() - (global_default ? 1 : 0);
  }

  // derivePredictor (EpipoleList.cpp:38-80) followed by the decoder's floatingToFixed
  // (DecLib.cpp:3138).  Walks the available entries in key order keeping the two smallest
  // |curPOC - entry.curPOC| distances (strictly smaller replaces, as written); on a tie the
  // predictor is `predictors[0] + predictors[1] / 2` with C++ precedence (integer division of the
  // second only, truncating) -- kept exactly.  The fixed result goes through fixedToFloating and
  // back, as in the reference.  MM_ERR_NOEPIPOLE: global epipole unavailable (CHECK :42);
  // MM_ERR_ARG: the distance-order CHECK (:75).
  int derive_predictor(int cur, Q3* out) const {
    auto g = m_.find({-1, -1});
    if (g == m_.end() || !g->second.available) return MM_ERR_NOEPIPOLE;
    int dist[2] = {INT_MAX, INT_MAX};
    Q3 pred[2] = {g->second.q, g->second.q};
    for (const auto& kv : m_) {
      if (!kv.second.available) continue;
      const int d = std::abs(cur - kv.first.first);
      if (d < dist[0]) {
        dist[0] = d;
        pred[0] = kv.second.q;
      } else if (d < dist[1]) {
        dist[1] = d;
        pred[1] = kv.second.q;
      }
    }
    Q3 p;
    if (dist[0] == dist[1]) {
      for (int i = 0; i < 3; i++) p[i] = pred[0][i] + pred[1][i] / 2;
    } else {
      if (dist[0] > dist[1]) return MM_ERR_ARG;
      p = pred[0];
    }
    for (int i = 0; i < 3; i++)
      (*out)[i] = floating_to_fixed(fixed_to_floating(p[i], EPIPOLE_PRECISION_FIXED), EPIPOLE_PRECISION_FIXED);
    return MM_OK;
  }

  const std::map<std::pair<int, int>, Entry>& entries() const { return m_; }
  // bumped by every change (a device copy of the list is refreshed when it moves)
  unsigned long long version() const { return version_; }

 private:
  std::map<std::pair<int, int>, Entry> m_;
  unsigned long long version_ = 0;
};

}  // namespace mmepi
