/*
 * walk_box.h — host-side encoding of a walk-stream box (layout.h: node part C, E), shared by the stream
 * builder (scene.cpp walk_place_and_write) and the culling property test (tests/native/lane_sim.hip).
 */
#pragma once
#include <algorithm>
#include <cmath>

namespace hrt {
namespace walkbox {

/* centre / half-extent of [mn, mx], E rounded up so that [C - E, C + E] holds [mn, mx] exactly */
inline void ce_of(const float* mn, const float* mx, float* C, float* E) {
  for (int k = 0; k < 3; k++) {
    const double lo = mn[k], hi = mx[k];
    const float c = (float)((lo + hi) * 0.5);
    double e = std::max((double)c - lo, hi - (double)c);
    e += e * 0x1p-50; /* the double differences are exact unless the exponents are far apart */
    float ef = (float)e;
    if ((double)ef < e) ef = nextafterf(ef, 3.40282347e+38f);
    C[k] = c;
    E[k] = ef;
  }
}

/* layout.h CE_FLOOR: C, E as ce_of, with max_k E_k raised to at least 2^-12 max_k |C_k| when it is smaller
 * (only boxes far smaller than their distance from the world origin: none in the reference scenes).
 * fmn, fmx = a float box holding [C - E, C + E] (the box itself when nothing was raised), for the
 * enclosing nodes' boxes, so each node's inflated box still holds its children's.  Returns whether E
 * was raised. */
inline bool ce_floored(const float* mn, const float* mx, float* C, float* E, float* fmn, float* fmx) {
  ce_of(mn, mx, C, E);
  const float cm = std::max(std::max(fabsf(C[0]), fabsf(C[1])), fabsf(C[2]));
  const float f = ldexpf(cm, -12); /* exact: a power-of-two scaling */
  if (!(std::max(std::max(E[0], E[1]), E[2]) < f)) {
    for (int k = 0; k < 3; k++) {
      fmn[k] = mn[k];
      fmx[k] = mx[k];
    }
    return false;
  }
  for (int k = 0; k < 3; k++) {
    E[k] = std::max(E[k], f);
    const double l = (double)C[k] - E[k], h = (double)C[k] + E[k];
    float lo = (float)l, hi = (float)h;
    if ((double)lo > l) lo = nextafterf(lo, -3.40282347e+38f);
    if ((double)hi < h) hi = nextafterf(hi, 3.40282347e+38f);
    fmn[k] = std::min(lo, mn[k]);
    fmx[k] = std::max(hi, mx[k]);
  }
  return true;
}

}  // namespace walkbox
}  // namespace hrt
