/* Exhaustive-style check of the kernel's division by dot(d, d) (render.hip div_rn): the fma-corrected
 * quotient with a per-ray RN(1/a) must equal IEEE x / a bit for bit wherever the fast path is taken, and
 * the kernel's cheaper domain test (a in [2^-49, 2^49], |q0| in [2^-50, 2^50]) may only select cases inside
 * the proven domain.
 * Usage: div_rn_check <n> <seed> <emin> <emax>   prints "<fast-path cases> <mismatches>".
 *        div_rn_check camera <seed>               the camera domain of start_sample (lane.h): EVERY
 *        divisor a = W - 1 in [1, 65534] with x = RN(px + g), px in [0, a] (edges and random), g the
 *        gen_f32 values 0, 2^-24, 0.5, 1 - 2^-24 and random multiples of 2^-24; the bare core
 *        fmaf(fmaf(-q0, a, x), y, q0) with y = RN(1/a), q0 = RN(x y) against IEEE x / a. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static float f(uint32_t u) { float x; memcpy(&x, &u, 4); return x; }
static uint32_t u(float x) { uint32_t v; memcpy(&v, &x, 4); return v; }

static int camera(uint64_t s) {
  long cases = 0, bad = 0;
  for (uint32_t ai = 1; ai <= 65534; ai++) {
    const float a = (float)ai;
    volatile float yv = 1.0f / a;
    const float y = yv;
    uint32_t pxs[8] = {0, 1, ai / 2, ai - 1, ai, 0, 0, 0};
    for (int k = 5; k < 8; k++) {
      s ^= s << 13; s ^= s >> 7; s ^= s << 17;
      pxs[k] = (uint32_t)(s % (uint64_t)(ai + 1));
    }
    for (int k = 0; k < 8; k++) {
      float gs[8] = {0.0f, 0x1p-24f, 0.5f, 1.0f - 0x1p-24f, 0, 0, 0, 0};
      for (int j = 4; j < 8; j++) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        gs[j] = (float)(uint32_t)(s >> 40) * 0x1p-24f; /* gen_f32: (u32 >> 8) * 2^-24 */
      }
      for (int j = 0; j < 8; j++) {
        volatile float xv = (float)pxs[k] + gs[j];
        const float x = xv;
        volatile float qv = x / a;
        const float q0 = x * y;
        const float got = fmaf(fmaf(-q0, a, x), y, q0);
        cases++;
        if (u(got) != u(qv)) bad++;
      }
    }
  }
  printf("%ld %ld\n", cases, bad);
  return 0;
}

int main(int argc, char** argv) {
  if (argc >= 3 && strcmp(argv[1], "camera") == 0) return camera(strtoull(argv[2], 0, 10) * 0x9E3779B97F4A7C15ull + 1);
  if (argc < 5) return 2;
  long n = atol(argv[1]);
  uint64_t s = strtoull(argv[2], 0, 10) * 0x9E3779B97F4A7C15ull + 1;
  int emin = atoi(argv[3]), emax = atoi(argv[4]);
  long fast = 0, bad = 0;
  for (long i = 0; i < n; i++) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    uint64_t r = s;
    int ea = emin + (int)((r >> 40) % (uint64_t)(emax - emin + 1));
    int ex = emin + (int)((r >> 50) % (uint64_t)(emax - emin + 1));
    uint32_t ma = (uint32_t)r & 0x7fffff, mx = (uint32_t)(r >> 23) & 0x7fffff;
    if ((i & 7) == 0) ma = 0x7fffff;  /* significands of all ones: the hard reciprocals */
    if ((i & 15) == 1) mx = 0x7fffff;
    if ((i & 31) == 2) ma = 0;
    float a = f(((uint32_t)(ea + 127) << 23) | ma);
    float x = f(((uint32_t)(ex + 127) << 23) | mx | (uint32_t)((r >> 63) << 31));
    volatile float yv = 1.0f / a, qv = x / a;
    float y = yv, q = qv;
    float q0 = x * y;
    float ax = fabsf(x), aq = fabsf(q0);
    int proven = ax >= 0x1p-100f && ax <= 0x1p100f && aq >= 0x1p-100f && aq <= 0x1p100f && a >= 0x1p-100f && a <= 0x1p100f;
    /* the kernel's split test (lane.h div_rn / div_rn_y) must select a subset of the proven domain */
    int kernel = a >= 0x1p-49f && a <= 0x1p49f && aq >= 0x1p-50f && aq <= 0x1p50f;
    if (kernel && !proven) bad++;
    if (!proven) continue;
    fast++;
    float got = fmaf(fmaf(-q0, a, x), y, q0);
    if (u(got) != u(q)) bad++;
  }
  printf("%ld %ld\n", fast, bad);
  return 0;
}
