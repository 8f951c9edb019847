/*
 * hd_math.h — host/device math shared by the gfx950 megakernel, the host scene lowering and the
 * CPU oracle.  Everything here is the arithmetic that decides a path's branches, so it must give
 * the SAME bits on x86-64 (g++/clang, SSE2) and on gfx950:
 *   - build with -ffp-contract=off everywhere (no FMA contraction), no fast-math;
 *   - f32 '/' and sqrt are IEEE correctly rounded on both sides (hipcc default);
 *   - transcendentals are NOT taken from glibc / ocml (their last bits differ): they are evaluated in
 *     f64 with only +,-,*,/,sqrt (all IEEE correctly rounded on both sides) and rounded once to f32,
 *     which also makes them correctly rounded in all but ~1e-8 of cases (KATs: tests/golden).
 *
 * Reference semantics restated here (paths relative to the reference repo):
 *   Vec3 = cgmath::Vector3<f32>  (src/math.rs:10): dot = (x*x'+y*y')+z*z', normalize = v*(1/|v|),
 *       cross as cgmath, Vec3/s divides each component.
 *   math.rs helpers: near_zero :42-45, reflect :47-49, refract :51-56, reflectance :58-62.
 *   rand 0.8.5 distributions: gen::<f32>() = (u32>>8)*2^-24; gen_range(lo..hi) for f32 =
 *       ((bits(0x3F800000|(u32>>9)) - 1) * (hi-lo) + lo), retried when it lands on hi.
 *   The reference RNG is rand::thread_rng() (ChaCha12, OS-seeded, no seed control).  It cannot be
 *   reproduced; this file substitutes xoshiro128** streams keyed by (seed, pixel, sample), which is
 *   what makes fixed-seed parity and 1/2/4/8-GPU bit-identity possible.
 */
#pragma once
#include <stdint.h>
#include <string.h>
#include <math.h>

#if defined(__HIP__)
#include <hip/hip_runtime.h>
#define HRT_HD __host__ __device__ inline
#else
#define HRT_HD inline
#endif

namespace hrt {

/* ------------------------------------------------------------------------------------------------
 * bit casts
 * ----------------------------------------------------------------------------------------------*/
HRT_HD uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
HRT_HD float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* RN(1 / x), the IEEE quotient 1.0f / x.  On the device, for x whose biased exponent lies in
 * [RCP_FAST_EXP_LO, RCP_FAST_EXP_HI], v_rcp_f32 followed by one fma Newton step, y + y (1 - x y): 3 instructions
 * instead of the ~11 of the IEEE division sequence.  That it is the IEEE quotient bit for bit was checked on the
 * MI355X for EVERY f32 of that range (tests/native/rcp_check.hip, profiles/r06_rcp_check.txt).  rcp_fast: x known
 * to lie in that range; rcp_rn: any x, the lanes outside the range (0, denormals, huge, inf, NaN) take the IEEE
 * division under a wave vote.  The host (oracle, lane simulator) divides. */
#ifndef HRT_RCP_FAST
#define HRT_RCP_FAST 1
#endif
constexpr uint32_t RCP_FAST_EXP_LO = 1u, RCP_FAST_EXP_HI = 252u; /* |x| in [2^-126, 2^126): every such x checked */
HRT_HD bool rcp_fast_domain(float x) { return ((f2u(x) >> 23) & 255u) - RCP_FAST_EXP_LO <= RCP_FAST_EXP_HI - RCP_FAST_EXP_LO; }
HRT_HD float rcp_fast(float x) {
#if defined(__HIP_DEVICE_COMPILE__) && HRT_RCP_FAST
  const float y = __builtin_amdgcn_rcpf(x);
  return fmaf(fmaf(-x, y, 1.0f), y, y);
#else
  return 1.0f / x;
#endif
}
HRT_HD float rcp_rn(float x) {
#if defined(__HIP_DEVICE_COMPILE__) && HRT_RCP_FAST
  float q = rcp_fast(x);
  const bool ok = rcp_fast_domain(x);
  if (__builtin_amdgcn_ballot_w64(!ok)) { /* a wave-uniform branch: the IEEE sequence only when a lane needs it */
    if (!ok) q = 1.0f / x;
  }
  return q;
#else
  return 1.0f / x;
#endif
}
HRT_HD uint64_t d2u(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }
HRT_HD double u2d(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }

/* ------------------------------------------------------------------------------------------------
 * Vec3 with cgmath operation order
 * ----------------------------------------------------------------------------------------------*/
struct Vec3 {
  float x, y, z;
  HRT_HD float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
  HRT_HD float& operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }
};
HRT_HD Vec3 v3(float x, float y, float z) { Vec3 r; r.x = x; r.y = y; r.z = z; return r; }
HRT_HD Vec3 operator+(Vec3 a, Vec3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
HRT_HD Vec3 operator-(Vec3 a, Vec3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
HRT_HD Vec3 operator-(Vec3 a) { return v3(-a.x, -a.y, -a.z); }
HRT_HD Vec3 operator*(float s, Vec3 a) { return v3(s * a.x, s * a.y, s * a.z); }
HRT_HD Vec3 operator*(Vec3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
HRT_HD Vec3 operator/(Vec3 a, float s) { return v3(a.x / s, a.y / s, a.z / s); }
HRT_HD Vec3 mul_elem(Vec3 a, Vec3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
HRT_HD float dot(Vec3 a, Vec3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
HRT_HD Vec3 cross(Vec3 a, Vec3 b) {
  return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
HRT_HD float magnitude(Vec3 a) { return sqrtf(dot(a, a)); }
HRT_HD Vec3 normalize(Vec3 a) { return a * (1.0f / magnitude(a)); }

/* math.rs:42-45 */
HRT_HD bool near_zero(Vec3 v) {
  const float s = 1e-8f;
  return (fabsf(v.x) < s) && (fabsf(v.y) < s) && (fabsf(v.z) < s);
}
/* math.rs:47-49: v - 2*dot(v,n)*n, i.e. (2*dot)*n */
HRT_HD Vec3 reflect(Vec3 v, Vec3 n) { return v - (2.0f * dot(v, n)) * n; }
/* math.rs:51-56 */
HRT_HD float min_rs(float a, float b) { return fminf(a, b); } /* Rust f32::min == IEEE minNum */
HRT_HD Vec3 refract(Vec3 uv, Vec3 n, float etai_over_etat) {
  float cos_theta = min_rs(dot(-uv, n), 1.0f);
  Vec3 r_out_perp = etai_over_etat * (uv + cos_theta * n);
  Vec3 r_out_parallel = (-sqrtf(fabsf(1.0f - dot(r_out_perp, r_out_perp)))) * n;
  return r_out_perp + r_out_parallel;
}

/* Rust saturating float->int casts (`as i32`, `as u32`).  On the device these are the gfx950 conversions
 * themselves: v_cvt_i32_f32 / v_cvt_u32_f32 truncate toward zero, clamp out-of-range values (infinities
 * included) to the type's range and turn NaN into 0 -- Rust's saturating semantics, one instruction instead of
 * the compiler's three nested range branches per conversion (the Perlin lattice indices: 3 per octave, 21 per
 * noise texture call).  tests/test_gpu_parity.py::test_device_float_to_int_casts holds them to the host's
 * branchy form bit for bit on every edge value (HRT_HW_CVT=0 keeps the branches on the device, for A/B).
 * sat_f2i32_cmp: the compare-and-select form everywhere (lane.h: the Perlin lattice over tables in global memory, where
 * the straight-line octave loop's longer live ranges cost Final's kernel 16 B more spills per lane). */
#ifndef HRT_HW_CVT
#define HRT_HW_CVT 1
#endif
HRT_HD int32_t sat_f2i32_cmp(float f) {
  if (!(f == f)) return 0;
  if (f >= 2147483648.0f) return 2147483647;
  if (f < -2147483648.0f) return (int32_t)(-2147483647 - 1);
  return (int32_t)f;
}
HRT_HD int32_t sat_f2i32(float f) {
#if defined(__HIP_DEVICE_COMPILE__) && HRT_HW_CVT
  int32_t r;
  asm("v_cvt_i32_f32 %0, %1" : "=v"(r) : "v"(f));
  return r;
#else
  return sat_f2i32_cmp(f);
#endif
}
HRT_HD uint32_t sat_f2u32(float f) {
#if defined(__HIP_DEVICE_COMPILE__) && HRT_HW_CVT
  uint32_t r;
  asm("v_cvt_u32_f32 %0, %1" : "=v"(r) : "v"(f));
  return r;
#else
  if (!(f == f) || f <= 0.0f) return 0u;
  if (f >= 4294967296.0f) return 4294967295u;
  return (uint32_t)f;
#endif
}

/* ------------------------------------------------------------------------------------------------
 * Deterministic f32 transcendentals, evaluated in f64 (see file header).
 * ----------------------------------------------------------------------------------------------*/
namespace detail {
/* pi/2 = P1 + P2 + P3, P1/P2 have 30 significant bits so n*P1, n*P2 are exact for |n| < 2^23 */
constexpr double P1 = 0x1.921fb54000000p+0;
constexpr double P2 = 0x1.10b4611800000p-30;
constexpr double P3 = 0x1.313198a2e0370p-61;
constexpr double TWO_OVER_PI = 0x1.45f306dc9c883p-1;
constexpr double D_PI = 0x1.921fb54442d18p+1;
constexpr double D_PIO2 = 0x1.921fb54442d18p+0;
constexpr double D_PIO4 = 0x1.921fb54442d18p-1;
constexpr double D_PIO8 = 0x1.921fb54442d18p-2;
constexpr double D_TAN_PIO8 = 0x1.a827999fcef32p-2;
constexpr double D_TAN_PIO16 = 0.198912367379658006911597622644676; /* threshold only */
constexpr double D_TAN_3PIO16 = 0.668178637919298919997757686523080; /* threshold only */
constexpr double D_LN2 = 0x1.62e42fefa39efp-1;
constexpr double D_SQRT2 = 0x1.6a09e667f3bcdp+0;

/* sin(r), cos(r) for |r| <= pi/4 (+eps): Taylor series, truncation error < 1e-21 */
HRT_HD double sin_poly(double r) {
  double z = r * r;
  double p = 0x1.71b8ef6dcf572p-66;
  p = p * z + -0x1.2f49b46814157p-57;
  p = p * z + 0x1.952c77030ad4ap-49;
  p = p * z + -0x1.ae7f3e733b81fp-41;
  p = p * z + 0x1.6124613a86d09p-33;
  p = p * z + -0x1.ae64567f544e4p-26;
  p = p * z + 0x1.71de3a556c734p-19;
  p = p * z + -0x1.a01a01a01a01ap-13;
  p = p * z + 0x1.1111111111111p-7;
  p = p * z + -0x1.5555555555555p-3;
  return r + (r * z) * p;
}
HRT_HD double cos_poly(double r) {
  double z = r * r;
  double p = -0x1.0ce396db7f853p-70;
  p = p * z + 0x1.e542ba4020225p-62;
  p = p * z + -0x1.6827863b97d97p-53;
  p = p * z + 0x1.ae7f3e733b81fp-45;
  p = p * z + -0x1.93974a8c07c9dp-37;
  p = p * z + 0x1.1eed8eff8d898p-29;
  p = p * z + -0x1.27e4fb7789f5cp-22;
  p = p * z + 0x1.a01a01a01a01ap-16;
  p = p * z + -0x1.6c16c16c16c17p-10;
  p = p * z + 0x1.5555555555555p-5;
  return 1.0 + z * (-0.5 + z * p);
}
/* round-half-even to integer without libm (exact for |v| < 2^52) */
HRT_HD double rint_d(double v) {
  const double big = 4503599627370496.0; /* 2^52 */
  if (!(v == v)) return v;
  if (v >= 0.0) { if (v >= big) return v; return (v + big) - big; }
  if (v <= -big) return v;
  return (v - big) + big;
}
/* x reduced by pi/2: returns r in [-pi/4, pi/4] (approximately) and quadrant q (mod 4) */
HRT_HD double reduce_pio2(double x, int* q) {
  double n = rint_d(x * TWO_OVER_PI);
  double r = ((x - n * P1) - n * P2) - n * P3;
  /* quadrant = n mod 4 (n is an integer-valued double, |n| < 2^53) */
  double n4 = n - 4.0 * rint_d(n * 0.25);
  if (n4 < 0.0) n4 += 4.0;
  *q = (int)n4 & 3;
  return r;
}
/* atan(a) for 0 <= a <= 1 */
HRT_HD double atan01(double a) {
  double base = 0.0, t = a;
  if (a > D_TAN_3PIO16) { /* c = tan(pi/4) = 1 */
    t = (a - 1.0) / (a + 1.0);
    base = D_PIO4;
  } else if (a > D_TAN_PIO16) { /* c = tan(pi/8) */
    t = (a - D_TAN_PIO8) / (1.0 + a * D_TAN_PIO8);
    base = D_PIO8;
  }
  /* |t| <= tan(pi/16) ~ 0.1989: alternating series to t^27 */
  double z = t * t;
  double p = 1.0 / 27.0;
  p = p * z - 1.0 / 25.0;
  p = p * z + 1.0 / 23.0;
  p = p * z - 1.0 / 21.0;
  p = p * z + 1.0 / 19.0;
  p = p * z - 1.0 / 17.0;
  p = p * z + 1.0 / 15.0;
  p = p * z - 1.0 / 13.0;
  p = p * z + 1.0 / 11.0;
  p = p * z - 1.0 / 9.0;
  p = p * z + 1.0 / 7.0;
  p = p * z - 1.0 / 5.0;
  p = p * z + 1.0 / 3.0;
  return base + (t - (t * z) * p);
}
HRT_HD double atan2_d(double y, double x) {
  if (!(x == x) || !(y == y)) return x + y; /* NaN */
  const double inf = u2d(0x7ff0000000000000ull);
  bool xneg = (d2u(x) >> 63) != 0, yneg = (d2u(y) >> 63) != 0;
  double ax = xneg ? -x : x, ay = yneg ? -y : y;
  double r;
  if (ay == 0.0) {
    r = xneg ? D_PI : 0.0;
  } else if (ax == 0.0) {
    r = D_PIO2;
  } else if (ax == inf && ay == inf) {
    r = xneg ? 3.0 * D_PIO4 : D_PIO4;
  } else if (ax == inf) {
    r = xneg ? D_PI : 0.0;
  } else if (ay == inf) {
    r = D_PIO2;
  } else {
    if (ay <= ax) r = atan01(ay / ax);
    else r = D_PIO2 - atan01(ax / ay);
    if (xneg) r = D_PI - r;
  }
  return yneg ? -r : r;
}
HRT_HD double log_d(double x) {
  if (!(x == x)) return x;
  if (x < 0.0) return u2d(0x7ff8000000000000ull);
  if (x == 0.0) return -u2d(0x7ff0000000000000ull);
  uint64_t b = d2u(x);
  int e = (int)((b >> 52) & 0x7ff);
  if (e == 0x7ff) return x; /* +inf */
  /* inputs come from f32, so they are normal doubles */
  e -= 1023;
  double m = u2d((b & 0x000fffffffffffffull) | 0x3ff0000000000000ull); /* [1,2) */
  if (m > D_SQRT2) { m = m * 0.5; e += 1; }
  double s = (m - 1.0) / (m + 1.0);
  double z = s * s;
  double p = 1.0 / 23.0;
  p = p * z + 1.0 / 21.0;
  p = p * z + 1.0 / 19.0;
  p = p * z + 1.0 / 17.0;
  p = p * z + 1.0 / 15.0;
  p = p * z + 1.0 / 13.0;
  p = p * z + 1.0 / 11.0;
  p = p * z + 1.0 / 9.0;
  p = p * z + 1.0 / 7.0;
  p = p * z + 1.0 / 5.0;
  p = p * z + 1.0 / 3.0;
  double lnm = 2.0 * (s + (s * z) * p);
  return (double)e * D_LN2 + lnm;
}
}  // namespace detail

/* f32 sin, correctly rounded except in ~1e-8 of cases; exact reduction for |x| < 2^23 * pi/2 */
HRT_HD float sin_f(float xf) {
  double x = (double)xf;
  if (!(x == x) || fabs(x) == u2d(0x7ff0000000000000ull)) return xf - xf; /* NaN */
  if (xf == 0.0f) return xf;                                             /* keeps -0 */
  int q;
  double r = detail::reduce_pio2(x, &q);
  double v;
  switch (q) {
    case 0: v = detail::sin_poly(r); break;
    case 1: v = detail::cos_poly(r); break;
    case 2: v = -detail::sin_poly(r); break;
    default: v = -detail::cos_poly(r); break;
  }
  return (float)v;
}
HRT_HD float cos_f(float xf) {
  double x = (double)xf;
  if (!(x == x) || fabs(x) == u2d(0x7ff0000000000000ull)) return xf - xf;
  int q;
  double r = detail::reduce_pio2(x, &q);
  double v;
  switch (q) {
    case 0: v = detail::cos_poly(r); break;
    case 1: v = -detail::sin_poly(r); break;
    case 2: v = -detail::cos_poly(r); break;
    default: v = detail::sin_poly(r); break;
  }
  return (float)v;
}
HRT_HD float tan_f(float xf) {
  double x = (double)xf;
  if (!(x == x) || fabs(x) == u2d(0x7ff0000000000000ull)) return xf - xf;
  if (xf == 0.0f) return xf;
  int q;
  double r = detail::reduce_pio2(x, &q);
  double s = detail::sin_poly(r), c = detail::cos_poly(r);
  return (float)((q & 1) ? (-c / s) : (s / c));
}
HRT_HD float atan2_f(float y, float x) { return (float)detail::atan2_d((double)y, (double)x); }
/* acos via atan2(sqrt((1-x)(1+x)), x); the product is exact in f64 for f32 x; |x|>1 -> NaN */
HRT_HD float acos_f(float xf) {
  double x = (double)xf;
  if (!(x == x)) return xf;
  double s2 = (1.0 - x) * (1.0 + x);
  if (s2 < 0.0) return u2f(0x7fc00000u);
  return (float)detail::atan2_d(sqrt(s2), x);
}
HRT_HD float ln_f(float x) { return (float)detail::log_d((double)x); }
/* powf(x, 5.0) as used by math.rs:61: x^5 in f64 (x^2 exact), rounded once */
HRT_HD float pow5_f(float xf) {
  double x = (double)xf;
  double x2 = x * x;
  double x4 = x2 * x2;
  return (float)(x4 * x);
}

/* math.rs:58-62 Schlick */
HRT_HD float reflectance(float cosine, float refraction_index) {
  float r0 = (1.0f - refraction_index) / (1.0f + refraction_index);
  r0 = r0 * r0;
  return r0 + (1.0f - r0) * pow5_f(1.0f - cosine);
}

/* Rust f32 constants (std::f32::consts) */
constexpr float PI_F = 3.14159265358979323846264338327950288f;
constexpr float E_F = 2.71828182845904523536028747135266250f;

/* ------------------------------------------------------------------------------------------------
 * RNG: splitmix64 keying + xoshiro128** streams + rand 0.8.5 distribution transforms
 * ----------------------------------------------------------------------------------------------*/
HRT_HD uint64_t mix64(uint64_t z) { /* splitmix64 finaliser (a bijection) */
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
HRT_HD uint64_t splitmix64_next(uint64_t* s) {
  *s += 0x9E3779B97F4A7C15ull;
  return mix64(*s);
}
HRT_HD uint32_t rotl32(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }

struct Rng {
  uint32_t s0, s1, s2, s3;
  HRT_HD uint32_t next_u32() {
    uint32_t result = rotl32(s1 * 5u, 7) * 9u;
    uint32_t t = s1 << 9;
    s2 ^= s0;
    s3 ^= s1;
    s1 ^= s2;
    s0 ^= s3;
    s2 ^= t;
    s3 = rotl32(s3, 11);
    return result;
  }
  /* rand_core next_u64_via_u32: low word first */
  HRT_HD uint64_t next_u64() {
    uint64_t lo = next_u32();
    uint64_t hi = next_u32();
    return (hi << 32) | lo;
  }
  /* rand 0.8 Standard for f32: 24 random bits scaled by 2^-24 */
  HRT_HD float gen_f32() { return (float)(next_u32() >> 8) * 5.9604644775390625e-08f; }
  /* rand 0.8 UniformFloat::<f32>::sample_single(lo, hi) */
  HRT_HD float gen_range_f32(float lo, float hi) {
    float scale = hi - lo;
    for (;;) {
      float v12 = u2f(0x3F800000u | (next_u32() >> 9));
      float v01 = v12 - 1.0f;
      float res = v01 * scale + lo;
      if (res < hi) return res;
      /* edge case in rand: shrink scale by one ulp and retry */
      scale = u2f(f2u(scale) - 1u);
    }
  }
};

HRT_HD Rng rng_from_key(uint64_t key) {
  uint64_t s = key;
  uint64_t a = splitmix64_next(&s);
  uint64_t b = splitmix64_next(&s);
  Rng r;
  r.s0 = (uint32_t)a;
  r.s1 = (uint32_t)(a >> 32);
  r.s2 = (uint32_t)b;
  r.s3 = (uint32_t)(b >> 32);
  if ((r.s0 | r.s1 | r.s2 | r.s3) == 0u) r.s0 = 1u; /* xoshiro state must be non-zero */
  return r;
}
/* Per-path key: unique per (seed, global pixel index, sample index). */
HRT_HD uint64_t path_key(uint64_t seed, uint32_t pixel, uint32_t sample) {
  return mix64(mix64(seed) ^ (((uint64_t)pixel << 32) | (uint64_t)sample));
}
/* ConstantMedium draw (constant_medium.rs:58-59), keyed by (path, segment, medium id) so that it does
 * not depend on the order in which a traversal happens to evaluate the medium. */
HRT_HD float medium_xi(uint64_t pkey, uint32_t segment, uint32_t medium_id) {
  uint64_t k = mix64(pkey ^ mix64(0xC2B2AE3D27D4EB4Full ^ (((uint64_t)segment << 32) | medium_id)));
  return (float)((uint32_t)(k >> 32) >> 8) * 5.9604644775390625e-08f;
}

/* Scene-builder stream: replaces the thread_rng of the application.rs builders. */
HRT_HD Rng scene_rng(uint64_t seed) { return rng_from_key(mix64(seed ^ 0x5343454E45ull)); }

/* rand 0.8.5 UniformInt<usize/u64>::sample_single(lo..hi): widening multiply + zone rejection
 * (host only: used by the Sattolo shuffle of perlin_noise.rs:58-64). */
inline uint64_t gen_range_u64(Rng& r, uint64_t lo, uint64_t hi) {
  uint64_t range = hi - lo; /* == (hi - 1) - lo + 1 */
  if (range == 0) return r.next_u64();
  uint64_t zone = (range << __builtin_clzll(range)) - 1u;
  for (;;) {
    uint64_t v = r.next_u64();
    __uint128_t m = (__uint128_t)v * (__uint128_t)range;
    uint64_t hi_w = (uint64_t)(m >> 64), lo_w = (uint64_t)m;
    if (lo_w <= zone) return lo + hi_w;
  }
}

/* gen_range_f32(-1.0, 1.0) without its retry loop, same bits: there v01 * 2 - 1 <= 1 - 2^-22 < hi, so
 * rand's retry never fires; and v01 * 2 + (-1) is RN(2 v12 - 3) (v12 - 1 and the doubling are exact),
 * which one fma computes.  Saves a loop (and its exec-mask juggling) per draw in the rejection loops. */
HRT_HD float gen_signed_unit(Rng& r) {
  const float v12 = u2f(0x3F800000u | (r.next_u32() >> 9));
  return fmaf(v12, 2.0f, -3.0f);
}

/* math.rs:16-30 random_in_unit_sphere: rejection on Uniform(-1,1)^3 */
HRT_HD Vec3 random_in_unit_sphere(Rng& r) {
#if HRT_EXP_NOREJECT /* timing experiment only (wrong draws): the price of the rejection loops */
  { float x = gen_signed_unit(r), y = gen_signed_unit(r), z = gen_signed_unit(r); return v3(0.5f * x, 0.5f * y, 0.5f * z); }
#endif
  for (;;) {
    float x = gen_signed_unit(r);
    float y = gen_signed_unit(r);
    float z = gen_signed_unit(r);
    Vec3 p = v3(x, y, z);
    if (dot(p, p) < 1.0f) return p;
  }
}
/* math.rs:12-14 */
HRT_HD Vec3 random_unit_vector(Rng& r) { return normalize(random_in_unit_sphere(r)); }
/* math.rs:32-40 */
HRT_HD Vec3 random_in_unit_disk(Rng& r) {
#if HRT_EXP_NOREJECT
  { float x = gen_signed_unit(r), y = gen_signed_unit(r); return v3(0.5f * x, 0.5f * y, 0.0f); }
#endif
  for (;;) {
    float x = gen_signed_unit(r);
    float y = gen_signed_unit(r);
    Vec3 p = v3(x, y, 0.0f);
    if (dot(p, p) < 1.0f) return p;
  }
}

}  // namespace hrt
