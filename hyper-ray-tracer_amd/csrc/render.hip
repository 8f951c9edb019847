/*
 * render.hip — the gfx950 path-tracing megakernel and its device runtime (scene upload, launches).
 *
 * Replaces the per-tile task body of Application::render (src/application.rs:415-473) and
 * ray_color (:477-495) of SkillerRaptor/hyper-ray-tracer, including everything they reach through
 * dyn Hittable / Material / Texture.  One persistent launch renders a whole tile set:
 *
 *   - each LANE owns one pixel at a time and runs its spp samples back to back (the reference's
 *     sample loop, :443-449, so the per-pixel sum keeps the reference's order); when its pixel is
 *     done it takes the next one from a global work counter, claimed once per wave with a ballot +
 *     one atomicAdd (no lane idles while work remains);
 *   - every iteration of the wave loop advances every busy lane by exactly one ray segment
 *     (= one world.hit call): lanes whose path ended start their next sample in the same iteration;
 *   - the world is the pre-order node stream of layout.h, walked stackless with skip links in the
 *     reference's left-then-right order with the shrinking t_max, so closest hits, tie-breaks and
 *     medium evaluation agree with the recursive BvhNode::hit;
 *   - the hit record (point/normal/uv/front_face) is built once per segment for the winning
 *     primitive only, replaying the enclosing Translation/Rotation chain exactly as the reference
 *     recursion does; (u, v) are evaluated only when the material's texture reads them;
 *   - randomness: per-(pixel, sample) xoshiro128** streams (hd_math.h) drawn in the reference's
 *     order; ConstantMedium draws come from a (path, segment, medium) keyed sub-stream.
 * No MFMA: this is branchy 3-vector math.  All arithmetic on the branch-deciding path is shared with
 * the CPU oracle through hd_math.h and compiled with -ffp-contract=off.
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "scene_internal.h"

using namespace hrt;
namespace G = hrt::gpu;

namespace {

/* ------------------------------------------------------------------ kernel parameters */
struct KParams {
  const G::Node* nodes;
  const G::Prim* prims;
  const G::Inst* insts;
  const G::Medium* media;
  const G::Mat* mats;
  const G::Tex* texs;
  const G::Perlin* perlin;
  const uint8_t* images;
  uint32_t main_end;
  float ln_e;
  /* camera (camera.rs:16-31 after resize) */
  Vec3 cam_origin, cam_llc, cam_h, cam_v, cam_u, cam_vv;
  float lens_radius, time0, time1;
  /* render */
  uint32_t W, H, spp, max_depth, sample_offset;
  float t_min;
  Vec3 background;
  uint64_t seed;
  /* work */
  const G::TileDev* tiles;
  uint32_t n_tiles;
  uint32_t total_work;
  float4* out;
  uint32_t* counter;
  unsigned long long* stats; /* segments, samples, pixels, then (COUNT builds) nodes, prims, tex */
  /* sample chunks: a work item is (pixel, chunk of `chunk` consecutive samples) */
  uint32_t chunk, n_chunks, n_out;
  uint32_t n_prims;
  uint32_t n_nodes;    /* node-stream entries to stage in LDS */
  uint32_t stream_len; /* FAST: length of one octant stream */
  uint32_t postpone;   /* BASIC kernel: lanes that must have finished their walk before a wave shades */
  uint32_t motion_uniform; /* every moving sphere has time0 = motion_t0, time1 - time0 = motion_span */
  float motion_t0, motion_span;
  float4* partial; /* [n_chunks][n_out] chunk sums (n_chunks > 1) */
};

/* per-lane work counters of the instrumented (COUNT) instantiation */
struct Counts {
  uint32_t nodes, prims, tex;
  uint32_t walk_slots, shade_slots; /* lane slots of wave iterations: walk (node) loop, shading passes */
  uint32_t prim_slots;              /* lane slots of wave executions of the primitive block */
};

/* COUNT builds of the sphere-scene kernel: shader-clock cycles per wave phase (s_memtime stamps,
 * uniform per wave): [0] claim + sample start, [1] walk, [2] shading */
struct PhaseClock {
  unsigned long long cyc[3];
  unsigned long long last;
};

__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
  return v;
}

struct TRay {
  Vec3 o, d, inv;
  float time;
  float dd;  /* dot(d, d): sphere.rs:42 `a`, constant for the ray */
  float rdd; /* RN(1 / dd), for div_dd */
  float tau; /* (time - time0) / (time1 - time0) of the scene's moving spheres (uniform motion only) */
};

/* x / r.dd correctly rounded (bit-identical to IEEE division) in 3 instructions instead of the
 * ~11 of the general sequence: with y = RN(1/a), q0 = RN(x*y) is within one ulp of x/a, the
 * residual x - q0*a is exact in an fma, and RN(q0 + residual*y) is RN(x/a) (Markstein's theorem;
 * no under/overflow anywhere while |x|, |q0|, a lie in [2^-100, 2^100]).  Zero, NaN, inf and
 * extreme exponents take the IEEE sequence.  tests/test_fast_division.py checks 6e7 cases on the host
 * and 4e6 on the device (3e9 more were checked while writing it). */
__device__ __forceinline__ float div_rn(float x, float a, float y) {
  const float q0 = x * y;
  const float q = fmaf(fmaf(-q0, a, x), y, q0);
  const float ax = fabsf(x), aq = fabsf(q0);
  const bool fast = ax >= 0x1p-100f && ax <= 0x1p100f && aq >= 0x1p-100f && aq <= 0x1p100f &&
                    a >= 0x1p-100f && a <= 0x1p100f;
  return fast ? q : x / a;
}

/* a new origin/direction; the ray keeps its time */
__device__ __forceinline__ void set_dir(TRay& r, Vec3 o, Vec3 d) {
  r.o = o;
  r.d = d;
  /* aabb.rs:22 computes 1/d per call; the value is the same every time */
  r.inv = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  r.dd = dot(d, d);
  r.rdd = 1.0f / r.dd;
}

__device__ __forceinline__ void set_time(TRay& r, float time, const KParams& P) {
  r.time = time;
  /* moving_sphere.rs:55-58: identical for every moving sphere when they share time0/time1 */
  r.tau = P.motion_uniform ? (time - P.motion_t0) / P.motion_span : 0.0f;
}

__device__ __forceinline__ void set_ray(TRay& r, Vec3 o, Vec3 d, float time, const KParams& P) {
  set_dir(r, o, d);
  set_time(r, time, P);
}

__device__ __forceinline__ float4 ld4(const void* p) { return *reinterpret_cast<const float4*>(p); }

/* aabb.rs:20-47 (CULL_REFERENCE), its narrowed form (CULL_SLAB), or CULL_EXACT: the reference test
 * AND an inflated slab test that only rejects boxes no accepted hit can come from (layout.h).
 * `if t0 > t_min {t0} else {t_min}` (aabb.rs:30-35) is fmaxf(t0, t_min): in IEEE mode v_max_f32
 * returns the non-NaN operand exactly as the comparison form does (a NaN t0 leaves t_min), and the
 * forms differ at most in the sign of a zero, which the `t_max <= t_min` test (:36) cannot see. */
template <int CULL>
__device__ __forceinline__ bool box_hit(const float4& a, const float4& b, const TRay& r, float tmin,
                                        float tmax, bool ref_only = false) {
  const float mn[3] = {a.x, a.y, a.z}, mx[3] = {b.x, b.y, b.z};
  const float o[3] = {r.o.x, r.o.y, r.o.z}, inv[3] = {r.inv.x, r.inv.y, r.inv.z};
  float dmn[3], dmx[3];
#pragma unroll
  for (int k = 0; k < 3; k++) {
    dmn[k] = mn[k] - o[k];
    dmx[k] = mx[k] - o[k];
  }
  float ts[3], te[3];
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const float t0 = dmn[k] * inv[k], t1 = dmx[k] * inv[k];
    const bool neg = inv[k] < 0.0f; /* aabb.rs:28-29 swap */
    ts[k] = neg ? t1 : t0;
    te[k] = neg ? t0 : t1;
  }
  if (CULL == G::CULL_SLAB) {
    const float lo = fmaxf(fmaxf(fmaxf(ts[0], tmin), ts[1]), ts[2]);
    const float hi = fminf(fminf(fminf(te[0], tmax), te[1]), te[2]);
    return !(hi <= lo);
  }
  bool ok = true; /* the reference: each axis on its own against [t_min, t_max] */
#pragma unroll
  for (int k = 0; k < 3; k++) ok = ok & !(fminf(te[k], tmax) <= fmaxf(ts[k], tmin));
  if (CULL == G::CULL_REFERENCE) return ok;
  /* CULL_EXACT: the slab interval widened by margin(box) / |d_k| per axis */
  float dist = 0.0f;
#pragma unroll
  for (int k = 0; k < 3; k++) dist = fmaxf(dist, fmaxf(fabsf(dmn[k]), fabsf(dmx[k])));
  const float margin = G::EXACT_MARGIN * dist;
  float lo = tmin, hi = tmax;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const float w = margin * fabsf(inv[k]);
    lo = fmaxf(lo, ts[k] - w);
    hi = fminf(hi, te[k] + w);
  }
  return ok & (ref_only | !(hi < lo));
}

/* sphere.rs:38-55 / moving_sphere.rs:61-78: the accepted root only */
__device__ __forceinline__ bool sphere_root(const G::Prim* pp, uint32_t kind, const TRay& r, float tmin,
                                            float tmax, float& root, bool motion_uniform) {
  float4 p0 = ld4(pp->p0);
  Vec3 c = v3(p0.x, p0.y, p0.z);
  if (kind == G::P_MOVING) {
    float4 p1 = ld4(pp->p1);
    const float f = motion_uniform ? r.tau : (r.time - p1.w) / pp->p2[0];
    c = c + f * v3(p1.x, p1.y, p1.z);
  }
  Vec3 oc = r.o - c;
  float a = r.dd;
  float half_b = dot(oc, r.d);
  float cc = dot(oc, oc) - p0.w * p0.w;
  float disc = half_b * half_b - a * cc;
  if (disc < 0.0f) return false;
  float sq = sqrtf(disc);
  float t = div_rn(-half_b - sq, a, r.rdd);
  if (t < tmin || tmax < t) {
    t = div_rn(-half_b + sq, a, r.rdd);
    if (t < tmin || tmax < t) return false;
  }
  root = t;
  return true;
}

__device__ __forceinline__ void plane_axes(uint32_t plane, int& k, int& a, int& b) {
  /* rect.rs:55-59 */
  if (plane == HRT_PLANE_XY) { k = 2; a = 0; b = 1; }
  else if (plane == HRT_PLANE_YZ) { k = 0; a = 1; b = 2; }
  else { k = 1; a = 2; b = 0; }
}

/* rect.rs:53-68 */
__device__ __forceinline__ bool rect_t(const G::Prim* pp, uint32_t plane, const TRay& r, float tmin,
                                       float tmax, float& tout) {
  int k, a, b;
  plane_axes(plane, k, a, b);
  float4 p0 = ld4(pp->p0);
  float kk = pp->p1[0];
  float t = (kk - r.o[k]) / r.d[k];
  if (t < tmin || t > tmax) return false;
  float av = r.o[a] + t * r.d[a];
  float bv = r.o[b] + t * r.d[b];
  if (av < p0.x || av > p0.y || bv < p0.z || bv > p0.w) return false;
  tout = t;
  return true;
}

/* translation.rs:26-30 and rotation.rs:104-117: the ray handed to the child */
__device__ __forceinline__ void inst_ray(const G::Inst& in, Vec3& o, Vec3& d) {
  if (in.kind == G::I_TRANSLATE) {
    o = o - v3(in.d[0], in.d[1], in.d[2]);
    return;
  }
  int a = (int)(in.axis + 1) % 3, b = (int)(in.axis + 2) % 3;
  float s = in.sin_t, c = in.cos_t;
  Vec3 no = o, nd = d;
  no[a] = c * o[a] + s * o[b];
  no[b] = -s * o[a] + c * o[b];
  nd[a] = c * d[a] + s * d[b];
  nd[b] = -s * d[a] + c * d[b];
  o = no;
  d = nd;
}

struct PathKey {
  uint64_t pkey;
  uint32_t segment;
};

/* The world walk.  Closest hit over [begin, end) of the node stream with t in [tmin, closest]:
 * `winner` = node index of the accepted leaf (NONE if nothing).  MEDIA: ConstantMedium nodes are
 * evaluated (their boundary walks are nested calls with MEDIA = false). */
template <int CULL, bool FULL, bool MEDIA, bool COUNT, bool FAST = false>
__device__ void trace(const KParams& P, const G::Node* __restrict__ nodes, const G::Prim* __restrict__ prims,
                      uint32_t begin, uint32_t end, Vec3 o, Vec3 d, float time, float tmin, float& closest,
                      uint32_t& winner, const PathKey& pk, Counts& cn) {
  TRay r;
  set_ray(r, o, d, time, P);
  if constexpr (FAST) { /* the stream whose near-child order matches the ray's direction octant */
    const uint32_t oct = (d.x < 0.0f ? 1u : 0u) | (d.y < 0.0f ? 2u : 0u) | (d.z < 0.0f ? 4u : 0u);
    begin = oct * P.stream_len;
    end = begin + P.stream_len;
  }
  Vec3 so[G::MAX_INST_DEPTH], sd[G::MAX_INST_DEPTH];
  int sp = 0;
  uint32_t i = begin;
  while (i < end) {
    const G::Node* np = nodes + i;
    const float4 a = ld4(np->mn);
    const float4 b = ld4(np->mx);
    const uint32_t kp = __float_as_uint(b.w);
    const uint32_t kind = (kp >> 24) & G::KIND_MASK;
    const bool ref_only = (kp & G::NODE_REF_ONLY) != 0;
    const uint32_t payload = kp & 0xFFFFFFu;
    const uint32_t here = i;
    if constexpr (COUNT) cn.nodes++;
    if constexpr (FAST) {
      bool pass = box_hit<CULL>(a, b, r, tmin, closest);
      if (kind == G::K_BOX) {
        i = pass ? i + 1 : __float_as_uint(a.w);
        continue;
      }
      i++;
      if (!pass) continue;
      /* K_BOX_LEAF: up to LEAF_MAX primitives, tested in order */
      const uint32_t start = payload & 0x1FFFFFu, cnt = (payload >> 21) + 1u;
      for (uint32_t k = 0; k < cnt; k++) {
        const G::Prim* pp = prims + start + k;
        if constexpr (COUNT) cn.prims++;
        float t;
        if (sphere_root(pp, pp->km & 3u, r, tmin, closest, t, P.motion_uniform != 0)) {
          closest = t;
          winner = start + k;
        }
      }
      continue;
    }
    if (kind <= G::K_BOX_PRIM) {
      bool pass = box_hit<CULL>(a, b, r, tmin, closest, ref_only);
      if (kind == G::K_BOX) {
        i = pass ? i + 1 : __float_as_uint(a.w);
        continue;
      }
      i++;
      if (!pass) continue;
    } else if (kind == G::K_PRIM) {
      i++;
    } else {
      if constexpr (FULL) {
        i++;
        if (kind == G::K_INST_BEGIN) {
          so[sp] = r.o;
          sd[sp] = r.d;
          sp++;
          Vec3 no = r.o, nd = r.d;
          inst_ray(P.insts[payload], no, nd);
          set_dir(r, no, nd);
        } else if (kind == G::K_INST_END) {
          sp--;
          set_dir(r, so[sp], sd[sp]);
        } else if (kind == G::K_MEDIUM) {
          if constexpr (MEDIA) {
            /* constant_medium.rs:34-76 */
            const G::Medium m = P.media[payload];
            const float inf = __uint_as_float(0x7f800000u);
            float c1 = inf, c2 = inf;
            uint32_t w1 = G::NONE, w2 = G::NONE;
            trace<CULL, FULL, false, COUNT>(P, nodes, prims, m.bstart, m.bend, r.o, r.d, r.time, -inf, c1, w1, pk, cn);
            if (w1 == G::NONE) continue;
            trace<CULL, FULL, false, COUNT>(P, nodes, prims, m.bstart, m.bend, r.o, r.d, r.time, c1 + 0.0001f, c2, w2, pk, cn);
            if (w2 == G::NONE) continue;
            float r1 = c1, r2 = c2;
            if (r1 < tmin) r1 = tmin;
            if (r2 > closest) r2 = closest;
            if (r1 >= r2) continue;
            if (r1 < 0.0f) r1 = 0.0f;
            float ray_length = sqrtf(r.dd);
            float inside = (r2 - r1) * ray_length;
            float xi = medium_xi(pk.pkey, pk.segment, m.medium_id);
            float hit_distance = m.neg_inv_density * (ln_f(xi) / P.ln_e);
            if (hit_distance > inside) continue;
            closest = r1 + hit_distance / ray_length;
            winner = here;
          }
        }
      }
      continue;
    }
    /* one primitive (payload) */
    const G::Prim* pp = prims + payload;
    const uint32_t km = pp->km;
    const uint32_t pkind = km & 3u;
    if constexpr (COUNT) cn.prims++;
    float t;
    bool h;
    if (FULL && pkind == G::P_RECT) h = rect_t(pp, (km >> 2) & 3u, r, tmin, closest, t);
    else h = sphere_root(pp, pkind, r, tmin, closest, t, P.motion_uniform != 0);
    if (h) {
      closest = t;
      winner = FULL ? here : payload; /* BASIC kernels name the primitive directly */
    }
  }
}

/* ------------------------------------------------------------------ hit record + shading */
struct Rec {
  Vec3 p, n;
  float u, v;
  bool front;
  uint32_t mat;
};

__device__ __forceinline__ void set_face_normal(Rec& rec, Vec3 dir, Vec3 outward) {
  rec.front = dot(dir, outward) < 0.0f;
  rec.n = rec.front ? outward : -outward;
}

/* sphere.rs:31-35 */
__device__ __forceinline__ void sphere_uv(Vec3 p, float& u, float& v) {
  float theta = acos_f(-p.y);
  float phi = atan2_f(-p.z, p.x) + PI_F;
  u = phi / (2.0f * PI_F);
  v = theta / PI_F;
}

/* Record of the winning leaf in world space (hit_record.rs, sphere.rs:57-73, rect.rs:70-83,
 * constant_medium.rs:66-75, then translation.rs:33-35 / rotation.rs:119-132 on the way out). */
template <bool FULL>
__device__ Rec make_record(const KParams& P, uint32_t winner, float t, Vec3 wo, Vec3 wd, float time, float tau) {
  Rec rec;
  rec.u = 0.0f;
  rec.v = 0.0f;
  if constexpr (!FULL) { /* winner is the primitive index */
    const G::Prim* pp = P.prims + winner;
    const uint32_t km = pp->km;
    float4 p0 = ld4(pp->p0);
    Vec3 c = v3(p0.x, p0.y, p0.z);
    if ((km & 3u) == G::P_MOVING) {
      float4 p1 = ld4(pp->p1);
      const float f = P.motion_uniform ? tau : (time - p1.w) / pp->p2[0];
      c = c + f * v3(p1.x, p1.y, p1.z);
    }
    rec.mat = km >> 4;
    Vec3 at = wo + t * wd;
    Vec3 outward = (at - c) / p0.w;
    rec.p = at;
    set_face_normal(rec, wd, outward);
    return rec;
  } else {
    const G::Node* np = P.nodes + winner;
    const uint32_t kp = np->kp;
    const uint32_t kind = (kp >> 24) & G::KIND_MASK, payload = kp & 0xFFFFFFu;
    uint32_t parent;
    if (kind == G::K_MEDIUM) parent = P.media[payload].parent;
    else parent = P.prims[payload].parent;
    uint32_t chain[G::MAX_INST_DEPTH];
    Vec3 dirs[G::MAX_INST_DEPTH];
    int n = 0;
    for (uint32_t q = parent; q != G::NONE && n < G::MAX_INST_DEPTH; q = P.insts[q].parent) chain[n++] = q;
    Vec3 o = wo, d = wd;
    for (int l = n - 1; l >= 0; l--) {
      dirs[l] = d;
      inst_ray(P.insts[chain[l]], o, d);
    }
    if (kind == G::K_MEDIUM) {
      rec.p = o + t * d;
      rec.n = v3(0.0f, 0.0f, 0.0f);
      rec.front = false;
      rec.mat = P.media[payload].mat;
    } else {
      const G::Prim* pp = P.prims + payload;
      const uint32_t km = pp->km;
      const uint32_t pkind = km & 3u;
      rec.mat = km >> 4;
      const bool uv = P.mats[rec.mat].needs_uv != 0;
      float4 p0 = ld4(pp->p0);
      if (pkind == G::P_RECT) {
        int k, a, b;
        plane_axes((km >> 2) & 3u, k, a, b);
        float av = o[a] + t * d[a];
        float bv = o[b] + t * d[b];
        rec.p = o + t * d;
        rec.u = (av - p0.x) / pp->p1[1];
        rec.v = (bv - p0.z) / pp->p1[2];
        Vec3 outward = v3(0.0f, 0.0f, 0.0f);
        outward[k] = 1.0f;
        set_face_normal(rec, d, outward);
      } else {
        Vec3 c = v3(p0.x, p0.y, p0.z);
        if (pkind == G::P_MOVING) {
          float4 p1 = ld4(pp->p1);
          const float f = P.motion_uniform ? tau : (time - p1.w) / pp->p2[0];
          c = c + f * v3(p1.x, p1.y, p1.z);
        }
        Vec3 at = o + t * d;
        Vec3 outward = (at - c) / p0.w;
        if (uv) sphere_uv(outward, rec.u, rec.v);
        rec.p = at;
        set_face_normal(rec, d, outward);
      }
    }
    for (int l = 0; l < n; l++) {
      const G::Inst& in = P.insts[chain[l]];
      if (in.kind == G::I_TRANSLATE) {
        rec.p = rec.p + v3(in.d[0], in.d[1], in.d[2]);
        set_face_normal(rec, dirs[l], rec.n);
      } else {
        int a = (int)(in.axis + 1) % 3, b = (int)(in.axis + 2) % 3;
        float s = in.sin_t, c = in.cos_t;
        Vec3 p = rec.p, nn = rec.n;
        p[a] = c * rec.p[a] - s * rec.p[b];
        p[b] = s * rec.p[a] + c * rec.p[b];
        nn[a] = c * rec.n[a] - s * rec.n[b];
        nn[b] = s * rec.n[a] + c * rec.n[b];
        rec.p = p;
        rec.n = nn;
      }
    }
    return rec;
  }
}

/* perlin_noise.rs:80-123 */
__device__ float perlin_noise(const G::Perlin* pn, Vec3 point) {
  int32_t i = sat_f2i32(floorf(point.x));
  int32_t j = sat_f2i32(floorf(point.y));
  int32_t k = sat_f2i32(floorf(point.z));
  float u = point.x - floorf(point.x);
  float v = point.y - floorf(point.y);
  float w = point.z - floorf(point.z);
  u = u * u * (3.0f - 2.0f * u);
  v = v * v * (3.0f - 2.0f * v);
  w = w * w * (3.0f - 2.0f * w);
  float acc = 0.0f;
#pragma unroll
  for (int idx = 0; idx < 8; idx++) {
    const int x = idx / 4, y = (idx / 2) % 2, z = idx % 2;
    uint32_t px = pn->perm[0][(uint32_t)((i + x) & 255)];
    uint32_t py = pn->perm[1][(uint32_t)((j + y) & 255)];
    uint32_t pz = pn->perm[2][(uint32_t)((k + z) & 255)];
    float4 g = ld4(pn->ranvec[px ^ py ^ pz]);
    Vec3 weight = v3(u - (float)x, v - (float)y, w - (float)z);
    acc += ((float)x * u + (float)(1 - x) * (1.0f - u)) * ((float)y * v + (float)(1 - y) * (1.0f - v)) *
           ((float)z * w + (float)(1 - z) * (1.0f - w)) * dot(v3(g.x, g.y, g.z), weight);
  }
  return acc;
}

/* sign of sin_f(v) for 1e-6 <= |v| <= 1e6: sin_f reduces v by pi/2 (hd_math reduce_pio2, same
 * operations here) and returns sin_poly(r) / cos_poly(r) / -sin_poly(r) / -cos_poly(r) by quadrant;
 * for |r| < 1 sin_poly keeps the sign of r and cos_poly is positive, so only the reduction is needed.
 * (|n| < 2^20: rint is exact and n & 3 is reduce_pio2's quadrant.) */
__device__ __forceinline__ bool sin_negative(float vf) {
  const double x = (double)vf;
  const double n = __builtin_rint(x * detail::TWO_OVER_PI);
  const double r = ((x - n * detail::P1) - n * detail::P2) - n * detail::P3;
  const int q = (int)n & 3;
  return q == 3 || (q == 0 && r < 0.0) || (q == 2 && r > 0.0);
}

/* the full product, as the oracle computes it; a real call, so that its f64 temporaries do not
 * count towards the registers of the kernels it is reached from (it runs only for rare inputs) */
__device__ __attribute__((noinline)) bool checker_product_negative(float vx, float vy, float vz) {
  return (sin_f(vx) * sin_f(vy)) * sin_f(vz) < 0.0f;
}

/* checker_texture.rs:22-29: sin(10x) * sin(10y) * sin(10z) < 0, decided from the signs.  With every
 * |v| in [1e-6, 1e6] each f32 sine is nonzero (an f32 there is > 1e-9 from any multiple of pi) and the
 * product of three cannot underflow, so the product is negative exactly when an odd number of
 * factors are; anything else (zero, tiny, huge, NaN) takes sin_f's full product. */
__device__ __forceinline__ bool checker_odd(float vx, float vy, float vz) {
  const float ax = fabsf(vx), ay = fabsf(vy), az = fabsf(vz);
  const bool in_range = ax >= 1e-6f && ax <= 1e6f && ay >= 1e-6f && ay <= 1e6f && az >= 1e-6f && az <= 1e6f;
  if (in_range) return sin_negative(vx) != (sin_negative(vy) != sin_negative(vz));
  return checker_product_negative(vx, vy, vz);
}

/* textures/.rs value() */
template <bool FULL, bool COUNT>
__device__ Vec3 tex_value(const KParams& P, uint32_t id, float u, float v, Vec3 p, Counts& cn) {
  for (int guard = 0; guard < 64; guard++) {
    const G::Tex& T = P.texs[id];
    if constexpr (COUNT) cn.tex++;
    if (T.kind == G::T_SOLID) return v3(T.a[0], T.a[1], T.a[2]);
    if (T.kind == G::T_CHECKER) { /* checker_texture.rs:22-29 */
      id = checker_odd(10.0f * p.x, 10.0f * p.y, 10.0f * p.z) ? T.i0 : T.i1;
      continue;
    }
    if constexpr (FULL) {
      if (T.kind == G::T_NOISE) { /* noise_texture.rs:24-31 + turbulence perlin_noise.rs:66-78 */
        const G::Perlin* pn = P.perlin + T.i0;
        float scale = T.a[0];
        Vec3 q = scale * p;
        float accumulator = 0.0f, weight = 1.0f;
        for (int o = 0; o < 7; o++) {
          accumulator += weight * perlin_noise(pn, q);
          weight *= 0.5f;
          q = q * 2.0f;
        }
        float s = 1.0f + sin_f((scale * p.z) + (10.0f * fabsf(accumulator)));
        return (v3(1.0f, 1.0f, 1.0f) * 0.5f) * s;
      }
      if (T.kind == G::T_IMAGE) { /* image_texture.rs:36-62 */
        if (T.i1 == 0) return v3(1.0f, 0.0f, 1.0f);
        float uu = u < 0.0f ? 0.0f : (u > 1.0f ? 1.0f : u);
        float vc = v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v);
        float vv = 1.0f - vc;
        uint32_t ii = sat_f2u32(uu * (float)T.i1);
        uint32_t jj = sat_f2u32(vv * (float)T.i2);
        if (ii >= T.i1) ii = T.i1 - 1;
        if (jj >= T.i2) jj = T.i2 - 1;
        const uint8_t* px = P.images + T.i0 + ((size_t)jj * T.i1 + ii) * T.i3;
        const float cs = 1.0f / 255.0f;
        return v3(cs * (float)px[0], cs * (float)px[1], cs * (float)px[2]);
      }
    }
    break;
  }
  return v3(0.0f, 0.0f, 0.0f);
}

/* ------------------------------------------------------------------ one path, one segment at a time */
struct PathState {
  Rng rng;
  PathKey pk;
  uint32_t depth_left;
  Vec3 ro, rd;
  float rtime;
  Vec3 thr, rad;
  bool traced; /* the last segment() call made a world.hit call */
};

/* application.rs:444-447 + camera.rs:85-95: jitter, lens sample, shutter time */
__device__ __forceinline__ void start_sample(const KParams& P, PathState& ps, uint32_t px, uint32_t py,
                                             uint32_t sample) {
  ps.pk.pkey = path_key(P.seed, py * P.W + px, P.sample_offset + sample);
  ps.pk.segment = 0;
  ps.rng = rng_from_key(ps.pk.pkey);
  float u = ((float)px + ps.rng.gen_f32()) / ((float)P.W - 1.0f);
  float v = ((float)py + ps.rng.gen_f32()) / ((float)P.H - 1.0f);
  Vec3 disk = random_in_unit_disk(ps.rng);
  ps.rtime = ps.rng.gen_range_f32(P.time0, P.time1);
  Vec3 rdk = P.lens_radius * disk;
  Vec3 offset = P.cam_u * rdk.x + P.cam_vv * rdk.y;
  ps.ro = P.cam_origin + offset;
  ps.rd = (((P.cam_llc + u * P.cam_h) + v * P.cam_v) - P.cam_origin) - offset;
  ps.thr = v3(1.0f, 1.0f, 1.0f);
  ps.rad = v3(0.0f, 0.0f, 0.0f);
  ps.depth_left = P.max_depth;
}

/* The part of one ray_color step after world.hit (application.rs:483-494): background on a miss,
 * else hit record, emission and scatter.  (ro, rd, rtime) is the segment just traced; the scattered
 * ray goes to ps.ro/ps.rd.  Returns true when the path is finished. */
template <bool FULL, bool COUNT>
__device__ __forceinline__ bool shade(const KParams& P, PathState& ps, uint32_t winner, float closest, Vec3 ro,
                                      Vec3 rd, float rtime, float tau, Counts& cn) {
  if (winner == G::NONE) {
    ps.rad = ps.rad + mul_elem(ps.thr, P.background);
    return true;
  }
  Rec rec = make_record<FULL>(P, winner, closest, ro, rd, rtime, tau);
  const G::Mat M = P.mats[rec.mat];
  Vec3 emitted = v3(0.0f, 0.0f, 0.0f);
  Vec3 att = v3(0.0f, 0.0f, 0.0f), ndir = v3(0.0f, 0.0f, 0.0f);
  bool scattered = false;
  Rng& rng = ps.rng;
  if (M.kind == G::M_LAMBERTIAN) { /* lambertian.rs:27-38 */
    ndir = rec.n + random_unit_vector(rng);
    if (near_zero(ndir)) ndir = rec.n;
    att = tex_value<FULL, COUNT>(P, M.tex, rec.u, rec.v, rec.p, cn);
    scattered = true;
  } else if (M.kind == G::M_METAL) { /* metal.rs:29-42 */
    Vec3 reflected = reflect(normalize(rd), rec.n);
    ndir = reflected + M.a[3] * random_in_unit_sphere(rng);
    scattered = dot(ndir, rec.n) > 0.0f;
    att = v3(M.a[0], M.a[1], M.a[2]);
  } else if (M.kind == G::M_DIELECTRIC) { /* dielectric.rs:31-55 */
    float ratio = rec.front ? (1.0f / M.a[0]) : M.a[0];
    Vec3 ud = normalize(rd);
    float cos_theta = min_rs(dot(-ud, rec.n), 1.0f);
    float sin_theta = sqrtf(1.0f - cos_theta * cos_theta);
    bool cannot_refract = (ratio * sin_theta) > 1.0f;
    if (cannot_refract || reflectance(cos_theta, ratio) > rng.gen_f32()) ndir = reflect(ud, rec.n);
    else ndir = refract(ud, rec.n, ratio);
    att = v3(1.0f, 1.0f, 1.0f);
    scattered = true;
  } else if (FULL && M.kind == G::M_DIFFUSE_LIGHT) { /* diffuse_light.rs:20-28 */
    emitted = tex_value<FULL, COUNT>(P, M.tex, rec.u, rec.v, rec.p, cn);
  } else if (FULL && M.kind == G::M_ISOTROPIC) { /* isotropic.rs:26-33 */
    att = tex_value<FULL, COUNT>(P, M.tex, rec.u, rec.v, rec.p, cn);
    ndir = random_in_unit_sphere(rng);
    scattered = true;
  }
  /* L = emitted + att * L_next, accumulated front to back */
  ps.rad = ps.rad + mul_elem(ps.thr, emitted);
  if (!scattered) return true;
  ps.thr = mul_elem(ps.thr, att);
  ps.ro = rec.p;
  ps.rd = ndir;
  ps.depth_left--;
  return false;
}

/* One step of ray_color (application.rs:477-495).  Returns true when the path is finished.
 * dbg (debug kernel only): receives o, d, time, t, winner of the traced segment. */
template <int CULL, bool FULL, bool COUNT, bool FAST>
__device__ __forceinline__ bool segment(const KParams& P, const G::Node* nodes, const G::Prim* prims,
                                        PathState& ps, Counts& cn, float* dbg) {
  ps.traced = false;
  if (ps.depth_left == 0) return true; /* depth cap: black (:478-480) */
  float closest = __uint_as_float(0x7f800000u);
  uint32_t winner = G::NONE;
  trace<CULL, FULL, FULL, COUNT, FAST>(P, nodes, prims, 0u, P.main_end, ps.ro, ps.rd, ps.rtime, P.t_min, closest,
                                       winner, ps.pk, cn);
  ps.traced = true;
  ps.pk.segment++;
  if (dbg) {
    dbg[0] = ps.ro.x; dbg[1] = ps.ro.y; dbg[2] = ps.ro.z;
    dbg[3] = ps.rd.x; dbg[4] = ps.rd.y; dbg[5] = ps.rd.z;
    dbg[6] = ps.rtime; dbg[7] = closest; dbg[8] = __uint_as_float(winner);
  }
  const float tau = P.motion_uniform ? (ps.rtime - P.motion_t0) / P.motion_span : 0.0f;
  return shade<FULL, COUNT>(P, ps, winner, closest, ps.ro, ps.rd, ps.rtime, tau, cn);
}

/* Diagnostics: trace ONE path (pixel, sample) and record every segment (9 floats each). */
template <int CULL, bool FULL, bool FAST>
__global__ void debug_path_kernel(KParams P, uint32_t px, uint32_t py, uint32_t sample, float* out,
                                  uint32_t max_seg, uint32_t* n_out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  PathState ps;
  Counts cn{0u, 0u, 0u, 0u, 0u, 0u};
  start_sample(P, ps, px, py, sample);
  uint32_t n = 0;
  float scratch[9];
  for (;;) {
    bool done = segment<CULL, FULL, false, FAST>(P, P.nodes, P.prims, ps, cn, n < max_seg ? out + 9 * n : scratch);
    if (ps.traced) n++;
    if (done) break;
  }
  *n_out = n;
  out[9 * max_seg + 0] = ps.rad.x;
  out[9 * max_seg + 1] = ps.rad.y;
  out[9 * max_seg + 2] = ps.rad.z;
}

/* ------------------------------------------------------------------ the megakernel */
/* LDS: the node stream and primitive records are copied into LDS once per workgroup (they are
 * read ~60 times per ray by dependent loads; LDS latency is a fraction of an L2 hit). */
template <bool LDS, bool FAST>
constexpr int block_threads() { return LDS ? (FAST ? 1024 : 512) : 256; }

/* Copy the node stream and primitive records into this workgroup's LDS. */
__device__ __forceinline__ void stage_scene(const KParams& P, float4* lds, const G::Node*& nodes, const G::Prim*& prims) {
  const uint32_t n4 = P.n_nodes * (uint32_t)(sizeof(G::Node) / 16);
  const uint32_t p4 = P.n_prims * (uint32_t)(sizeof(G::Prim) / 16);
  const float4* gn = reinterpret_cast<const float4*>(P.nodes);
  const float4* gp = reinterpret_cast<const float4*>(P.prims);
  for (uint32_t k = threadIdx.x; k < n4; k += blockDim.x) lds[k] = gn[k];
  for (uint32_t k = threadIdx.x; k < p4; k += blockDim.x) lds[n4 + k] = gp[k];
  __syncthreads();
  nodes = reinterpret_cast<const G::Node*>(lds);
  prims = reinterpret_cast<const G::Prim*>(lds + n4);
}

/* A lane's current work item: one pixel and a chunk [sample, sample_end) of its samples. */
struct Item {
  uint32_t pxy; /* px | py << 16 */
  uint32_t out_idx, chunk, sample, sample_end;
};

/* Idle lanes of the wave claim work items with ONE atomicAdd (ballot + popcount).  Items are
 * ordered [tile][8x8 block][chunk][64 pixels], so a wave starts on 64 neighbouring pixels. */
__device__ __forceinline__ void claim_work(const KParams& P, uint32_t lane, bool& has_item, bool& exhausted,
                                           Item& it) {
  const bool want = !has_item && !exhausted;
  const unsigned long long want_mask = __ballot(want);
  if (!want_mask) return;
  const uint32_t cnt = (uint32_t)__popcll(want_mask);
  const int leader = __ffsll((long long)want_mask) - 1;
  uint32_t base = 0;
  if ((int)lane == leader) base = atomicAdd(P.counter, cnt);
  base = __shfl(base, leader);
  if (!want) return;
  const uint32_t rank = (uint32_t)__popcll(want_mask & ((1ull << lane) - 1ull));
  const uint32_t w = base + rank;
  if (w >= P.total_work) {
    exhausted = true;
    return;
  }
  /* tile (binary search on pad_start), then [8x8 block][chunk][64 pixels] inside it */
  uint32_t lo = 0, hi = P.n_tiles - 1;
  while (lo < hi) {
    uint32_t mid = (lo + hi + 1) >> 1;
    if (P.tiles[mid].pad_start <= w) lo = mid; else hi = mid - 1;
  }
  const G::TileDev T = P.tiles[lo];
  const uint32_t q = w - T.pad_start;
  const uint32_t blk = q / (64u * P.n_chunks), rem = q - blk * 64u * P.n_chunks;
  const uint32_t c = rem >> 6, in = rem & 63u;
  const uint32_t lx = (blk % T.bw) * 8u + (in & 7u), ly = (blk / T.bw) * 8u + (in >> 3);
  if (lx < T.w && ly < T.h) {
    has_item = true;
    it.pxy = (T.x + lx) | ((T.y + ly) << 16);
    it.out_idx = T.out_off + ly * T.w + lx;
    it.chunk = c;
    it.sample = c * P.chunk;
    it.sample_end = min(P.spp, it.sample + P.chunk);
  }
}

/* A finished sample: add it to the chunk sum in order (application.rs:448); a finished chunk goes to
 * the output (one chunk: sqrt(sum/spp), alpha 1, :451-456) or to its partial-sum slot. */
__device__ __forceinline__ void finish_sample(const KParams& P, Item& it, Vec3& sum, Vec3 rad, float scale,
                                              bool& has_item, uint32_t& n_samples, uint32_t& n_pixels) {
  sum = sum + rad;
  n_samples++;
  if (++it.sample == it.sample_end) {
    if (P.n_chunks == 1) {
      P.out[it.out_idx] = make_float4(sqrtf(sum.x * scale), sqrtf(sum.y * scale), sqrtf(sum.z * scale), 1.0f);
      n_pixels++;
    } else {
      P.partial[(size_t)it.chunk * P.n_out + it.out_idx] = make_float4(sum.x, sum.y, sum.z, 0.0f);
      if (it.chunk == 0) n_pixels++;
    }
    has_item = false;
    sum = v3(0.0f, 0.0f, 0.0f);
  }
}

__device__ __forceinline__ void init_path_state(PathState& ps) {
  ps.rng.s0 = ps.rng.s1 = ps.rng.s2 = ps.rng.s3 = 1u;
  ps.pk = PathKey{0ull, 0u};
  ps.depth_left = 0;
  ps.ro = v3(0.0f, 0.0f, 0.0f);
  ps.rd = v3(0.0f, 0.0f, 1.0f);
  ps.rtime = 0.0f;
  ps.thr = v3(1.0f, 1.0f, 1.0f);
  ps.rad = v3(0.0f, 0.0f, 0.0f);
  ps.traced = false;
}

__device__ __forceinline__ void flush_counts(const KParams& P, const Counts& cn) {
  atomicAdd(&P.stats[3], (unsigned long long)cn.nodes);
  atomicAdd(&P.stats[4], (unsigned long long)cn.prims);
  atomicAdd(&P.stats[5], (unsigned long long)cn.tex);
  atomicAdd(&P.stats[6], (unsigned long long)cn.walk_slots);
  atomicAdd(&P.stats[7], (unsigned long long)cn.shade_slots);
  atomicAdd(&P.stats[8], (unsigned long long)cn.prim_slots);
}

__device__ __forceinline__ void flush_stats(const KParams& P, uint32_t n_seg, uint32_t n_samples, uint32_t n_pixels,
                                            const Counts& cn, bool count) {
  atomicAdd(&P.stats[0], (unsigned long long)n_seg);
  atomicAdd(&P.stats[1], (unsigned long long)n_samples);
  atomicAdd(&P.stats[2], (unsigned long long)n_pixels);
  if (count) {
    atomicAdd(&P.stats[3], (unsigned long long)cn.nodes);
    atomicAdd(&P.stats[4], (unsigned long long)cn.prims);
    atomicAdd(&P.stats[5], (unsigned long long)cn.tex);
    atomicAdd(&P.stats[6], (unsigned long long)cn.walk_slots);
    atomicAdd(&P.stats[7], (unsigned long long)cn.shade_slots);
    atomicAdd(&P.stats[8], (unsigned long long)cn.prim_slots);
  }
}

/* The general kernel (every feature): each iteration of the wave loop advances every busy lane by
 * exactly one ray segment.  Lanes whose path ended start their next sample in the same iteration. */
template <int CULL, bool FULL, bool COUNT, bool LDS, bool FAST>
__global__ __launch_bounds__((block_threads<LDS, FAST>())) void render_kernel(KParams P) {
  extern __shared__ float4 lds_scene[];
  const G::Node* nodes = P.nodes;
  const G::Prim* prims = P.prims;
  if constexpr (LDS) stage_scene(P, lds_scene, nodes, prims);
  const uint32_t lane = threadIdx.x & 63u;
  const float scale = 1.0f / (float)P.spp; /* application.rs:403 */

  bool has_item = false, exhausted = false, in_path = false;
  Item it{0u, 0u, 0u, 0u, 0u};
  Vec3 sum = v3(0.0f, 0.0f, 0.0f);
  PathState ps;
  init_path_state(ps);
  uint32_t n_seg = 0, n_samples = 0, n_pixels = 0;
  Counts cn{0u, 0u, 0u, 0u, 0u, 0u};

  uint32_t seg_nodes = 0; /* COUNT: node visits of this lane's last segment */
  for (;;) {
    if constexpr (COUNT) { /* every lane is active here: the walk took as long as its longest lane */
      cn.walk_slots += wave_max(seg_nodes);
      cn.shade_slots++;
      seg_nodes = 0;
    }
    claim_work(P, lane, has_item, exhausted, it);
    if (!__any(has_item || !exhausted)) break;
    if (!has_item) continue;
    if (!in_path) {
      start_sample(P, ps, it.pxy & 0xFFFFu, it.pxy >> 16, it.sample);
      in_path = true;
    }
    const uint32_t nodes_before = cn.nodes;
    const bool done = segment<CULL, FULL, COUNT, FAST>(P, nodes, prims, ps, cn, nullptr);
    if constexpr (COUNT) seg_nodes = cn.nodes - nodes_before;
    if (ps.traced) n_seg++;
    if (done) {
      in_path = false;
      finish_sample(P, it, sum, ps.rad, scale, has_item, n_samples, n_pixels);
    }
  }
  flush_stats(P, n_seg, n_samples, n_pixels, cn, COUNT);
}

/* One node of the BASIC world walk (spheres and moving spheres under boxes; trace() restricted).
 * Both 16-B halves of the node are loaded and the box tested for every node kind (a PRIM node's box
 * result is ignored), so the only divergent branch is the primitive test. */
template <int CULL, bool COUNT>
__device__ __forceinline__ void basic_step(const KParams& P, const G::Node* __restrict__ nodes,
                                           const G::Prim* __restrict__ prims, uint32_t& i, const TRay& r,
                                           float& closest, uint32_t& winner, Counts& cn) {
  const G::Node* np = nodes + i;
  const float4 a = ld4(np->mn);
  const float4 b = ld4(np->mx);
  const uint32_t kp = __float_as_uint(b.w);
  const uint32_t kind = (kp >> 24) & G::KIND_MASK;
  const float tmin = P.t_min;
  if constexpr (COUNT) cn.nodes++;
  const bool pass = box_hit<CULL>(a, b, r, tmin, closest, (kp & G::NODE_REF_ONLY) != 0) || kind == G::K_PRIM;
  i = pass ? i + 1 : __float_as_uint(a.w);
  const bool test = pass && kind != G::K_BOX;
  if constexpr (COUNT) cn.prim_slots += __any(test) ? 1u : 0u;
  if (test) {
    const uint32_t payload = kp & 0xFFFFFFu;
    const G::Prim* pp = prims + payload;
    if constexpr (COUNT) cn.prims++;
    float t;
    if (sphere_root(pp, pp->km & 3u, r, tmin, closest, t, P.motion_uniform != 0)) {
      closest = t;
      winner = payload;
    }
  }
}

/* The BASIC kernel (sphere scenes: the Random family), with POSTPONED shading.  A lane's walk state
 * (node, closest, winner, ray) lives across passes: the wave steps the walks of all its lanes one
 * node at a time and leaves the node loop only when at least P.postpone lanes have finished theirs
 * (or none is still walking); those lanes shade, start their next segment or sample, and the wave
 * goes back to stepping.  Every lane still runs exactly the reference's sequence of world.hit calls
 * and draws, so the image is the same as render_kernel's; only the wave's SIMD occupancy changes
 * (a wave no longer idles on its slowest lane's walk before every shading step). */
#ifndef HRT_WALK_UNROLL
#define HRT_WALK_UNROLL 2
#endif
constexpr int WALK_UNROLL = HRT_WALK_UNROLL; /* node steps between two checks of the wave's exit test */
#ifndef HRT_BASIC_WAVES
#define HRT_BASIC_WAVES 6
#endif
/* waves per SIMD of the sphere-scene kernel: caps its VGPRs at 512 / waves (granule 8); with the
 * scene in LDS two workgroups share a CU, so a workgroup is 128 * waves
 * threads (4 SIMDs x waves x 64 / 2). */
constexpr int BASIC_WAVES = HRT_BASIC_WAVES;
template <bool LDS>
constexpr int basic_block_threads() { return LDS ? 128 * BASIC_WAVES : 256; }

template <int CULL, bool COUNT, bool LDS>
__global__ __launch_bounds__(basic_block_threads<LDS>(), BASIC_WAVES)
void render_basic_kernel(KParams P) {
  extern __shared__ float4 lds_scene[];
  const G::Node* nodes = P.nodes;
  const G::Prim* prims = P.prims;
  if constexpr (LDS) stage_scene(P, lds_scene, nodes, prims);
  const uint32_t lane = threadIdx.x & 63u;
  const float scale = 1.0f / (float)P.spp; /* application.rs:403 */
  const float inf = __uint_as_float(0x7f800000u);
  const uint32_t end = P.main_end;
  const uint32_t need = P.postpone;

  bool has_item = false, exhausted = false;
  bool walking = false; /* a segment is in flight (walk running, or finished and waiting to shade) */
  Item it{0u, 0u, 0u, 0u, 0u};
  Vec3 sum = v3(0.0f, 0.0f, 0.0f);
  PathState ps;
  init_path_state(ps);
  TRay r;
  set_ray(r, ps.ro, ps.rd, 0.0f, P);
  uint32_t node = G::NONE, winner = G::NONE;
  float closest = inf;
  uint32_t n_seg = 0, n_samples = 0, n_pixels = 0; /* wave totals (uniform) */
  Counts cn{0u, 0u, 0u, 0u, 0u, 0u};
  PhaseClock pc{{0ull, 0ull, 0ull}, 0ull};
  auto stamp = [&](int phase) {
    if constexpr (COUNT) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      if (phase >= 0) pc.cyc[phase] += t - pc.last;
      pc.last = t;
    }
  };
  stamp(-1);

  for (;;) {
    /* lanes without work claim it; lanes with work but no segment in flight start a sample */
    claim_work(P, lane, has_item, exhausted, it);
    if (!__any(has_item || !exhausted)) break;
    if (has_item && !walking) {
      start_sample(P, ps, it.pxy & 0xFFFFu, it.pxy >> 16, it.sample);
      walking = true;
      set_ray(r, ps.ro, ps.rd, ps.rtime, P);
      closest = inf;
      winner = G::NONE;
      node = ps.depth_left == 0 ? G::NONE : 0u; /* max_depth 0: black without a world.hit (:478-480) */
    }
    /* step the walks until enough lanes have finished (lanes not walking hold node >= end) */
    if constexpr (COUNT) cn.shade_slots++;
    stamp(0);
    const unsigned long long walkers = __ballot(walking);
    for (;;) {
#pragma unroll
      for (int u = 0; u < WALK_UNROLL; u++) {
        if constexpr (COUNT) cn.walk_slots++;
        if (node < end) basic_step<CULL, COUNT>(P, nodes, prims, node, r, closest, winner, cn);
      }
      const unsigned long long live = __ballot(node < end);
      if (!live || (uint32_t)__popcll(walkers & ~live) >= need) break;
    }
    stamp(1);
    /* shade the finished segments (application.rs:483-494) */
    const bool shading = walking && node >= end;
    const bool traced = shading && node != G::NONE;
    bool sample_done = false, chunk_done = false;
    if (shading) {
      const bool done =
          !traced || shade<false, COUNT>(P, ps, winner, closest, r.o, r.d, r.time, r.tau, cn) || ps.depth_left == 0;
      if (done) {
        /* application.rs:448: samples of a chunk summed in order */
        walking = false;
        node = G::NONE;
        sum = sum + ps.rad;
        sample_done = true;
        if (++it.sample == min(P.spp, (it.chunk + 1u) * P.chunk)) {
          if (P.n_chunks == 1) /* sqrt(sum / spp), alpha 1 (:451-456) */
            P.out[it.out_idx] = make_float4(sqrtf(sum.x * scale), sqrtf(sum.y * scale), sqrtf(sum.z * scale), 1.0f);
          else
            P.partial[(size_t)it.chunk * P.n_out + it.out_idx] = make_float4(sum.x, sum.y, sum.z, 0.0f);
          chunk_done = true;
          has_item = false;
          sum = v3(0.0f, 0.0f, 0.0f);
        }
      } else {
        set_dir(r, ps.ro, ps.rd); /* the scattered ray keeps the sample's shutter time */
        closest = inf;
        winner = G::NONE;
        node = 0u;
      }
    }
    n_seg += (uint32_t)__popcll(__ballot(traced));
    n_samples += (uint32_t)__popcll(__ballot(sample_done));
    n_pixels += (uint32_t)__popcll(__ballot(chunk_done && it.chunk == 0u));
    stamp(2);
  }
  if (lane == 0) {
    atomicAdd(&P.stats[0], (unsigned long long)n_seg);
    atomicAdd(&P.stats[1], (unsigned long long)n_samples);
    atomicAdd(&P.stats[2], (unsigned long long)n_pixels);
  }
  if constexpr (COUNT) {
    flush_counts(P, cn);
    if (lane == 0)
      for (int k = 0; k < 3; k++) atomicAdd(&P.stats[9 + k], pc.cyc[k]);
  }
}

/* chunk sums -> pixel, in chunk order (fixed, so 1/2/4/8-GPU splits give identical bits);
 * then sqrt(sum * (1/spp)) with alpha 1 (application.rs:451-456) */
__global__ __launch_bounds__(256) void reduce_chunks(const float4* __restrict__ partial, float4* __restrict__ out,
                                                     uint32_t n_out, uint32_t n_chunks, uint32_t spp) {
  const float scale = 1.0f / (float)spp;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n_out; i += gridDim.x * blockDim.x) {
    float4 a = partial[i];
    Vec3 sum = v3(a.x, a.y, a.z);
    for (uint32_t c = 1; c < n_chunks; c++) {
      float4 b = partial[(size_t)c * n_out + i];
      sum = sum + v3(b.x, b.y, b.z);
    }
    out[i] = make_float4(sqrtf(sum.x * scale), sqrtf(sum.y * scale), sqrtf(sum.z * scale), 1.0f);
  }
}

__global__ void math_kernel(int op, const float* x, const float* y, float* out, uint32_t n) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float a = x[i], b = y ? y[i] : 0.0f, r = 0.0f;
  switch (op) {
    case 0: r = sin_f(a); break;
    case 1: r = cos_f(a); break;
    case 2: r = acos_f(a); break;
    case 3: r = atan2_f(a, b); break;
    case 4: r = ln_f(a); break;
    case 5: r = pow5_f(a); break;
    case 6: r = tan_f(a); break;
    case 7: r = div_rn(a, b, 1.0f / b); break; /* the walk's division by dot(d, d) */
  }
  out[i] = r;
}

/* ------------------------------------------------------------------ host helpers */
struct HipError {
  hrt_status code;
  std::string msg;
};

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw HipError{HRT_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e)};
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    hip_check(hipGetDevice(&prev), "hipGetDevice");
    if (dev >= 0 && dev != prev) hip_check(hipSetDevice(dev), "hipSetDevice");
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

template <class F>
hrt_status hguard(F&& f) {
  try {
    f();
    return HRT_OK;
  } catch (const HipError& e) {
    set_error(e.msg);
    return e.code;
  } catch (const std::bad_alloc&) {
    set_error("out of host memory");
    return HRT_ERR_OOM;
  } catch (const std::exception& e) {
    set_error(e.what());
    return HRT_ERR_INVALID_ARG;
  }
}

constexpr size_t SLOT_HDR = 128; /* work counter + 12 stats words, padded */

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

/* persistent grid: as many workgroups as are co-resident on the device (cached per kernel/device) */
int resident_grid(const void* fn, int block, int device, size_t smem, bool lds) {
  struct Key {
    const void* fn;
    int device;
    size_t smem;
    int grid;
  };
  static std::mutex mu;
  static std::vector<Key> cache;
  std::lock_guard<std::mutex> lk(mu);
  for (const Key& k : cache)
    if (k.fn == fn && k.device == device && k.smem == smem) return k.grid;
  if (lds) hip_check(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem),
                     "hipFuncSetAttribute(LDS)");
  int per_cu = 0;
  hip_check(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, block, smem),
            "hipOccupancyMaxActiveBlocksPerMultiprocessor");
  hipDeviceProp_t prop;
  hip_check(hipGetDeviceProperties(&prop, device), "hipGetDeviceProperties");
  const int g = std::max(1, per_cu) * prop.multiProcessorCount;
  cache.push_back(Key{fn, device, smem, g});
  return g;
}

template <int CULL, bool FULL, bool COUNT, bool LDS, bool FAST>
void launch(const KParams& kp, int device, hipStream_t stream, size_t smem) {
  const void* fn = (const void*)render_kernel<CULL, FULL, COUNT, LDS, FAST>;
  const int block = block_threads<LDS, FAST>();
  const int grid = resident_grid(fn, block, device, LDS ? smem : 0, LDS);
  hipLaunchKernelGGL((render_kernel<CULL, FULL, COUNT, LDS, FAST>), dim3(grid), dim3(block), LDS ? smem : 0, stream,
                     kp);
  hip_check(hipGetLastError(), "render_kernel launch");
}

template <int CULL, bool COUNT, bool LDS>
void launch_basic(const KParams& kp, int device, hipStream_t stream, size_t smem) {
  const void* fn = (const void*)render_basic_kernel<CULL, COUNT, LDS>;
  const int block = basic_block_threads<LDS>();
  const int grid = resident_grid(fn, block, device, LDS ? smem : 0, LDS);
  hipLaunchKernelGGL((render_basic_kernel<CULL, COUNT, LDS>), dim3(grid), dim3(block), LDS ? smem : 0, stream, kp);
  hip_check(hipGetLastError(), "render_basic_kernel launch");
}

/* LDS residency: the reference-order stream must fit twice per CU (two 512-thread workgroups of the
 * 160 KiB), the 8 SAH octant streams once (one 1024-thread workgroup). */
constexpr size_t LDS_SCENE_MAX = 72 * 1024;
constexpr size_t LDS_FAST_MAX = 150 * 1024;

struct Plan {
  bool full, fast, lds;
  bool general; /* sphere scene forced onto the general kernel (diagnostics: HRT_KERNEL=general) */
  int cull;
  size_t smem;
};

Plan plan(const hrt_scene* s, const hrt_camera* cam, uint32_t flags) {
  Plan pl;
  pl.full = (s->feature_mask & ~G::F_BASIC) != 0;
  /* default: exact.  A ray time outside the interval the BVH boxes were built for can put a moving
   * sphere outside its box: only the reference test is then faithful. */
  const bool shutter_ok = cam->time0 >= s->box_t0 && cam->time1 <= s->box_t1;
  pl.cull = s->cull_mode;
  if ((flags & HRT_RENDER_FAST_CULL) && s->all_boxes_ok && shutter_ok) pl.cull = G::CULL_SLAB;
  if ((flags & HRT_RENDER_REFERENCE_CULL) || !shutter_ok) pl.cull = G::CULL_REFERENCE;
  /* SAH streams: opt-in approximate mode for sphere-only scenes (boxes over t in [0, 1]) */
  pl.fast = !pl.full && pl.cull == G::CULL_SLAB && s->f_stream_len > 0 && (flags & HRT_RENDER_SAH) != 0 &&
            cam->time0 >= 0.0f && cam->time1 <= 1.0f;
  pl.smem = pl.fast ? (8 * (size_t)s->f_stream_len * sizeof(G::Node) + s->f_prims.size() * sizeof(G::Prim))
                    : (s->main_end * sizeof(G::Node) + s->g_prims.size() * sizeof(G::Prim));
  pl.lds = (flags & HRT_RENDER_NO_LDS) == 0 && !pl.full && pl.smem <= (pl.fast ? LDS_FAST_MAX : LDS_SCENE_MAX);
  const char* k = getenv("HRT_KERNEL");
  pl.general = k && strcmp(k, "general") == 0;
  return pl;
}

template <bool COUNT>
void launch_any(const hrt_scene* s, const Plan& pl, const KParams& kp, hipStream_t stream) {
  const size_t smem = pl.lds ? pl.smem : 0;
  if (pl.fast) {
    if (pl.lds) launch<G::CULL_SLAB, false, COUNT, true, true>(kp, s->device, stream, smem);
    else launch<G::CULL_SLAB, false, COUNT, false, true>(kp, s->device, stream, 0);
  } else if (pl.general && !pl.full) {
    const int c = pl.cull;
    if (c == G::CULL_EXACT) pl.lds ? launch<G::CULL_EXACT, false, COUNT, true, false>(kp, s->device, stream, smem)
                                   : launch<G::CULL_EXACT, false, COUNT, false, false>(kp, s->device, stream, 0);
    else if (c == G::CULL_SLAB) pl.lds ? launch<G::CULL_SLAB, false, COUNT, true, false>(kp, s->device, stream, smem)
                                       : launch<G::CULL_SLAB, false, COUNT, false, false>(kp, s->device, stream, 0);
    else pl.lds ? launch<G::CULL_REFERENCE, false, COUNT, true, false>(kp, s->device, stream, smem)
                : launch<G::CULL_REFERENCE, false, COUNT, false, false>(kp, s->device, stream, 0);
  } else if (pl.cull == G::CULL_EXACT) {
    if (pl.full) launch<G::CULL_EXACT, true, COUNT, false, false>(kp, s->device, stream, 0);
    else if (pl.lds) launch_basic<G::CULL_EXACT, COUNT, true>(kp, s->device, stream, smem);
    else launch_basic<G::CULL_EXACT, COUNT, false>(kp, s->device, stream, 0);
  } else if (pl.cull == G::CULL_SLAB) {
    if (pl.full) launch<G::CULL_SLAB, true, COUNT, false, false>(kp, s->device, stream, 0);
    else if (pl.lds) launch_basic<G::CULL_SLAB, COUNT, true>(kp, s->device, stream, smem);
    else launch_basic<G::CULL_SLAB, COUNT, false>(kp, s->device, stream, 0);
  } else {
    if (pl.full) launch<G::CULL_REFERENCE, true, COUNT, false, false>(kp, s->device, stream, 0);
    else if (pl.lds) launch_basic<G::CULL_REFERENCE, COUNT, true>(kp, s->device, stream, smem);
    else launch_basic<G::CULL_REFERENCE, COUNT, false>(kp, s->device, stream, 0);
  }
}

/* BASIC-kernel tuning knob, 1..64 lanes (read per launch; any value gives the same image):
 *   HRT_POSTPONE   a wave leaves the walk to shade once this many lanes have finished theirs. */
uint32_t env_knob(const char* name, uint32_t dflt) {
  const char* e = getenv(name);
  const long x = e ? strtol(e, nullptr, 10) : 0;
  return (uint32_t)(x >= 1 && x <= 64 ? x : dflt);
}

/* scene + camera + render knobs of a launch (work-distribution fields are set by the caller) */
KParams scene_params(const hrt_scene* s, const hrt_camera* cam, const hrt_render_params* p, const Plan& pl) {
  KParams kp;
  memset(&kp, 0, sizeof(kp));
  uint8_t* base = (uint8_t*)s->d_blob;
  kp.nodes = (const G::Node*)(base + (pl.fast ? s->off_fnodes : s->off_nodes));
  kp.prims = (const G::Prim*)(base + (pl.fast ? s->off_fprims : s->off_prims));
  kp.insts = (const G::Inst*)(base + s->off_insts);
  kp.media = (const G::Medium*)(base + s->off_media);
  kp.mats = (const G::Mat*)(base + s->off_mats);
  kp.texs = (const G::Tex*)(base + s->off_texs);
  kp.perlin = (const G::Perlin*)(base + s->off_perlin);
  kp.images = (const uint8_t*)(base + s->off_images);
  kp.main_end = s->main_end;
  kp.ln_e = s->ln_e;
  kp.cam_origin = v3(cam->origin[0], cam->origin[1], cam->origin[2]);
  kp.cam_llc = v3(cam->lower_left_corner[0], cam->lower_left_corner[1], cam->lower_left_corner[2]);
  kp.cam_h = v3(cam->horizontal[0], cam->horizontal[1], cam->horizontal[2]);
  kp.cam_v = v3(cam->vertical[0], cam->vertical[1], cam->vertical[2]);
  kp.cam_u = v3(cam->u[0], cam->u[1], cam->u[2]);
  kp.cam_vv = v3(cam->v[0], cam->v[1], cam->v[2]);
  kp.lens_radius = cam->lens_radius;
  kp.time0 = cam->time0;
  kp.time1 = cam->time1;
  kp.W = p->width;
  kp.H = p->height;
  kp.spp = p->samples;
  kp.max_depth = p->max_depth;
  kp.sample_offset = p->sample_offset;
  kp.t_min = p->t_min;
  kp.background = v3(p->background[0], p->background[1], p->background[2]);
  kp.seed = p->seed;
  kp.n_nodes = pl.fast ? 8 * s->f_stream_len : s->main_end;
  kp.n_prims = (uint32_t)(pl.fast ? s->f_prims.size() : s->g_prims.size());
  kp.stream_len = pl.fast ? s->f_stream_len : 0;
  kp.postpone = env_knob("HRT_POSTPONE", 60);
  kp.motion_uniform = s->motion_uniform ? 1u : 0u;
  kp.motion_t0 = s->motion_t0;
  kp.motion_span = s->motion_span;
  return kp;
}

}  // namespace

/* ============================================================================ device runtime */
namespace hrt {

hrt_status device_upload(hrt_scene* s, int device) {
  return hguard([&] {
    if (device < 0) hip_check(hipGetDevice(&device), "hipGetDevice");
    DeviceGuard dg(device);
    device_release(s);
    size_t off = 0;
    auto section = [&](size_t bytes) {
      size_t o = off;
      off = align256(off + std::max<size_t>(bytes, 16));
      return o;
    };
    s->off_nodes = section(s->g_nodes.size() * sizeof(G::Node));
    s->off_prims = section(s->g_prims.size() * sizeof(G::Prim));
    s->off_insts = section(s->g_insts.size() * sizeof(G::Inst));
    s->off_media = section(s->g_media.size() * sizeof(G::Medium));
    s->off_mats = section(s->g_mats.size() * sizeof(G::Mat));
    s->off_texs = section(s->g_texs.size() * sizeof(G::Tex));
    s->off_perlin = section(s->perlin.size() * sizeof(G::Perlin));
    s->off_images = section(s->images.size());
    s->off_fnodes = section(s->f_nodes.size() * sizeof(G::Node));
    s->off_fprims = section(s->f_prims.size() * sizeof(G::Prim));
    s->blob_bytes = off;
    std::vector<uint8_t> blob(off, 0);
    auto put = [&](size_t o, const void* src, size_t bytes) {
      if (bytes) memcpy(blob.data() + o, src, bytes);
    };
    put(s->off_nodes, s->g_nodes.data(), s->g_nodes.size() * sizeof(G::Node));
    put(s->off_prims, s->g_prims.data(), s->g_prims.size() * sizeof(G::Prim));
    put(s->off_insts, s->g_insts.data(), s->g_insts.size() * sizeof(G::Inst));
    put(s->off_media, s->g_media.data(), s->g_media.size() * sizeof(G::Medium));
    put(s->off_mats, s->g_mats.data(), s->g_mats.size() * sizeof(G::Mat));
    put(s->off_texs, s->g_texs.data(), s->g_texs.size() * sizeof(G::Tex));
    put(s->off_perlin, s->perlin.data(), s->perlin.size() * sizeof(G::Perlin));
    put(s->off_images, s->images.data(), s->images.size());
    put(s->off_fnodes, s->f_nodes.data(), s->f_nodes.size() * sizeof(G::Node));
    put(s->off_fprims, s->f_prims.data(), s->f_prims.size() * sizeof(G::Prim));
    s->device = device; /* from here on device_release() cleans up whatever was allocated */
    hip_check(hipMalloc(&s->d_blob, off), "hipMalloc(scene)");
    hip_check(hipMemcpy(s->d_blob, blob.data(), off, hipMemcpyHostToDevice), "hipMemcpy(scene)");
    s->slot_mutex = new std::mutex();
    for (auto& sl : s->slots) {
      hipEvent_t ev;
      hip_check(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate");
      sl.event = ev;
      sl.used = false;
      sl.tiles_cap = 0;
    }
  });
}

void device_release(hrt_scene* s) {
  if (!s || s->device < 0) return;
  int prev = -1;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(s->device);
  for (auto& sl : s->slots) {
    if (sl.event) {
      (void)hipEventSynchronize((hipEvent_t)sl.event);
      (void)hipEventDestroy((hipEvent_t)sl.event);
    }
    if (sl.d_mem) (void)hipFree(sl.d_mem);
    if (sl.d_partial) (void)hipFree(sl.d_partial);
    if (sl.h_tiles) (void)hipHostFree(sl.h_tiles);
    sl = hrt_scene::Slot();
  }
  delete static_cast<std::mutex*>(s->slot_mutex);
  s->slot_mutex = nullptr;
  if (s->d_blob) (void)hipFree(s->d_blob);
  s->d_blob = nullptr;
  if (prev >= 0) (void)hipSetDevice(prev);
  s->device = -1;
}

}  // namespace hrt

extern "C" {

hrt_status hrt_render_tiles_device(hrt_scene* s, const hrt_camera* cam, const hrt_render_params* p,
                                   const hrt_tile* tiles, uint32_t n_tiles, float* d_rgba, void* stream_,
                                   hrt_render_stats* stats) {
  return hguard([&] {
    if (!s || !cam || !p || !tiles || !d_rgba || n_tiles == 0)
      throw HipError{HRT_ERR_INVALID_ARG, "hrt_render_tiles_device: null argument"};
    if (!s->committed || !s->d_blob) throw HipError{HRT_ERR_STATE, "scene not committed"};
    if (p->width < 2 || p->height < 2 || p->width > 65535 || p->height > 65535 || p->samples == 0 || (p->flags & ~(uint32_t)(HRT_RENDER_COUNT_WORK | HRT_RENDER_NO_LDS | HRT_RENDER_REFERENCE_CULL |
                                     HRT_RENDER_FAST_CULL | HRT_RENDER_SAH)) != 0)
      throw HipError{HRT_ERR_INVALID_ARG, "bad render params (width/height >= 2, samples > 0, known flags)"};
    if (!(cam->time0 < cam->time1)) throw HipError{HRT_ERR_INVALID_ARG, "camera time0 must be < time1"};
    /* sample chunks: spp <= 32 keeps one work item per pixel (the reference's sequential sum);
     * larger spp splits into <= 16 chunks so the frame's tail is a chunk, not a whole pixel */
    const uint32_t spp = p->samples;
    const uint32_t chunk = spp <= 32 ? spp : std::max<uint32_t>(32, (spp + 15) / 16);
    const uint32_t n_chunks = (spp + chunk - 1) / chunk;
    std::vector<G::TileDev> td(n_tiles);
    uint64_t pad = 0, outp = 0;
    for (uint32_t i = 0; i < n_tiles; i++) {
      const hrt_tile& t = tiles[i];
      if (t.w == 0 || t.h == 0 || (uint64_t)t.x + t.w > p->width || (uint64_t)t.y + t.h > p->height)
        throw HipError{HRT_ERR_INVALID_ARG, "tile outside the image"};
      uint32_t bw = (t.w + 7) / 8, bh = (t.h + 7) / 8;
      td[i] = G::TileDev{t.x, t.y, t.w, t.h, bw, (uint32_t)pad, (uint32_t)outp, 0};
      pad += (uint64_t)bw * bh * 64 * n_chunks;
      outp += (uint64_t)t.w * t.h;
    }
    if (pad >= 0xFFFF0000ull) throw HipError{HRT_ERR_UNSUPPORTED, "more than 4G pixels in one call"};
    hipStream_t stream = (hipStream_t)stream_;
    DeviceGuard dg(s->device);
    /* scratch slot: device [counter u32 | pad | stats 8 x u64 | pad to HDR | tiles], pinned host [stats | tiles] */
    std::lock_guard<std::mutex> lock(*static_cast<std::mutex*>(s->slot_mutex));
    hrt_scene::Slot& sl = s->slots[s->next_slot++ % hrt_scene::N_SLOTS];
    if (sl.used) hip_check(hipEventSynchronize((hipEvent_t)sl.event), "hipEventSynchronize(slot)");
    size_t tiles_bytes = n_tiles * sizeof(G::TileDev);
    if (tiles_bytes > sl.tiles_cap) {
      if (sl.d_mem) hip_check(hipFree(sl.d_mem), "hipFree(slot)");
      if (sl.h_tiles) hip_check(hipHostFree(sl.h_tiles), "hipHostFree(slot)");
      sl.d_mem = sl.h_tiles = nullptr;
      sl.tiles_cap = 0;
      size_t cap = std::max<size_t>(tiles_bytes, 64 * sizeof(G::TileDev));
      hip_check(hipMalloc(&sl.d_mem, SLOT_HDR + cap), "hipMalloc(slot)");
      hip_check(hipHostMalloc(&sl.h_tiles, SLOT_HDR + cap, hipHostMallocDefault), "hipHostMalloc(slot)");
      sl.tiles_cap = cap;
    }
    const size_t partial_bytes = n_chunks > 1 ? (size_t)n_chunks * outp * sizeof(float4) : 0;
    if (partial_bytes > sl.partial_cap) {
      if (sl.d_partial) hip_check(hipFree(sl.d_partial), "hipFree(partial)");
      sl.d_partial = nullptr;
      sl.partial_cap = 0;
      hip_check(hipMalloc(&sl.d_partial, partial_bytes), "hipMalloc(partial)");
      sl.partial_cap = partial_bytes;
    }
    void* scratch = sl.d_mem;
    memcpy((uint8_t*)sl.h_tiles + SLOT_HDR, td.data(), tiles_bytes);
    hip_check(hipMemsetAsync(scratch, 0, SLOT_HDR, stream), "hipMemsetAsync");
    hip_check(hipMemcpyAsync((uint8_t*)scratch + SLOT_HDR, (uint8_t*)sl.h_tiles + SLOT_HDR, tiles_bytes, hipMemcpyHostToDevice,
                             stream), "hipMemcpyAsync(tiles)");
    const Plan pl = plan(s, cam, p->flags);
    KParams kp = scene_params(s, cam, p, pl);
    kp.tiles = (const G::TileDev*)((uint8_t*)scratch + SLOT_HDR);
    kp.n_tiles = n_tiles;
    kp.total_work = (uint32_t)pad;
    kp.out = (float4*)d_rgba;
    kp.counter = (uint32_t*)scratch;
    kp.stats = (unsigned long long*)((uint8_t*)scratch + 8);
    kp.chunk = chunk;
    kp.n_chunks = n_chunks;
    kp.n_out = (uint32_t)outp;
    kp.partial = (float4*)sl.d_partial;
    if (p->flags & HRT_RENDER_COUNT_WORK) launch_any<true>(s, pl, kp, stream);
    else launch_any<false>(s, pl, kp, stream);
    if (n_chunks > 1) {
      uint32_t blocks = (uint32_t)std::min<uint64_t>((outp + 255) / 256, 4096);
      hipLaunchKernelGGL(reduce_chunks, dim3(blocks), dim3(256), 0, stream, (const float4*)sl.d_partial,
                         (float4*)d_rgba, (uint32_t)outp, n_chunks, spp);
      hip_check(hipGetLastError(), "reduce_chunks launch");
    }
    unsigned long long* h = (unsigned long long*)sl.h_tiles;
    if (stats) hip_check(hipMemcpyAsync(h, (uint8_t*)scratch + 8, 96, hipMemcpyDeviceToHost, stream), "hipMemcpyAsync(stats)");
    hip_check(hipEventRecord((hipEvent_t)sl.event, stream), "hipEventRecord(slot)");
    sl.used = true;
    if (stats) {
      hip_check(hipEventSynchronize((hipEvent_t)sl.event), "hipEventSynchronize(stats)");
      stats->segments = h[0];
      stats->samples = h[1];
      stats->pixels = h[2];
      stats->node_visits = h[3];
      stats->prim_tests = h[4];
      stats->tex_evals = h[5];
      stats->walk_slots = h[6];
      stats->shade_slots = h[7];
      stats->prim_slots = h[8];
      for (int k = 0; k < 3; k++) stats->phase_cycles[k] = h[9 + k];
    }
  });
}

hrt_status hrt_render_device(hrt_scene* s, const hrt_camera* cam, const hrt_render_params* p, uint32_t x0,
                             uint32_t y0, uint32_t w, uint32_t h, float* d_rgba, void* stream,
                             hrt_render_stats* stats) {
  hrt_tile t{x0, y0, w, h};
  return hrt_render_tiles_device(s, cam, p, &t, 1, d_rgba, stream, stats);
}

hrt_status hrt_render(hrt_scene* s, const hrt_camera* cam, const hrt_render_params* p, uint32_t x0,
                      uint32_t y0, uint32_t w, uint32_t h, float* rgba_out, hrt_render_stats* stats) {
  if (!s || !rgba_out || !s->committed) {
    set_error("hrt_render: null argument or scene not committed");
    return (s && !s->committed) ? HRT_ERR_STATE : HRT_ERR_INVALID_ARG;
  }
  float* d_out = nullptr;
  hrt_status st = hguard([&] {
    DeviceGuard dg(s->device);
    hip_check(hipMalloc((void**)&d_out, (size_t)w * h * 16 + 16), "hipMalloc(out)");
  });
  if (st != HRT_OK) return st;
  hrt_render_stats local;
  st = hrt_render_device(s, cam, p, x0, y0, w, h, d_out, nullptr, stats ? stats : &local);
  if (st == HRT_OK) {
    st = hguard([&] {
      DeviceGuard dg(s->device);
      hip_check(hipMemcpy(rgba_out, d_out, (size_t)w * h * 16, hipMemcpyDeviceToHost), "hipMemcpy(out)");
    });
  }
  {
    int prev = -1;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(s->device);
    (void)hipFree(d_out);
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  return st;
}

hrt_status hrt_debug_trace_path(hrt_scene* s, const hrt_camera* cam, const hrt_render_params* p, uint32_t x,
                                uint32_t y, uint32_t sample, uint32_t max_segments, float* out, uint32_t* n_segments) {
  return hguard([&] {
    if (!s || !cam || !p || !out || !n_segments || max_segments == 0)
      throw HipError{HRT_ERR_INVALID_ARG, "hrt_debug_trace_path: bad argument"};
    if (!s->committed || !s->d_blob) throw HipError{HRT_ERR_STATE, "scene not committed"};
    if (x >= p->width || y >= p->height) throw HipError{HRT_ERR_INVALID_ARG, "pixel outside the image"};
    DeviceGuard dg(s->device);
    const Plan pl = plan(s, cam, p->flags);
    KParams kp = scene_params(s, cam, p, pl);
    size_t bytes = (9 * (size_t)max_segments + 3) * sizeof(float);
    float* d_out = nullptr;
    uint32_t* d_n = nullptr;
    hip_check(hipMalloc((void**)&d_out, bytes), "hipMalloc");
    hip_check(hipMalloc((void**)&d_n, 4), "hipMalloc");
    if (pl.fast) hipLaunchKernelGGL((debug_path_kernel<G::CULL_SLAB, false, true>), dim3(1), dim3(64), 0, 0, kp, x, y, sample, d_out, max_segments, d_n);
    else if (pl.full && pl.cull == G::CULL_EXACT) hipLaunchKernelGGL((debug_path_kernel<G::CULL_EXACT, true, false>), dim3(1), dim3(64), 0, 0, kp, x, y, sample, d_out, max_segments, d_n);
    else if (pl.cull == G::CULL_EXACT) hipLaunchKernelGGL((debug_path_kernel<G::CULL_EXACT, false, false>), dim3(1), dim3(64), 0, 0, kp, x, y, sample, d_out, max_segments, d_n);
    else if (pl.full && pl.cull == G::CULL_SLAB) hipLaunchKernelGGL((debug_path_kernel<G::CULL_SLAB, true, false>), dim3(1), dim3(64), 0, 0, kp, x, y, sample, d_out, max_segments, d_n);
    else if (pl.full) hipLaunchKernelGGL((debug_path_kernel<G::CULL_REFERENCE, true, false>), dim3(1), dim3(64), 0, 0, kp, x, y, sample, d_out, max_segments, d_n);
    else if (pl.cull == G::CULL_SLAB) hipLaunchKernelGGL((debug_path_kernel<G::CULL_SLAB, false, false>), dim3(1), dim3(64), 0, 0, kp, x, y, sample, d_out, max_segments, d_n);
    else hipLaunchKernelGGL((debug_path_kernel<G::CULL_REFERENCE, false, false>), dim3(1), dim3(64), 0, 0, kp, x, y, sample, d_out, max_segments, d_n);
    hip_check(hipGetLastError(), "debug_path_kernel launch");
    hip_check(hipMemcpy(out, d_out, bytes, hipMemcpyDeviceToHost), "hipMemcpy");
    hip_check(hipMemcpy(n_segments, d_n, 4, hipMemcpyDeviceToHost), "hipMemcpy");
    (void)hipFree(d_out);
    (void)hipFree(d_n);
  });
}

hrt_status hrt_debug_device_math(int32_t op, const float* x, const float* y, float* out, uint32_t n) {
  return hguard([&] {
    if (!x || !out || op < 0 || op > 7) throw HipError{HRT_ERR_INVALID_ARG, "bad argument"};
    if (n == 0) return;
    float *dx = nullptr, *dy = nullptr, *dout = nullptr;
    hip_check(hipMalloc((void**)&dx, n * 4), "hipMalloc");
    hip_check(hipMalloc((void**)&dout, n * 4), "hipMalloc");
    if (y) hip_check(hipMalloc((void**)&dy, n * 4), "hipMalloc");
    hip_check(hipMemcpy(dx, x, n * 4, hipMemcpyHostToDevice), "hipMemcpy");
    if (y) hip_check(hipMemcpy(dy, y, n * 4, hipMemcpyHostToDevice), "hipMemcpy");
    hipLaunchKernelGGL(math_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, op, dx, dy, dout, n);
    hip_check(hipGetLastError(), "math_kernel launch");
    hip_check(hipMemcpy(out, dout, n * 4, hipMemcpyDeviceToHost), "hipMemcpy");
    (void)hipFree(dx);
    (void)hipFree(dout);
    if (dy) (void)hipFree(dy);
  });
}

}  // extern "C"
