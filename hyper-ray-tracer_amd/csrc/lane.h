/*
 * lane.h — what ONE lane of the path-tracing kernels does: ray set-up, the box / sphere / rect tests,
 * the resumable world walks (basic_step, full_step, and trace() for the segment-at-a-time kernel),
 * hit records, textures, scattering and sample start.  Everything here is __host__ __device__:
 * render.hip's kernels schedule these functions over waves, and tests/native/lane_sim.hip runs the
 * same functions one lane at a time on the host, so the per-lane logic of the kernels is checked
 * against the CPU oracle without a GPU (wave scheduling cannot change a lane's result: a lane's
 * sequence of tests and draws depends only on its own state).
 */
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "hrt/hd_math.h"
#include "hrt/hrt.h"
#include "layout.h"

/* `inline` everywhere: lane.h is included by both kernel translation units (ODR) */
#define HRT_LANE __host__ __device__ inline
#define HRT_LANE_FI __host__ __device__ __forceinline__
#define HRT_LANE_NI __host__ __device__ inline __attribute__((noinline))

namespace hrt {
namespace lane {

namespace G = hrt::gpu;

HRT_LANE_FI uint32_t umax(uint32_t a, uint32_t b) { return a > b ? a : b; }

#ifndef HRT_EXP_PK
#define HRT_EXP_PK 0 /* experiment: packed-f32 box test (A/B on the GPU before it becomes the default) */
#endif

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
  const float4* chains; /* layout.h CHAIN_F4 float4 per instance */
  uint32_t main_end;
  float ln_e;
  /* camera (camera.rs:16-31 after resize) */
  Vec3 cam_origin, cam_llc, cam_h, cam_v, cam_u, cam_vv;
  float lens_radius, time0, time1;
  /* render */
  uint32_t W, H, spp, max_depth, sample_offset;
  float rw1, rh1; /* RN(1 / (W - 1)), RN(1 / (H - 1)): set_pixel_rcp */
  float t_min;
  Vec3 background;
  uint64_t seed;
  /* work */
  const G::TileDev* tiles;
  uint32_t n_tiles;
  uint32_t total_work;
  uint32_t tile_stride; /* > 0: every tile's items padded to this many (tile = item / stride) */
  float4* out;
  uint32_t* counter;
  uint32_t claim_fine; /* work items from here on are claimed one per lane (kernel_common.h claim_work) */
  unsigned long long* stats; /* segments, samples, pixels, then (COUNT builds) nodes, prims, tex */
  /* sample chunks: a work item is (pixel, chunk of consecutive samples); lane.h chunk_range */
  uint32_t chunk, n_chunks, n_out;
  uint32_t chunk_head, chunk_first; /* head chunks (the first holds chunk_first samples, the rest `chunk`) */
  uint32_t pad_px;                  /* padded pixels of the call's tiles */
  uint32_t head_items;              /* pad_px x chunk_head: the head chunks' items come first (claim_work) */
  uint32_t n_prims;
  uint32_t n_nodes;    /* node-stream entries to stage in LDS */
  uint32_t stream_len; /* FAST: length of one octant stream */
  uint32_t postpone;   /* BASIC kernel: lanes that must have finished their walk before a wave shades */
  uint32_t prim_batch; /* BASIC kernel: lanes that must wait for a primitive test before the wave runs them */
  uint32_t walk_cap;   /* watchdog: more consecutive walk-loop iterations than any valid walk needs */
  uint32_t motion_uniform; /* every moving sphere has time0 = motion_t0, time1 - time0 = motion_span */
  float motion_t0, motion_span;
  float4* partial; /* [n_chunks][n_out] chunk sums (n_chunks > 1): a claim's 64 lanes write one chunk of 64
                      consecutive pixels, whole cache lines (r05; [n_out][n_chunks] wrote 2.35x the sums' bytes
                      on Final, 16-B writes into lines a wave completes only chunks later) */
  /* sphere-scene walk stream (layout.h; render_basic_kernel under CULL_EXACT) */
  const uint8_t* walk;
  uint32_t walk_bytes; /* whole stream */
  uint32_t walk_end;   /* byte offset one past the last record */
  uint32_t walk_hot;   /* WM_HYB: offsets below this are staged in LDS (layout.h placement) */
  uint32_t lane_lds;   /* sphere kernel: LDS byte offset of the per-lane result slots (after the staged scene) */
  uint32_t n_insts, n_media, n_mats, n_texs; /* record counts (render_gwalk_kernel stages them in LDS) */
  uint32_t n_perlin;   /* Perlin tables (12 KB each); perlin_lds: the kernel stages them in LDS (stage_perlin) */
  uint32_t perlin_lds;
  uint32_t walk_half;  /* the walk stream's node-part split (layout.h WALK_SPLIT_HALF) or 16 */
  uint32_t walk_c16;   /* 16-B node parts (layout.h WALK_C16): walk_end is then the node count */
  uint32_t walk_pbase; /* walk_c16: byte offset of the payloads */
};

/* Sample-chunk size: spp <= cmin keeps one work item per pixel (the reference's sequential sum), larger
 * spp splits into at most cdiv chunks of >= cmin samples.  The defaults depend on spp and on the scene's
 * class alone (never on the tile split), so every split sums a pixel's samples in the same chunks.  A
 * chunk should be long enough that claiming it and writing its partial sum are cheap next to its
 * samples, and short enough that the launch's last items (run with the device mostly idle) end soon:
 * - sphere scenes (render_basic_kernel: block claims, short passes): >= 16 samples, <= 32 chunks;
 * - general scenes: <= 8 chunks of >= 32 samples; when the main node stream is deep (> 1024 nodes:
 *   expensive samples of very uneven length) <= 64 chunks of >= 1 sample.
 * Measured: Earth+Perlin 1000 spp 11447 Mrays/s with 8 chunks vs 9703 with 32;
 * at 128 spp min 64 / 32 / 16 = 8934 / 9931 / 7930; Cornell 64 spp 6900 / 6971 / 6963; Cornell's 1/8 share
 * at 10000 spp flat over 8 .. 512 chunks (r04); Final 800^2 x 64 spp (r04, general walk kernel) chunk 16 /
 * 8 / 4 / 2 / 1 = 1794 / 2300 / 2669 / 3001 / 3104 (r02, segment kernel: 64 / 32 / 16 = 548 / 735 / 928). */
enum ChunkClass : uint32_t { CHUNK_SPHERE = 0, CHUNK_GENERAL = 1, CHUNK_GENERAL_DEEP = 2 };
inline uint32_t chunk_class(uint32_t feature_mask, uint32_t main_nodes) {
  if ((feature_mask & ~G::F_BASIC) == 0) return CHUNK_SPHERE;
  return main_nodes > 1024u ? CHUNK_GENERAL_DEEP : CHUNK_GENERAL;
}
inline uint32_t sample_chunk(uint32_t spp, uint32_t cls, uint32_t cmin = 0, uint32_t cdiv = 0) {
  if (cmin == 0) cmin = cls == CHUNK_GENERAL ? 32u : (cls == CHUNK_SPHERE ? 16u : 1u);
  if (cdiv == 0) cdiv = cls == CHUNK_SPHERE ? 32u : (cls == CHUNK_GENERAL ? 8u : 64u);
  const uint32_t even = (spp + cdiv - 1) / cdiv;
  return spp <= cmin ? spp : (even > cmin ? even : cmin);
}

/* The chunks of a pixel's spp samples (r03): HEAD chunks of c samples (the first holds the remainder r),
 * then a TAIL of halving chunks c/2, c/2, c/4, c/4, ..., 1, 1.  The tail's items run last, chunk-major
 * (kernel_common.h claim_work), so a launch ends on short items instead of full chunks: the last
 * items run with the device mostly idle, and their length was the loss of small launches (one GPU's
 * 1/8 share of C2 ran at 84% of the whole frame's rate with uniform 16-sample chunks).  The schedule
 * depends on spp and c alone, so every tile split sums a pixel's samples in the same chunks, added in
 * chunk order.  No tail when it would leave less than one head chunk, or with tail = false. */
inline void chunk_plan(uint32_t spp, uint32_t c, uint32_t levels, uint32_t& n_head, uint32_t& first, uint32_t& n_tail) {
  uint32_t T = 0, L = 0;
  if (levels && spp > c)
    for (uint32_t m = 1; (c >> m) >= 1u && m <= levels; m++) {
      T += 2u * (c >> m);
      L++;
    }
  if (T > 0 && (spp - c < T)) T = L = 0; /* spp - T < c */
  const uint32_t H = spp - T;
  n_head = (H + c - 1) / c;
  first = H - (n_head - 1) * c;
  n_tail = 2u * L;
}

/* The chunk schedule of a render: sample_chunk + chunk_plan, with the chunk doubled while the partial sums
 * of a whole frame (n_chunks x W x H x 16 B) would exceed CHUNK_PARTIAL_BUDGET (one-sample chunks
 * of a deep general scene at 3840x2160 would need 8.5 GB per in-flight launch).  The cap depends on the FULL
 * image size, never on the tile split, so every split still sums a pixel's samples in the same chunks.  No
 * BASELINE configuration reaches it (C4, the largest: 40 chunks x 133 MB = 5.3 GB). */
constexpr unsigned long long CHUNK_PARTIAL_BUDGET = 6ull << 30;
inline void frame_chunks(uint32_t spp, uint32_t cls, uint32_t W, uint32_t H, uint32_t cmin, uint32_t cmax, uint32_t levels,
                         uint32_t& c, uint32_t& n_head, uint32_t& first, uint32_t& n_tail) {
  c = sample_chunk(spp, cls, cmin, cmax);
  const unsigned long long frame = (unsigned long long)W * H * 16u;
  for (;;) {
    chunk_plan(spp, c, levels, n_head, first, n_tail);
    if (n_head + n_tail <= 1 || (unsigned long long)(n_head + n_tail) * frame <= CHUNK_PARTIAL_BUDGET || c >= spp) return;
    c = c > spp / 2 ? spp : 2 * c;
  }
}

/* samples [s0, s1) of chunk k */
HRT_LANE_FI void chunk_range(const KParams& P, uint32_t k, uint32_t& s0, uint32_t& s1) {
  if (k < P.chunk_head) {
    s0 = k == 0 ? 0u : P.chunk_first + (k - 1u) * P.chunk;
    s1 = P.chunk_first + k * P.chunk;
    return;
  }
  const uint32_t j = k - P.chunk_head;
  uint32_t s = P.chunk_first + (P.chunk_head - 1u) * P.chunk;
  for (uint32_t i = 0; i < j; i++) s += P.chunk >> (1u + (i >> 1));
  s0 = s;
  s1 = s + (P.chunk >> (1u + (j >> 1)));
}

/* per-lane work counters of the instrumented (COUNT) instantiation */
struct Counts {
  uint32_t nodes, prims, tex;
  uint32_t walk_slots, shade_slots; /* lane slots of wave iterations: walk (node) loop, shading passes */
  uint32_t prim_slots;              /* lane slots of wave executions of the primitive block */
  uint32_t park_slots, wait_slots;  /* sphere kernel walk steps: lanes parked on a leaf / done, waiting to shade */
  uint32_t steps;                   /* walk kernels: lane slots of the walk loop that stepped a node (nodes also counts
                                       the nodes leaf programs test) */
};

struct TRay {
  Vec3 o, d, inv;
  Vec3 noinv; /* -(o * inv) per axis for the walk's inflated test (box_ce); NaN in all three when an inv
                 or a product is not a finite normal number (every inflated test then passes) */
  float time;
  float dd;  /* dot(d, d): sphere.rs:42 `a`, constant for the ray */
  float rdd; /* RN(1 / dd) for div_rn, or NaN when dd is outside div_rn's fast domain */
  float tau; /* (time - time0) / (time1 - time0) of the scene's moving spheres under uniform motion, else the
               time itself: the walks read only this field (one register for both) */
};

/* x / r.dd correctly rounded (bit-identical to IEEE division) by a 3-instruction core: with
 * y = RN(1/a), q0 = RN(x*y) is within one ulp of x/a, the
 * residual x - q0*a is exact in an fma, and RN(q0 + residual*y) is RN(x/a) (Markstein's theorem;
 * no under/overflow anywhere while |x|, |q0|, a lie in [2^-100, 2^100]).  Zero, NaN, inf and
 * extreme exponents take the IEEE sequence.  tests/test_fast_division.py checks 6e7 cases on the host
 * and 4e6 on the device (3e9 more were checked while writing it).
 * The domain test is split so that one check per call remains: the per-ray y is NaN unless
 * a in [2^-49, 2^49] (div_rn_y), and the call checks |q0| in [2^-50, 2^50].  Together they imply
 * |x| = |q0 a| (1 +- 2^-23) in [2^-100, 2^100], so this domain lies inside the one above; a NaN y
 * fails the |q0| check.  Default build (HRT_DIV_VOTE 0): the IEEE fallback is if-converted, so a call
 * executes the core AND the ~11-instruction IEEE sequence and selects (measured cheaper than a
 * branch); HRT_DIV_VOTE 1 puts the fallback behind a wave vote instead.  Only the camera divisions
 * (start_sample) run the bare 3-instruction core, with no fallback. */
HRT_LANE_FI float div_rn_y(float a) { return a >= 0x1p-49f && a <= 0x1p49f ? rcp_fast(a) : u2f(0x7fc00000u); }
HRT_LANE_FI float div_rn(float x, float a, float y) {
  const float q0 = x * y;
  float q = fmaf(fmaf(-q0, a, x), y, q0);
  const float aq = fabsf(q0);
  const bool fast = aq >= 0x1p-50f && aq <= 0x1p50f;
#ifndef HRT_DIV_VOTE
#define HRT_DIV_VOTE 0 /* measured: the vote costs more than the if-converted IEEE sequence */
#endif
#if defined(__HIP_DEVICE_COMPILE__) && HRT_DIV_VOTE
  if (__any(!fast)) {
    if (!fast) q = x / a;
  }
#else
  if (!fast) q = x / a;
#endif
  return q;
}

/* r.noinv from r.o and r.inv, or NaN in all three components (NaN MODE: no inflated culling for this
 * ray, every inflated test passes; the reference tests still decide).  NaN mode when an inv component is
 * not a finite normal number or a product is not finite:
 *  - box_ce's D is exact only for a normal |inv| (a zero or denormal inv drops its axis from D);
 *  - a direction component of 0 (inv infinite) is also the only way a reference test can accept a NaN t:
 *    rect.rs:61-70 divides (k - o_k) by d_k, and with the origin ON the rect's plane and the ray parallel to
 *    it that is 0 / 0; NaN passes `t < t_min || t > t_max` and the bounds checks, so the reference accepts
 *    a "hit" at t = NaN wherever the rect lies along the ray, beyond the closest hit too (DESIGN G20).  No
 *    inflated box can hold such a hit, so the walk must not cull for this ray at all. */
HRT_LANE_FI void set_noinv(TRay& r) {
  r.noinv = v3(-(r.o.x * r.inv.x), -(r.o.y * r.inv.y), -(r.o.z * r.inv.z));
  auto normal = [](float x) { return (int)(fabsf(x) >= 0x1p-126f) & (int)(fabsf(x) <= 3.40282347e+38f); }; /* 0 on NaN */
  auto finite = [](float x) { return (int)(fabsf(x) <= 3.40282347e+38f); };
  if (!(normal(r.inv.x) & normal(r.inv.y) & normal(r.inv.z) & finite(r.noinv.x) & finite(r.noinv.y) & finite(r.noinv.z)))
    r.noinv = v3(u2f(0x7fc00000u), u2f(0x7fc00000u), u2f(0x7fc00000u));
}
HRT_LANE_FI bool nan_mode(const TRay& r) { return r.noinv.x != r.noinv.x; }

/* a new origin/direction; the ray keeps its time */
/* (1/d.x, 1/d.y, 1/d.z) with IEEE division's bits (hd_math.h rcp_fast): one wave vote for the three; the lanes
 * with a component outside the fast range (a zero, denormal or huge component) divide */
HRT_LANE_FI Vec3 inv_rn(Vec3 d) {
  Vec3 q = v3(rcp_fast(d.x), rcp_fast(d.y), rcp_fast(d.z));
#if defined(__HIP_DEVICE_COMPILE__) && HRT_RCP_FAST
  const bool ok = (int)rcp_fast_domain(d.x) & (int)rcp_fast_domain(d.y) & (int)rcp_fast_domain(d.z);
  if (__builtin_amdgcn_ballot_w64(!ok)) {
    if (!ok) q = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  }
#endif
  return q;
}

HRT_LANE_FI void set_dir(TRay& r, Vec3 o, Vec3 d) {
  r.o = o;
  r.d = d;
  /* aabb.rs:22 computes 1/d per call; the value is the same every time */
  r.inv = inv_rn(d);
  set_noinv(r);
  r.dd = dot(d, d);
  r.rdd = div_rn_y(r.dd);
}

HRT_LANE_FI void set_time(TRay& r, float time, const KParams& P) {
  r.time = time;
  /* moving_sphere.rs:55-58: identical for every moving sphere when they share time0/time1 */
  r.tau = P.motion_uniform ? (time - P.motion_t0) / P.motion_span : time;
}

HRT_LANE_FI void set_ray(TRay& r, Vec3 o, Vec3 d, float time, const KParams& P) {
  set_dir(r, o, d);
  set_time(r, time, P);
}

HRT_LANE_FI float4 ld4(const void* p) { return *reinterpret_cast<const float4*>(p); }

/* ------------------------------------------------------------------ the sphere-scene walk stream */
/* The walk of render_basic_kernel under CULL_EXACT, over the walk stream (layout.h): positions are
 * byte offsets, read from LDS (the stream staged at LDS address 0), from global memory through a buffer
 * descriptor (32-bit offsets, no 64-bit address arithmetic per step), or from a host pointer (the lane
 * simulator). */
enum : int { WM_LDS = 0, WM_BUF = 1, WM_HOST = 2, WM_HYB = 3 /* LDS below `hot`, global memory above */ };
struct WalkSrc {
  const uint8_t* base; /* WM_BUF: the section in global memory; WM_HOST: the host copy */
  uint32_t hot;        /* WM_HYB */
  uint32_t half = 16;  /* WM_HOST: bytes from a node part's first 16 B to its second (the kernels: a template
                          constant, layout.h WALK_SPLIT_HALF or 16) */
#if defined(__HIP_DEVICE_COMPILE__)
  __amdgpu_buffer_rsrc_t rsrc; /* WM_BUF */
#endif
};

template <int MEM>
HRT_LANE_FI float4 wload(const WalkSrc& src, uint32_t off) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (MEM == WM_LDS) {
    typedef __attribute__((address_space(3))) const float4 lds_float4;
    return *(const lds_float4*)(size_t)off;
  } else if constexpr (MEM == WM_BUF) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v v = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(src.rsrc, (int)off, 0, 0));
    return make_float4(v.x, v.y, v.z, v.w);
  } else if constexpr (MEM == WM_HYB) {
    if (off < src.hot) return wload<WM_LDS>(src, off);
    return wload<WM_BUF>(src, off);
  }
#endif
  return *reinterpret_cast<const float4*>(src.base + off);
}

/* Where a walk stream's leaf PAYLOADS are read: a hybrid stream stages node parts only (scene.cpp
 * walk_place_and_write puts every payload behind them, in global memory), so its payloads are plain
 * buffer reads, with no per-lane choice between LDS and global memory */
template <int MEM>
constexpr int payload_mem() { return MEM == WM_HYB ? WM_BUF : MEM; }

#ifndef HRT_HYB_ANYG
#define HRT_HYB_ANYG 2 /* 2: the buffer loads under the exec mask of the lanes that need them (r04: C4 1/8 share at
                          * 256 spp 5330 -> 5621 Mrays/s over 1, profiles/r04g_ab.txt); 1: skipped when no
                          * lane of the wave needs them (5291 -> 5424 over 0); 0: every lane issues them */
#endif
/* Both 16-B halves of the node part at `off` (walk_box).  WM_HYB: every lane issues an LDS read AND a
 * buffer read of each half, into registers of their own, and keeps one by a select: the LDS lanes' buffer
 * offset lies beyond the descriptor's range (no memory access; zeros), the global lanes read LDS address 0
 * (a broadcast).  The per-lane branch of wload<WM_HYB> made the compiler wait for the buffer load before
 * the LDS read that writes the same registers: two serialised L2 latencies per step. */
template <int MEM, uint32_t HALF = 16>
HRT_LANE_FI void wload_node(const WalkSrc& src, uint32_t off, float4& a, float4& b) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (MEM == WM_HYB) {
    const bool in_lds = off < src.hot;
    const uint32_t loff = in_lds ? off : 0u;
    [[maybe_unused]] const uint32_t goff = in_lds ? 0x7FFFFF00u : off;
    const float4 la = wload<WM_LDS>(src, loff), lb = wload<WM_LDS>(src, loff + HALF);
#if HRT_HYB_ANYG == 2
    /* the buffer loads only for the lanes that need them (exec mask), into registers of their own */
    float4 ga = make_float4(0.0f, 0.0f, 0.0f, 0.0f), gb = ga;
    if (!in_lds) {
      ga = wload<WM_BUF>(src, off);
      gb = wload<WM_BUF>(src, off + HALF);
    }
#elif HRT_HYB_ANYG
    /* the buffer loads only when a lane of the wave needs them (a wave-uniform branch) */
    float4 ga = make_float4(0.0f, 0.0f, 0.0f, 0.0f), gb = ga;
    if (__builtin_amdgcn_ballot_w64(!in_lds)) {
      ga = wload<WM_BUF>(src, goff);
      gb = wload<WM_BUF>(src, goff + HALF);
    }
#else
    const float4 ga = wload<WM_BUF>(src, goff), gb = wload<WM_BUF>(src, goff + HALF);
#endif
    a = in_lds ? la : ga;
    b = in_lds ? lb : gb;
    return;
  }
#endif
  a = wload<MEM>(src, off);
  b = wload<MEM>(src, off + (MEM == WM_HOST ? src.half : HALF));
}


/* ---- 16-B node parts (layout.h WALK_C16) ----
 * One 16-B read per node step instead of two (LDS, or under the exec mask of the lanes whose part lies beyond
 * the staged set in a hybrid stream); the box's six binary16 values are widened exactly to f32, so box_ce sees
 * the encoded box's own numbers; the links are 16-bit node indices. */
HRT_LANE_FI float h2f(uint32_t bits16) { return (float)__builtin_bit_cast(_Float16, (uint16_t)bits16); }
template <int MEM>
HRT_LANE_FI float4 wload_part16(const WalkSrc& src, uint32_t off) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (MEM == WM_HYB) { /* as wload_node: an LDS read for every lane, a buffer read for the global lanes */
    const bool in_lds = off < src.hot;
    const float4 l = wload<WM_LDS>(src, in_lds ? off : 0u);
    float4 g = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (!in_lds) g = wload<WM_BUF>(src, off);
    return in_lds ? l : g;
  }
#endif
  return wload<MEM>(src, off);
}
/* a walk position of a 16-B stream parked on a leaf (WALK_C16_LEAF | payload index) */
HRT_LANE_FI bool walk_pending16(uint32_t i) { return (i >> 15) == 1u; }
template <bool C16>
HRT_LANE_FI bool walk_pend(uint32_t i) {
  if constexpr (C16) return walk_pending16(i);
  return i - G::WALK_PEND < 0x7FFFFFFFu;
}
/* the payload offset of the leaf a lane is parked on */
template <bool C16>
HRT_LANE_FI uint32_t pend_payload(const KParams& P, uint32_t i) {
  if constexpr (C16) return P.walk_pbase + (i & G::WALK_C16_MAX) * G::WALK_PAYLOAD_BYTES;
  return i - G::WALK_PEND;
}

/* aabb.rs:20-47 (CULL_REFERENCE), its narrowed form (CULL_SLAB), or CULL_EXACT: the reference test
 * AND an inflated slab test that only rejects boxes no accepted hit can come from (layout.h).
 * `if t0 > t_min {t0} else {t_min}` (aabb.rs:30-35) is fmaxf(t0, t_min): in IEEE mode v_max_f32
 * returns the non-NaN operand exactly as the comparison form does (a NaN t0 leaves t_min), and the
 * forms differ at most in the sign of a zero, which the `t_max <= t_min` test (:36) cannot see. */
template <int CULL>
HRT_LANE_FI bool box_hit(const float4& a, const float4& b, const TRay& r, float tmin,
                                        float tmax, bool ref_only = false) {
  const float inv[3] = {r.inv.x, r.inv.y, r.inv.z};
  float dmn[3], dmx[3], t0[3], t1[3];
#if HRT_EXP_PK
  /* x and y in packed f32 (v_pk_add_f32 / v_pk_mul_f32: the same IEEE operations, two per issue) */
  typedef float f2 __attribute__((ext_vector_type(2)));
  const f2 oxy = {r.o.x, r.o.y}, ixy = {r.inv.x, r.inv.y};
  const f2 dmnxy = f2{a.x, a.y} - oxy, dmxxy = f2{b.x, b.y} - oxy;
  const f2 t0xy = dmnxy * ixy, t1xy = dmxxy * ixy;
  dmn[0] = dmnxy.x; dmn[1] = dmnxy.y; dmn[2] = a.z - r.o.z;
  dmx[0] = dmxxy.x; dmx[1] = dmxxy.y; dmx[2] = b.z - r.o.z;
  t0[0] = t0xy.x; t0[1] = t0xy.y; t0[2] = dmn[2] * inv[2];
  t1[0] = t1xy.x; t1[1] = t1xy.y; t1[2] = dmx[2] * inv[2];
#else
  const float mn[3] = {a.x, a.y, a.z}, mx[3] = {b.x, b.y, b.z};
  const float o[3] = {r.o.x, r.o.y, r.o.z};
#pragma unroll
  for (int k = 0; k < 3; k++) {
    dmn[k] = mn[k] - o[k];
    dmx[k] = mx[k] - o[k];
    t0[k] = dmn[k] * inv[k];
    t1[k] = dmx[k] * inv[k];
  }
#endif
  float ts[3], te[3];
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const bool neg = inv[k] < 0.0f; /* aabb.rs:28-29 swap */
    ts[k] = neg ? t1[k] : t0[k];
    te[k] = neg ? t0[k] : t1[k];
  }
  if (CULL == G::CULL_SLAB) {
    const float lo = fmaxf(fmaxf(fmaxf(ts[0], tmin), ts[1]), ts[2]);
    const float hi = fminf(fminf(fminf(te[0], tmax), te[1]), te[2]);
    return !(hi <= lo);
  }
  bool ok = true; /* the reference: each axis on its own against [t_min, t_max] */
#pragma unroll
  for (int k = 0; k < 3; k++) ok = ok & !(fminf(te[k], tmax) <= fmaxf(ts[k], tmin));
  /* aabb.rs:30-36 with a NaN t_max (the closest after a NaN hit, G20) or t_min (a medium's second boundary
   * walk after a NaN first hit): `if te < t_max {te} else {t_max}` keeps the NaN and `t_max <= t_min` is
   * false, so every axis passes; fminf / fmaxf would drop the NaN instead */
  ok = ok | (tmax != tmax) | (tmin != tmin);
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
  return ok & (ref_only | nan_mode(r) | !(hi < lo));
}

/* The two halves of CULL_EXACT on their own, for the sphere-scene walk (basic_box / basic_prim).
 *
 * The reference test is MONOTONE under box inclusion: a BVH box contains its children's boxes
 * (Aabb::surrounding_box), so per axis a child's [ts, te] lies inside its parent's (the products
 * (mn - o) * inv round monotonically; a NaN axis, 0 * inf, passes as "no constraint" for every box
 * with that face, see box_hit), and closest only shrinks along the walk.  So if the reference fails an
 * inner node, it fails every leaf below it, at any later closest.  The walk can therefore apply the
 * reference test at LEAVES only (right before the primitive test) and cull inner nodes with the
 * inflated test alone: it tests exactly the primitives the exact walk tests, in the same order, with
 * the same closest. */
HRT_LANE_FI bool box_ref(const float4& a, const float4& b, const TRay& r, float tmin, float tmax) {
  const float mn[3] = {a.x, a.y, a.z}, mx[3] = {b.x, b.y, b.z};
  const float o[3] = {r.o.x, r.o.y, r.o.z}, inv[3] = {r.inv.x, r.inv.y, r.inv.z};
  bool ok = true;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const float t0 = (mn[k] - o[k]) * inv[k], t1 = (mx[k] - o[k]) * inv[k];
    const bool neg = inv[k] < 0.0f; /* aabb.rs:28-29 */
    const float ts = neg ? t1 : t0, te = neg ? t0 : t1;
    ok = ok & !(fminf(te, tmax) <= fmaxf(ts, tmin));
  }
  return ok | (tmax != tmax) | (tmin != tmin); /* a NaN bound passes every axis (box_hit) */
}

/* sphere.rs:38-55 / moving_sphere.rs:61-78 for a sphere of centre c (at the ray's time) and radius
 * `radius`: the accepted root only */
HRT_LANE_FI bool sphere_root_at(Vec3 c, float radius, const TRay& r, float tmin, float tmax, float& root) {
  Vec3 oc = r.o - c;
  float a = r.dd;
  float half_b = dot(oc, r.d);
  float cc = dot(oc, oc) - radius * radius;
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

/* constant_medium.rs:37-48 on a boundary that is one sphere: boundary.hit(ray, -inf, inf) and then
 * boundary.hit(ray, t1 + 0.0001, inf) from ONE evaluation of the quadratic (sphere.rs:38-55: oc, half_b,
 * c, the discriminant, its root and the two candidate roots are the same numbers in both calls; only the
 * accepted interval differs, and each call's comparisons are made exactly as sphere_root_at makes them).
 * Returns the number of boundary hits (0, 1 or 2) with t1, t2. */
HRT_LANE_FI int sphere_pair_at(Vec3 c, float radius, Vec3 o, Vec3 d, float& t1, float& t2) {
  const float inf = u2f(0x7f800000u);
  Vec3 oc = o - c;
  float a = dot(d, d); /* set_dir's r.dd */
  const float y = div_rn_y(a);
  float half_b = dot(oc, d);
  float cc = dot(oc, oc) - radius * radius;
  float disc = half_b * half_b - a * cc;
  if (disc < 0.0f) return 0;
  float sq = sqrtf(disc);
  const float near = div_rn(-half_b - sq, a, y);
  float t = near; /* the first call accepts its first root: (t < -inf || inf < t) is false */
  if (t < -inf || inf < t) {
    t = div_rn(-half_b + sq, a, y);
    if (t < -inf || inf < t) return 0;
  }
  t1 = t;
  const float tmin2 = t1 + 0.0001f;
  t = near;
  if (t < tmin2 || inf < t) {
    t = div_rn(-half_b + sq, a, y);
    if (t < tmin2 || inf < t) return 1;
  }
  t2 = t;
  return 2;
}

/* sphere.rs:38-55 / moving_sphere.rs:61-78: the accepted root only */
/* the record's p0, p1 and p2[0] already in registers (gwalk_one) */
HRT_LANE_FI bool sphere_root_v(const float4 p0, const float4 p1, float p2x, uint32_t kind, const TRay& r, float tmin,
                               float tmax, float& root, bool motion_uniform) {
  Vec3 c = v3(p0.x, p0.y, p0.z);
  if (kind == G::P_MOVING) {
    const float f = motion_uniform ? r.tau : (r.tau - p1.w) / p2x; /* r.tau: the time (TRay) */
    c = c + f * v3(p1.x, p1.y, p1.z);
  }
  return sphere_root_at(c, p0.w, r, tmin, tmax, root);
}

HRT_LANE_FI bool sphere_root(const G::Prim* pp, uint32_t kind, const TRay& r, float tmin,
                                            float tmax, float& root, bool motion_uniform) {
  const float4 p0 = ld4(pp->p0);
  if (kind != G::P_MOVING) return sphere_root_v(p0, p0, 0.0f, kind, r, tmin, tmax, root, motion_uniform);
  return sphere_root_v(p0, ld4(pp->p1), pp->p2[0], kind, r, tmin, tmax, root, motion_uniform);
}

/* Component i of v, and v with components a and b replaced, by selects: writing through Vec3's
 * runtime-indexed operator[] (a reference to a member chosen at run time) puts the vector in scratch
 * memory on the GPU, which in the walk loop cost more than all its arithmetic. */
HRT_LANE_FI float comp(const Vec3& v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }
HRT_LANE_FI Vec3 with2(Vec3 v, int a, float va, int b, float vb) {
  v.x = a == 0 ? va : (b == 0 ? vb : v.x);
  v.y = a == 1 ? va : (b == 1 ? vb : v.y);
  v.z = a == 2 ? va : (b == 2 ? vb : v.z);
  return v;
}

HRT_LANE_FI void plane_axes(uint32_t plane, int& k, int& a, int& b) {
  /* rect.rs:55-59 */
  if (plane == HRT_PLANE_XY) { k = 2; a = 0; b = 1; }
  else if (plane == HRT_PLANE_YZ) { k = 0; a = 1; b = 2; }
  else { k = 1; a = 2; b = 0; }
}

/* rect.rs:53-68 (p0 and k = p1[0] of the record) */
/* rect.rs:61-70 with the plane's axes fixed at compile time */
template <int K, int A, int B>
HRT_LANE_FI bool rect_axes(const float4 p0, float kk, const TRay& r, float tmin, float tmax, float& tout) {
  float t = (kk - comp(r.o, K)) / comp(r.d, K);
  if (t < tmin || t > tmax) return false;
  float av = comp(r.o, A) + t * comp(r.d, A);
  float bv = comp(r.o, B) + t * comp(r.d, B);
  if (av < p0.x || av > p0.y || bv < p0.z || bv > p0.w) return false;
  tout = t;
  return true;
}
#ifndef HRT_RECT_SPECIAL
#define HRT_RECT_SPECIAL 0 /* 1: a wave whose lanes test rects of one plane runs rect_axes for it (as rotate_any) */
#endif
HRT_LANE_FI bool rect_tv(const float4 p0, float kk, uint32_t plane, const TRay& r, float tmin, float tmax, float& tout) {
#if HRT_RECT_SPECIAL && defined(__HIP_DEVICE_COMPILE__)
  const uint32_t pw = __builtin_amdgcn_readfirstlane(plane);
  if (!__builtin_amdgcn_ballot_w64(plane != pw)) {
    if (pw == HRT_PLANE_XY) return rect_axes<2, 0, 1>(p0, kk, r, tmin, tmax, tout);
    if (pw == HRT_PLANE_YZ) return rect_axes<0, 1, 2>(p0, kk, r, tmin, tmax, tout);
    return rect_axes<1, 2, 0>(p0, kk, r, tmin, tmax, tout);
  }
#endif
  int k, a, b;
  plane_axes(plane, k, a, b);
  float t = (kk - comp(r.o, k)) / comp(r.d, k);
  if (t < tmin || t > tmax) return false;
  float av = comp(r.o, a) + t * comp(r.d, a);
  float bv = comp(r.o, b) + t * comp(r.d, b);
  if (av < p0.x || av > p0.y || bv < p0.z || bv > p0.w) return false;
  tout = t;
  return true;
}

HRT_LANE_FI bool rect_t(const G::Prim* pp, uint32_t plane, const TRay& r, float tmin, float tmax, float& tout) {
  return rect_tv(ld4(pp->p0), pp->p1[0], plane, r, tmin, tmax, tout);
}

/* rotation.rs:104-117 about axis AX (a, b the axes after it): the components picked at compile time */
template <int AX>
HRT_LANE_FI void rotate_axis(float s, float c, Vec3& o, Vec3& d) {
  constexpr int a = (AX + 1) % 3, b = (AX + 2) % 3;
  const float oa = comp(o, a), ob = comp(o, b), da = comp(d, a), db = comp(d, b);
  o = with2(o, a, c * oa + s * ob, b, -s * oa + c * ob);
  d = with2(d, a, c * da + s * db, b, -s * da + c * db);
}
/* The same operations for a per-lane axis.  HRT_ROT_SPECIAL 1 (default): a wave whose lanes all turn about y (every
 * reference scene: RotateY only) runs rotate_axis<1>, its components fixed at compile time, instead of the run-time
 * axis arithmetic and the component selects of the generic form below; 2: one branch per axis (more registers);
 * 0: the generic form only.  Same operations on the same operands, so the bits are the same
 * (tests/test_lane_sim.py::test_rotation_forms_bit_identical).  r06: C5's 1/8 share +7.6%, Final +3.2%
 * (profiles/r06_rotation_ab.txt). */
#ifndef HRT_ROT_SPECIAL
#define HRT_ROT_SPECIAL 1
#endif
HRT_LANE_FI void rotate_any(uint32_t axis, float s, float c, Vec3& o, Vec3& d) {
#if HRT_ROT_SPECIAL == 1 && defined(__HIP_DEVICE_COMPILE__)
  if (!__builtin_amdgcn_ballot_w64(axis != 1u)) { /* every lane about y */
    rotate_axis<1>(s, c, o, d);
    return;
  }
#elif HRT_ROT_SPECIAL == 2
  if (axis == 1u) rotate_axis<1>(s, c, o, d);
  else if (axis == 0u) rotate_axis<0>(s, c, o, d);
  else rotate_axis<2>(s, c, o, d);
  return;
#endif
  const int a = (int)(axis + 1) % 3, b = (int)(axis + 2) % 3;
  const float oa = comp(o, a), ob = comp(o, b), da = comp(d, a), db = comp(d, b);
  o = with2(o, a, c * oa + s * ob, b, -s * oa + c * ob);
  d = with2(d, a, c * da + s * db, b, -s * da + c * db);
}

/* translation.rs:26-30 and rotation.rs:104-117: the ray handed to the child */
HRT_LANE_FI void inst_ray(const G::Inst& in, Vec3& o, Vec3& d) {
  if ((in.kind & G::I_KIND_MASK) == G::I_TRANSLATE) {
    o = o - v3(in.d[0], in.d[1], in.d[2]);
    return;
  }
  rotate_any(in.axis, in.sin_t, in.cos_t, o, d);
}

/* The ray in the frame of instance q's children: the world ray through q's enclosing chain, outermost
 * first, exactly as the walk transformed it on the way in (translation.rs:26-30, rotation.rs:104-117).
 * Parent links are followed instead of keeping a per-lane stack (chains are short). */
/* one level of a chain record (layout.h CHAIN_F4): the operations of inst_ray */
HRT_LANE_FI void chain_level(const float4 v, Vec3& o, Vec3& d) {
  if (f2u(v.w) == G::I_TRANSLATE) {
    o = o - v3(v.x, v.y, v.z);
    return;
  }
  rotate_any(f2u(v.z), v.x, v.y, o, d);
}

/* the first `levels` levels of instance q's chain (all of them: q's children's frame) */
HRT_LANE_FI void apply_chain_levels(const KParams& P, uint32_t q, uint32_t levels, Vec3& o, Vec3& d) {
  const float4* c = P.chains + (size_t)q * G::CHAIN_F4;
  for (uint32_t l = 0; l < levels; l++) chain_level(c[1 + l], o, d);
}

HRT_LANE_FI void apply_chain(const KParams& P, uint32_t q, Vec3& o, Vec3& d) {
  if (q == G::NONE) return;
  apply_chain_levels(P, q, f2u(P.chains[(size_t)q * G::CHAIN_F4].x), o, d);
}

/* The walk enters instance `in` (K_INST_BEGIN): the ray of its children's frame.  set_dir's derived
 * fields are recomputed only when the frame changes them and the subtree reads them (layout.h IF_*):
 * a Translation keeps d, so 1/d and d.d stay; a Rotation whose subtree holds only rects needs none of
 * them.  Fields left alone keep the enclosing frame's values, which every instance below restores on
 * its way out, so they are right again when the walk leaves this instance. */
HRT_LANE_FI void inst_enter(const G::Inst& in, TRay& r) {
  Vec3 no = r.o, nd = r.d;
  inst_ray(in, no, nd);
  r.o = no;
  if ((in.kind & G::I_KIND_MASK) == G::I_TRANSLATE) return;
  r.d = nd;
  if (in.kind & G::IF_INV) {
    r.inv = inv_rn(nd);
    set_noinv(r); /* NaN mode in this frame (box_hit) */
  }
  if (in.kind & G::IF_DD) {
    r.dd = dot(nd, nd);
    r.rdd = div_rn_y(r.dd);
  }
}

/* ... and leaves it (K_INST_END): the enclosing frame's ray, re-derived from the walk's starting ray
 * (base_o, base_d) through the enclosing chain, and what inst_enter changed recomputed. */
HRT_LANE_FI void inst_leave(const KParams& P, const G::Inst& in, TRay& r, Vec3 base_o, Vec3 base_d) {
  Vec3 no = base_o, nd = base_d;
  apply_chain(P, in.parent, no, nd);
  r.o = no;
  if ((in.kind & G::I_KIND_MASK) == G::I_TRANSLATE) return;
  r.d = nd;
  if (in.kind & G::IF_INV) {
    r.inv = inv_rn(nd);
    set_noinv(r); /* NaN mode in this frame (box_hit) */
  }
  if (in.kind & G::IF_DD) {
    r.dd = dot(nd, nd);
    r.rdd = div_rn_y(r.dd);
  }
}

struct PathKey {
  uint64_t pkey;
  uint32_t segment;
};

/* HRT_MEDIUM_PAIR: layout.h */

/* A medium's boundary that is ONE sphere / moving sphere (Medium.sphere; its record p0, p1, p2 in registers):
 * both boundary queries of constant_medium.rs:37-48 from one evaluation of the quadratic (sphere_pair_at),
 * the sphere at the ray's time as moving_sphere.rs:55-58 computes it.  Returns the number of hits. */
HRT_LANE_FI int medium_pair(const KParams& P, const float4 p0, const float4 p1, float p2x, uint32_t km, const TRay& r,
                            float& c1, float& c2) {
  Vec3 c = v3(p0.x, p0.y, p0.z);
  if ((km & 3u) == G::P_MOVING) {
    const float tau = P.motion_uniform ? (r.time - P.motion_t0) / P.motion_span : r.time;
    const float f = P.motion_uniform ? tau : (tau - p1.w) / p2x;
    c = c + f * v3(p1.x, p1.y, p1.z);
  }
  return sphere_pair_at(c, p0.w, r.o, r.d, c1, c2);
}

/* constant_medium.rs:50-76 after the two boundary hits c1 < c2: the scatter distance against the part of
 * [c1, c2] in [tmin, closest]; a scatter becomes the closest hit, at the medium node `here` */
HRT_LANE_FI void medium_scatter(const KParams& P, const G::Medium& m, float c1, float c2, const TRay& r, float tmin,
                                float& closest, uint32_t& winner, uint32_t here, const PathKey& pk) {
  float r1 = c1, r2 = c2;
  if (r1 < tmin) r1 = tmin;
  if (r2 > closest) r2 = closest;
  if (r1 >= r2) return;
  if (r1 < 0.0f) r1 = 0.0f;
  const float ray_length = sqrtf(r.dd);
  const float inside = (r2 - r1) * ray_length;
  const float xi = medium_xi(pk.pkey, pk.segment, m.medium_id);
  const float hit_distance = m.neg_inv_density * (ln_f(xi) / P.ln_e);
  if (hit_distance > inside) return;
  closest = r1 + hit_distance / ray_length;
  winner = here;
}
/* The world walk.  Closest hit over [begin, end) of the node stream with t in [tmin, closest]:
 * `winner` = node index of the accepted leaf (NONE if nothing).  MEDIA: ConstantMedium nodes are
 * evaluated (their boundary walks are nested calls with MEDIA = false). */
template <int CULL, bool FULL, bool MEDIA, bool COUNT, bool FAST = false>
HRT_LANE void trace_ray(const KParams& P, const G::Node* __restrict__ nodes, const G::Prim* __restrict__ prims,
                        uint32_t begin, uint32_t end, TRay r, float tmin, float& closest, uint32_t& winner,
                        const PathKey& pk, Counts& cn);

template <int CULL, bool FULL, bool MEDIA, bool COUNT, bool FAST = false>
HRT_LANE void trace(const KParams& P, const G::Node* __restrict__ nodes, const G::Prim* __restrict__ prims,
                      uint32_t begin, uint32_t end, Vec3 o, Vec3 d, float time, float tmin, float& closest,
                      uint32_t& winner, const PathKey& pk, Counts& cn) {
  TRay r;
  set_ray(r, o, d, time, P);
  if constexpr (FAST) { /* the stream whose near-child order matches the ray's direction octant */
    const uint32_t oct = (d.x < 0.0f ? 1u : 0u) | (d.y < 0.0f ? 2u : 0u) | (d.z < 0.0f ? 4u : 0u);
    begin = oct * P.stream_len;
    end = begin + P.stream_len;
  }
  trace_ray<CULL, FULL, MEDIA, COUNT, FAST>(P, nodes, prims, begin, end, r, tmin, closest, winner, pk, cn);
}

/* The walk over [begin, end) of the node stream with a set-up ray r (its o, d are the frame the walk
 * starts in: instance ends re-derive their parent frame from them). */
template <int CULL, bool FULL, bool MEDIA, bool COUNT, bool FAST>
HRT_LANE void trace_ray(const KParams& P, const G::Node* __restrict__ nodes, const G::Prim* __restrict__ prims,
                        uint32_t begin, uint32_t end, TRay r, float tmin, float& closest, uint32_t& winner,
                        const PathKey& pk, Counts& cn) {
  const Vec3 base_o = r.o, base_d = r.d; /* the ray this walk started with */
  uint32_t i = begin;
  while (i < end) {
    const G::Node* np = nodes + i;
    const float4 a = ld4(np->mn);
    const float4 b = ld4(np->mx);
    const uint32_t kp = f2u(b.w);
    const uint32_t kind = (kp >> 24) & G::KIND_MASK;
    const bool ref_only = (kp & G::NODE_REF_ONLY) != 0;
    const uint32_t payload = kp & 0xFFFFFFu;
    const uint32_t here = i;
    if constexpr (COUNT) cn.nodes++;
    if constexpr (FAST) {
      bool pass = box_hit<CULL>(a, b, r, tmin, closest);
      if (kind == G::K_BOX) {
        i = pass ? i + 1 : f2u(a.w);
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
        i = pass ? i + 1 : umax(f2u(a.w), i + 1); /* skip links point forward: every walk ends */
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
          inst_enter(P.insts[payload], r);
        } else if (kind == G::K_INST_END) {
          inst_leave(P, P.insts[payload], r, base_o, base_d);
        } else if (kind == G::K_MEDIUM) {
          if constexpr (MEDIA) {
            /* constant_medium.rs:34-76 */
            const G::Medium m = P.media[payload];
            const float inf = u2f(0x7f800000u);
            float c1 = inf, c2 = inf;
            if (HRT_MEDIUM_PAIR && m.sphere != G::NONE) { /* one sphere: both queries from one quadratic */
              const G::Prim* bp = prims + m.sphere;
              const int hits = medium_pair(P, ld4(bp->p0), ld4(bp->p1), bp->p2[0], bp->km, r, c1, c2);
              if constexpr (COUNT) { /* the work counters of the two boundary walks it replaces */
                cn.nodes += hits > 0 ? 2u : 1u;
                cn.prims += hits > 0 ? 2u : 1u;
              }
              if (hits < 2) continue;
            } else {
              uint32_t w1 = G::NONE, w2 = G::NONE;
              trace<CULL, FULL, false, COUNT>(P, nodes, prims, m.bstart, m.bend, r.o, r.d, r.time, -inf, c1, w1, pk, cn);
              if (w1 == G::NONE) continue;
              trace<CULL, FULL, false, COUNT>(P, nodes, prims, m.bstart, m.bend, r.o, r.d, r.time, c1 + 0.0001f, c2, w2, pk, cn);
              if (w2 == G::NONE) continue;
            }
            medium_scatter(P, m, c1, c2, r, tmin, closest, winner, here, pk);
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

HRT_LANE_FI void set_face_normal(Rec& rec, Vec3 dir, Vec3 outward) {
  rec.front = dot(dir, outward) < 0.0f;
  rec.n = rec.front ? outward : -outward;
}

/* sphere.rs:31-35 */
/* out of line: two f64 transcendentals, needed only under an ImageTexture; (u, v) returned in registers */
struct UV {
  float u, v;
};
HRT_LANE_NI UV sphere_uv_v(Vec3 p) {
  float theta = acos_f(-p.y);
  float phi = atan2_f(-p.z, p.x) + PI_F;
  return UV{phi / (2.0f * PI_F), theta / PI_F};
}
HRT_LANE_FI void sphere_uv(Vec3 p, float& u, float& v) {
  const UV r = sphere_uv_v(p);
  u = r.u;
  v = r.v;
}

/* Record of the winning leaf in world space (hit_record.rs, sphere.rs:57-73, rect.rs:70-83,
 * constant_medium.rs:66-75, then translation.rs:33-35 / rotation.rs:119-132 on the way out). */
template <bool FULL>
HRT_LANE Rec make_record(const KParams& P, uint32_t winner, float t, Vec3 wo, Vec3 wd, float time, float tau) {
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
    Vec3 o = wo, d = wd;
    apply_chain(P, parent, o, d);
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
        float av = comp(o, a) + t * comp(d, a);
        float bv = comp(o, b) + t * comp(d, b);
        rec.p = o + t * d;
        rec.u = (av - p0.x) / pp->p1[1];
        rec.v = (bv - p0.z) / pp->p1[2];
        const Vec3 outward = v3(k == 0 ? 1.0f : 0.0f, k == 1 ? 1.0f : 0.0f, k == 2 ? 1.0f : 0.0f);
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
    /* back out through the chain, innermost first (translation.rs:32-40, rotation.rs:119-137) */
    if (parent != G::NONE) {
      const float4* ch = P.chains + (size_t)parent * G::CHAIN_F4;
      for (int l = (int)f2u(ch[0].x) - 1; l >= 0; l--) {
        const float4 v = ch[1 + l];
        if (f2u(v.w) == G::I_TRANSLATE) {
          rec.p = rec.p + v3(v.x, v.y, v.z);
          Vec3 po = wo, pd = wd; /* the ray as this level's parent saw it: the chain's first l levels */
          apply_chain_levels(P, parent, (uint32_t)l, po, pd);
          set_face_normal(rec, pd, rec.n);
        } else {
          const int axis = (int)f2u(v.z);
          int a = (axis + 1) % 3, b = (axis + 2) % 3;
          float s = v.x, c = v.y;
          const float pa = comp(rec.p, a), pb = comp(rec.p, b), na = comp(rec.n, a), nb = comp(rec.n, b);
          rec.p = with2(rec.p, a, c * pa - s * pb, b, s * pa + c * pb);
          rec.n = with2(rec.n, a, c * na - s * nb, b, s * na + c * nb);
        }
      }
    }
    return rec;
  }
}

/* perlin_noise.rs:80-123 over tables read through `pn`: a generic pointer, or (device, tables staged in LDS by
 * the kernel) an LDS address-space pointer, so the 8 x 4 gathers per call are ds_read, not flat loads */
#ifndef HRT_PERLIN_SELECT
#define HRT_PERLIN_SELECT 1 /* r06: C3 +1.3% (17 218 -> 17 445 Mrays/s, profiles/r06_perlin_select_ab.txt) */
#endif
#ifndef HRT_PERLIN_XADDR
#define HRT_PERLIN_XADDR 1 /* tables staged in LDS carry their gradients' addresses (kernel_common.h stage_perlin) */
#endif
/* XADDR: `pn` is an LDS pointer to tables staged by stage_perlin, whose permutation words XOR to the gradient's LDS
 * address; otherwise the layout.h tables as built (global memory, the host) */
/* HWCVT: the lattice's `floor() as i32` by the hardware conversion (hd_math.h sat_f2i32); otherwise the compare form
 * (sat_f2i32_cmp).  Only the sphere kernel's HEAVY shading takes it (C3 +4.6-6.4%): in the general kernel the
 * straight-line octave loop's longer live ranges cost Final 16 B more spills per lane and 3.5 GB of scratch writes per
 * frame for no time (profiles/r06i_final_summary.md against r06h's) */
template <bool XADDR = false, bool HWCVT = false, class PN>
HRT_LANE_FI float perlin_noise_t(PN pn, Vec3 point) {
  /* perlin_noise.rs:86-88 `floor() as i32` */
  const int32_t i = HWCVT ? sat_f2i32(floorf(point.x)) : sat_f2i32_cmp(floorf(point.x));
  const int32_t j = HWCVT ? sat_f2i32(floorf(point.y)) : sat_f2i32_cmp(floorf(point.y));
  const int32_t k = HWCVT ? sat_f2i32(floorf(point.z)) : sat_f2i32_cmp(floorf(point.z));
  float u = point.x - floorf(point.x);
  float v = point.y - floorf(point.y);
  float w = point.z - floorf(point.z);
  u = u * u * (3.0f - 2.0f * u);
  v = v * v * (3.0f - 2.0f * v);
  w = w * w * (3.0f - 2.0f * w);
#if HRT_PERLIN_SELECT
  /* default since r06 (0: the reference's multiply form): perlin_noise.rs:108-114's factor x u + (1 - x)(1 - u) for x in {0, 1} is
   * exactly (1 - u) or u -- u is in [0, 1] or NaN, so 0 u = +0, the sum adds +0 to a value >= 0 (or NaN to
   * NaN) and 1 v = v -- without the multiplies and adds strict IEEE code keeps (12 VALU per octave;
   * tests/test_lane_sim.py checks both forms against the oracle bit for bit) */
  const float u0 = 1.0f - u, v0 = 1.0f - v, w0 = 1.0f - w;
#endif
  float acc = 0.0f;
#pragma unroll
  for (int idx = 0; idx < 8; idx++) {
    const int x = idx / 4, y = (idx / 2) % 2, z = idx % 2;
    /* perlin_noise.rs:92-94 `(i + i_x) & 255` in i32, which wraps in a release build at i = i32::MAX (a
     * saturated huge coordinate): the same bits in u32, without C++'s signed-overflow UB (UBSan, r05) */
    /* XADDR (LDS): ((i + x) & 255) = (i & 255) + x in the doubled tables (layout.h Perlin), the corner pair one
     * ds_read2; the global-memory form keeps the masked index into the first copy (the pair as two global loads
     * cost Final's general kernel 16 B more spills per lane in the out-of-line noise call's saves) */
    const uint32_t ix = XADDR ? ((uint32_t)i & 255u) + (uint32_t)x : ((uint32_t)i + (uint32_t)x) & 255u;
    const uint32_t iy = XADDR ? ((uint32_t)j & 255u) + (uint32_t)y : ((uint32_t)j + (uint32_t)y) & 255u;
    const uint32_t iz = XADDR ? ((uint32_t)k & 255u) + (uint32_t)z : ((uint32_t)k + (uint32_t)z) & 255u;
    uint32_t px = pn->perm[0][ix];
    uint32_t py = pn->perm[1][iy];
    uint32_t pz = pn->perm[2][iz];
    Vec3 g;
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (XADDR) { /* perlin_noise.rs:96: ranvec[perm_x ^ perm_y ^ perm_z], the XOR already an address */
      typedef __attribute__((address_space(3))) const float4 lds_f4; /* a 16-B record: one ds_read */
      const float4 q = *(const lds_f4*)(size_t)(px ^ py ^ pz);
      g = v3(q.x, q.y, q.z);
    } else
#endif
    {
      const uint32_t g_i = px ^ py ^ pz;
      g = v3(pn->ranvec[g_i][0], pn->ranvec[g_i][1], pn->ranvec[g_i][2]);
    }
    Vec3 weight = v3(u - (float)x, v - (float)y, w - (float)z);
#if HRT_PERLIN_SELECT
    acc += ((x ? u : u0) * (y ? v : v0)) * (z ? w : w0) * dot(g, weight);
#else
    acc += ((float)x * u + (float)(1 - x) * (1.0f - u)) * ((float)y * v + (float)(1 - y) * (1.0f - v)) *
           ((float)z * w + (float)(1 - z) * (1.0f - w)) * dot(g, weight);
#endif
  }
  return acc;
}
HRT_LANE float perlin_noise(const G::Perlin* pn, Vec3 point) { return perlin_noise_t(pn, point); }

/* noise_texture.rs:24-31 + turbulence perlin_noise.rs:66-78 (the scalar part of the texture value) */
template <bool XADDR = false, bool HWCVT = false, class PN>
HRT_LANE_FI float noise_value_t(PN pn, float scale, Vec3 p) {
  Vec3 q = scale * p;
  float accumulator = 0.0f, weight = 1.0f;
#pragma unroll 1
  for (int o = 0; o < 7; o++) { /* rolled: keeps the code (and the callers' register demand) small */
    accumulator += weight * perlin_noise_t<XADDR, HWCVT>(pn, q);
    weight *= 0.5f;
    q = q * 2.0f;
  }
  return 1.0f + sin_f((scale * p.z) + (10.0f * fabsf(accumulator)));
}

/* The noise texture's value with its tables at `pn`.  PLDS (device): the tables are in LDS (`pn` a generic
 * pointer into the kernel's staged tables: its low 32 bits are the LDS address).  Out of line, with every
 * input passed by value (no caller struct through memory). */
template <bool PLDS, bool HWCVT = false>
HRT_LANE_NI float noise_value(const G::Perlin* pn, float scale, Vec3 p) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (PLDS) {
    typedef __attribute__((address_space(3))) const G::Perlin lds_perlin;
    return noise_value_t<HRT_PERLIN_XADDR != 0, HWCVT>((const lds_perlin*)(size_t)(uint32_t)(size_t)pn, scale, p);
  }
#endif
  return noise_value_t<false, HWCVT>(pn, scale, p);
}

/* image_texture.rs:36-62 */
HRT_LANE_FI Vec3 image_value(const uint8_t* images, uint32_t off, uint32_t w, uint32_t h, uint32_t comps, float u, float v) {
  if (w == 0) return v3(1.0f, 0.0f, 1.0f);
  float uu = u < 0.0f ? 0.0f : (u > 1.0f ? 1.0f : u);
  float vc = v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v);
  float vv = 1.0f - vc;
  uint32_t ii = sat_f2u32(uu * (float)w);
  uint32_t jj = sat_f2u32(vv * (float)h);
  if (ii >= w) ii = w - 1;
  if (jj >= h) jj = h - 1;
  const uint8_t* px = images + off + ((size_t)jj * w + ii) * comps;
  const float cs = 1.0f / 255.0f;
  return v3(cs * (float)px[0], cs * (float)px[1], cs * (float)px[2]);
}

/* sign of sin_f(v) for 1e-6 <= |v| <= 1e6: sin_f reduces v by pi/2 (hd_math reduce_pio2, same
 * operations here) and returns sin_poly(r) / cos_poly(r) / -sin_poly(r) / -cos_poly(r) by quadrant;
 * for |r| < 1 sin_poly keeps the sign of r and cos_poly is positive, so only the reduction is needed.
 * (|n| < 2^20: rint is exact and n & 3 is reduce_pio2's quadrant.) */
HRT_LANE_FI bool sin_negative(float vf) {
  const double x = (double)vf;
  const double n = __builtin_rint(x * detail::TWO_OVER_PI);
  const double r = ((x - n * detail::P1) - n * detail::P2) - n * detail::P3;
  const int q = (int)n & 3;
  return q == 3 || (q == 0 && r < 0.0) || (q == 2 && r > 0.0);
}

/* the full product, as the oracle computes it; a real call, so that its f64 temporaries do not
 * count towards the registers of the kernels it is reached from (it runs only for rare inputs) */
HRT_LANE_NI bool checker_product_negative(float vx, float vy, float vz) {
  return (sin_f(vx) * sin_f(vy)) * sin_f(vz) < 0.0f;
}

/* checker_texture.rs:22-29: sin(10x) * sin(10y) * sin(10z) < 0, decided from the signs.  With every
 * |v| in [1e-6, 1e6] each f32 sine is nonzero (an f32 there is > 1e-9 from any multiple of pi) and the
 * product of three cannot underflow, so the product is negative exactly when an odd number of
 * factors are; anything else (zero, tiny, huge, NaN) takes sin_f's full product. */
HRT_LANE_FI bool checker_odd(float vx, float vy, float vz) {
#if HRT_EXP_NOCHECKER /* timing experiment only (wrong colours): the price of the sine signs */
  return vx < 0.0f;
#endif
  const float ax = fabsf(vx), ay = fabsf(vy), az = fabsf(vz);
  const bool in_range = ax >= 1e-6f && ax <= 1e6f && ay >= 1e-6f && ay <= 1e6f && az >= 1e-6f && az <= 1e6f;
  if (in_range) return sin_negative(vx) != (sin_negative(vy) != sin_negative(vz));
  return checker_product_negative(vx, vy, vz);
}

/* textures/.rs value() */

/* INL: the noise texture's turbulence inline (a kernel with the registers to spare: a call saves and
 * restores the caller's live registers through scratch) instead of the out-of-line noise_value */
template <bool FULL, bool COUNT, bool INL = false, bool HWCVT = false>
HRT_LANE Vec3 tex_value(const KParams& P, uint32_t id, float u, float v, Vec3 p, Counts& cn) {
  for (int guard = 0; guard < 64; guard++) {
    const G::Tex& T = P.texs[id];
    if constexpr (COUNT) cn.tex++;
    if (T.kind == G::T_SOLID) return v3(T.a[0], T.a[1], T.a[2]);
    if (T.kind == G::T_CHECKER) { /* checker_texture.rs:22-29 */
      id = checker_odd(10.0f * p.x, 10.0f * p.y, 10.0f * p.z) ? T.i0 : T.i1;
      continue;
    }
    if constexpr (FULL) {
      if (T.kind == G::T_NOISE) { /* noise_texture.rs:24-31: 0.5 (1 + sin(...)) per channel */
        const G::Perlin* pn = P.perlin + T.i0;
        float s;
        if constexpr (INL) {
#if defined(__HIP_DEVICE_COMPILE__)
          typedef __attribute__((address_space(3))) const G::Perlin lds_perlin;
          if (P.perlin_lds) s = noise_value_t<HRT_PERLIN_XADDR != 0, HWCVT>((const lds_perlin*)(size_t)(uint32_t)(size_t)pn, T.a[0], p);
          else
#endif
            s = noise_value_t(pn, T.a[0], p);
        } else {
          s = P.perlin_lds ? noise_value<true, HWCVT>(pn, T.a[0], p) : noise_value<false>(pn, T.a[0], p);
        }
        return (v3(1.0f, 1.0f, 1.0f) * 0.5f) * s;
      }
      if (T.kind == G::T_IMAGE) return image_value(P.images, T.i0, T.i1, T.i2, T.i3, u, v);
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
/* host side: the reciprocals start_sample's camera divisions use (W, H >= 2) */
inline void set_pixel_rcp(KParams& P) {
  P.rw1 = 1.0f / ((float)P.W - 1.0f);
  P.rh1 = 1.0f / ((float)P.H - 1.0f);
}

HRT_LANE_FI void start_sample(const KParams& P, PathState& ps, uint32_t px, uint32_t py,
                                             uint32_t sample) {
#if HRT_EXP_CHEAPSEED /* timing experiment only (wrong streams): the price of the per-sample seeding */
  {
    const uint32_t k = (py * P.W + px) * 0x9E3779B9u ^ (P.sample_offset + sample) * 0x85EBCA6Bu;
    ps.pk.pkey = k;
    ps.rng.s0 = k | 1u; ps.rng.s1 = k ^ 0x6A09E667u; ps.rng.s2 = k ^ 0xBB67AE85u; ps.rng.s3 = k ^ 0x3C6EF372u;
  }
#else
  ps.pk.pkey = path_key(P.seed, py * P.W + px, P.sample_offset + sample);
  ps.rng = rng_from_key(ps.pk.pkey);
#endif
  ps.pk.segment = 0;
  /* application.rs:444-445 u, v: x / (W - 1) correctly rounded by div_rn's 3-instruction core with the
   * host's y = RN(1 / a), a = W - 1, and no IEEE fallback.  Why that is exact here (render parameters
   * hold 2 <= W, H <= 65535, so a is an integer in [1, 65534]; x = RN(px + gen_f32()) is 0 or an f32
   * multiple of 2^-24 in [2^-24, 2^16]):
   *  - x = 0 gives q0 = 0 and the core returns +0, as IEEE does;
   *  - q0 = RN(x y) is within 1.5 ulp of x / a, so the residual fma(-q0, a, x) is exact and
   *    q0 + r y = x / a + r (y - 1/a) with |r (y - 1/a)| <= a ulp 2^-24 / a = 2^-24 ulp of the quotient;
   *  - x / a = N 2^-24 / a with N integer, so its distance to any rounding midpoint (2j+1) 2^(e-24) is
   *    0 or >= 2^-24 2^min(e,0) / a >= 2^-17 ulp, far above the 2^-24 ulp perturbation;
   *  - it is never 0: x = a m would need the >= 25 odd significant bits of m (times a) in an f32.
   * So the final RN lands on RN(x / a).  tests/native/div_rn_check.c `camera` checks every a in
   * [1, 65534] at the edge values of x (tests/test_fast_division.py). */
  const float xu = (float)px + ps.rng.gen_f32(), aw = (float)P.W - 1.0f;
  const float xv = (float)py + ps.rng.gen_f32(), ah = (float)P.H - 1.0f;
  const float qu = xu * P.rw1, qv = xv * P.rh1;
  float u = fmaf(fmaf(-qu, aw, xu), P.rw1, qu);
  float v = fmaf(fmaf(-qv, ah, xv), P.rh1, qv);
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

/* The scatter of one ray_color step (application.rs:486-494) at the hit `rec` of a material of kind
 * `kind` (Metal: albedo, fuzz; Dielectric: ior); `tex()` is the material's texture at the hit (read
 * after the scatter's draws: textures draw no random numbers).  The scattered ray goes to
 * ps.ro/ps.rd.  Returns true when the path is finished. */
template <bool FULL, class TexFn>
HRT_LANE_FI bool scatter(PathState& ps, const Rec& rec, uint32_t kind, Vec3 albedo, float fuzz, float ior, Vec3 rd,
                         TexFn&& tex) {
  Vec3 emitted = v3(0.0f, 0.0f, 0.0f);
  Vec3 att = v3(0.0f, 0.0f, 0.0f), ndir = v3(0.0f, 0.0f, 0.0f);
  bool scattered = false;
  Rng& rng = ps.rng;
  bool textured = false; /* att (or, for a light, emitted) = the material's texture at the hit */
  /* Lambertian, Metal and Isotropic each start with random_in_unit_sphere (their first draws; Metal's
   * reflect draws nothing): ONE rejection loop shared by the three branches, so a wave holding several
   * of these materials runs the loop once, not once per branch. */
  Vec3 sph = v3(0.0f, 0.0f, 0.0f);
  if (kind == G::M_LAMBERTIAN || kind == G::M_METAL || (FULL && kind == G::M_ISOTROPIC))
    sph = random_in_unit_sphere(rng);
  if (kind == G::M_LAMBERTIAN) { /* lambertian.rs:27-38 */
    ndir = rec.n + normalize(sph); /* random_unit_vector, math.rs:12-14 */
    if (near_zero(ndir)) ndir = rec.n;
    textured = true;
    scattered = true;
  } else if (kind == G::M_METAL) { /* metal.rs:29-42 */
    Vec3 reflected = reflect(normalize(rd), rec.n);
    ndir = reflected + fuzz * sph;
    scattered = dot(ndir, rec.n) > 0.0f;
    att = albedo;
  } else if (kind == G::M_DIELECTRIC) { /* dielectric.rs:31-55 */
    float ratio = rec.front ? rcp_rn(ior) : ior;
    Vec3 ud = normalize(rd);
    float cos_theta = min_rs(dot(-ud, rec.n), 1.0f);
    float sin_theta = sqrtf(1.0f - cos_theta * cos_theta);
    bool cannot_refract = (ratio * sin_theta) > 1.0f;
    if (cannot_refract || reflectance(cos_theta, ratio) > rng.gen_f32()) ndir = reflect(ud, rec.n);
    else ndir = refract(ud, rec.n, ratio);
    att = v3(1.0f, 1.0f, 1.0f);
    scattered = true;
  } else if (FULL && kind == G::M_DIFFUSE_LIGHT) { /* diffuse_light.rs:20-28 */
    textured = true;
  } else if (FULL && kind == G::M_ISOTROPIC) { /* isotropic.rs:26-33 */
    ndir = sph;
    textured = true;
    scattered = true;
  }
  if (textured) {
    const Vec3 tv = tex();
    if (FULL && kind == G::M_DIFFUSE_LIGHT) emitted = tv;
    else att = tv;
  }
  /* L = emitted + att * L_next, accumulated front to back (only FULL scenes have emitters: without
   * them rad stays +0 until the path's miss, and adding thr x 0 would change no bit) */
  if constexpr (FULL) ps.rad = ps.rad + mul_elem(ps.thr, emitted);
  if (!scattered) return true;
  ps.thr = mul_elem(ps.thr, att);
  ps.ro = rec.p;
  ps.rd = ndir;
  ps.depth_left--;
  return false;
}

/* TRIM_PROGRAMS (general walk kernel): every leaf program is a one-node or one-sphere-medium one (layout.h
 * GL_ONE / GL_MED; scene w_generic false), so trace_ray's generic program is not compiled in */
enum : int { TRIM_MEDIA = 1, TRIM_HEAVY_TEX = 2, TRIM_PROGRAMS = 4 };

/* The part of one ray_color step after world.hit (application.rs:483-494): background on a miss,
 * else hit record, emission and scatter.  (ro, rd, rtime) is the segment just traced; the scattered
 * ray goes to ps.ro/ps.rd.  Returns true when the path is finished. */
#ifndef HRT_GEN_TEX_INLINE
#define HRT_GEN_TEX_INLINE 0 /* 1: the segment / general kernels evaluate the noise texture inline (A/B) */
#endif
template <bool FULL, bool COUNT, int TRIM = 0>
HRT_LANE_FI bool shade(const KParams& P, PathState& ps, uint32_t winner, float closest, Vec3 ro,
                                      Vec3 rd, float rtime, float tau, Counts& cn) {
  if (winner == G::NONE) {
    ps.rad = ps.rad + mul_elem(ps.thr, P.background);
    return true;
  }
  const Rec rec = make_record<FULL>(P, winner, closest, ro, rd, rtime, tau);
  const G::Mat M = P.mats[rec.mat];
  return scatter<FULL>(ps, rec, M.kind, v3(M.a[0], M.a[1], M.a[2]), M.a[3], M.a[0], rd,
                       [&]() { return tex_value<FULL && !(TRIM & TRIM_HEAVY_TEX), COUNT, HRT_GEN_TEX_INLINE != 0>(P, M.tex, rec.u, rec.v, rec.p, cn); });
}

/* shade() for the sphere kernel's walk stream: the winner is a leaf record (layout.h), which holds the
 * sphere and its material, so the hit record and the scatter read the walk stream only (LDS). */
#ifndef HRT_HEAVY_INLINE
#define HRT_HEAVY_INLINE 0 /* 1: the HEAVY instantiation evaluates textures inline (r03i A/B on C3: 16491 vs 17085 Mrays/s out of line) */
#endif
/* HEAVY: the scene also has noise / image textures (read from texs through the material, WT_GLOBAL):
 * Perlin turbulence and the sphere's (u, v) are out-of-line calls with by-value arguments (noise_value,
 * sphere_uv_v), made only by lanes whose material needs them; Perlin tables staged in LDS are read as LDS. */
template <bool COUNT, int WMEM, bool HEAVY = false>
HRT_LANE_FI bool shade_walk(const KParams& P, const WalkSrc& src, PathState& ps, uint32_t leaf, float closest,
                            Vec3 ro, Vec3 rd, float rtime, float tau, Vec3& sum, Counts& cn) {
  constexpr int MEM = payload_mem<WMEM>();
  if (leaf == G::NONE) { /* a sphere scene's path gathers radiance at its miss only: straight into the sum
                          * (sum + (+0 + thr bg) == sum + thr bg: the sum is never -0) */
    sum = sum + mul_elem(ps.thr, P.background);
    return true;
  }
  /* sphere.rs:57-73 / moving_sphere.rs:80-94 (leaf = the winning leaf's payload) */
  const float4 bmn = wload<MEM>(src, leaf), bmx = wload<MEM>(src, leaf + 16u);
  const float4 s0 = wload<MEM>(src, leaf + 32u);
  Vec3 c = v3(s0.x, s0.y, s0.z);
  if (f2u(bmn.w) & G::WL_MOVING) {
    const float4 s1 = wload<MEM>(src, leaf + 48u);
    const float f = P.motion_uniform ? tau : (rtime - s0.w) / s1.w;
    c = c + f * v3(s1.x, s1.y, s1.z);
  }
  Rec rec;
  rec.u = 0.0f;
  rec.v = 0.0f;
  const Vec3 at = ro + closest * rd;
  const Vec3 outward = (at - c) / bmx.w;
  rec.p = at;
  set_face_normal(rec, rd, outward);
  const float4 ma = wload<MEM>(src, leaf + 64u), mb = wload<MEM>(src, leaf + 80u);
  const uint32_t mw = f2u(mb.w);
  rec.mat = mw >> 8;
  const uint32_t wt = (mw >> 4) & 15u;
  return scatter<false>(ps, rec, mw & 15u, v3(ma.x, ma.y, ma.z), ma.w, ma.w, rd, [&]() {
    if (wt == G::WT_SOLID) {
      if constexpr (COUNT) cn.tex++;
      return v3(ma.x, ma.y, ma.z);
    }
    if (wt == G::WT_CHECKER) { /* checker_texture.rs:22-29 over two SolidColors */
      if constexpr (COUNT) cn.tex += 2;
      return checker_odd(10.0f * rec.p.x, 10.0f * rec.p.y, 10.0f * rec.p.z) ? v3(ma.x, ma.y, ma.z)
                                                                             : v3(mb.x, mb.y, mb.z);
    }
    if constexpr (HEAVY) { /* sphere.rs:31-35 (u, v) only under an image texture (Mat.needs_uv) */
      const G::Mat& M = P.mats[rec.mat];
      if (M.needs_uv) sphere_uv(outward, rec.u, rec.v);
      return tex_value<true, COUNT, HRT_HEAVY_INLINE != 0, true>(P, M.tex, rec.u, rec.v, rec.p, cn); /* HWCVT */
    }
    return tex_value<false, COUNT>(P, P.mats[rec.mat].tex, rec.u, rec.v, rec.p, cn);
  });
}

/* One step of ray_color (application.rs:477-495).  Returns true when the path is finished.
 * dbg (debug kernel only): receives o, d, time, t, winner of the traced segment.
 * TRIM (general scenes): features the scene does not have are compiled out, which changes nothing for
 * it: TRIM_MEDIA the medium branch of the walk (no ConstantMedium), TRIM_HEAVY_TEX the out-of-line
 * noise / image texture call (only solid and checker textures). */
template <int CULL, bool FULL, bool COUNT, bool FAST, int TRIM = 0>
HRT_LANE_FI bool segment(const KParams& P, const G::Node* nodes, const G::Prim* prims,
                                        PathState& ps, Counts& cn, float* dbg) {
  ps.traced = false;
  if (ps.depth_left == 0) return true; /* depth cap: black (:478-480) */
  float closest = u2f(0x7f800000u);
  uint32_t winner = G::NONE;
  trace<CULL, FULL, FULL && !(TRIM & TRIM_MEDIA), COUNT, FAST>(P, nodes, prims, 0u, P.main_end, ps.ro, ps.rd, ps.rtime, P.t_min, closest,
                                       winner, ps.pk, cn);
  ps.traced = true;
  ps.pk.segment++;
  if (dbg) {
    dbg[0] = ps.ro.x; dbg[1] = ps.ro.y; dbg[2] = ps.ro.z;
    dbg[3] = ps.rd.x; dbg[4] = ps.rd.y; dbg[5] = ps.rd.z;
    dbg[6] = ps.rtime; dbg[7] = closest; dbg[8] = u2f(winner);
  }
  const float tau = P.motion_uniform ? (ps.rtime - P.motion_t0) / P.motion_span : 0.0f;
  return shade<FULL, COUNT, TRIM>(P, ps, winner, closest, ps.ro, ps.rd, ps.rtime, tau, cn);
}

HRT_LANE_FI void init_path_state(PathState& ps) {
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

/* One node of the BASIC world walk (spheres and moving spheres under boxes; trace() restricted),
 * in two halves.  basic_box: both 16-B halves of the node are loaded and the box tested for every
 * node kind (a PRIM node's box result is ignored); the walk moves on (a passed node's successor is
 * node + 1, so the leaf is found again as i - 1), and a primitive that must be tested is left in
 * `pend` (its index).  basic_prim then tests it against the lane's current `closest`.  A lane runs
 * basic_prim before its next basic_box, so its sequence of tests is exactly basic_step's; the kernel
 * only chooses WHEN, batching the primitive tests of many lanes into one execution of the divergent
 * sphere block.  These walk the reference node stream under CULL_REFERENCE / CULL_SLAB (the
 * verbatim-reference and approximate modes); CULL_EXACT walks the walk stream (walk_box / walk_prim). */
/* The walk position of the BASIC kernel is ONE register: the next node's index, with WALK_PEND set
 * while the primitive of the leaf just passed (index - 1) waits for its test, or NONE when the lane
 * has no walk.  So "can step" is the single compare i < end, and the waiting primitive is read back
 * from the leaf's own record (basic_prim loads that record anyway for the reference test). */
constexpr uint32_t WALK_PEND = G::WALK_PEND;
HRT_LANE_FI bool walk_pending(uint32_t i) { return i - WALK_PEND < 0x7FFFFFFFu; } /* PEND set, i != NONE */

/* STRIDE: the walk position is a node index (1), or the node's LDS byte address (32, sizeof(Node)):
 * the LDS-resident stream is staged with its skip links turned into LDS addresses, so a step loads
 * its node straight from the position, with no address arithmetic. */
template <uint32_t STRIDE>
HRT_LANE_FI void load_node(const G::Node* nodes, uint32_t i, float4& a, float4& b) {
  static_assert(STRIDE == 1 || STRIDE == sizeof(G::Node), "node index or LDS byte address");
  if constexpr (STRIDE == 1) {
    a = ld4(nodes[i].mn);
    b = ld4(nodes[i].mx);
  } else {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef __attribute__((address_space(3))) const float4 lds_float4;
    const lds_float4* p = (const lds_float4*)(size_t)i;
    a = p[0];
    b = p[1];
#endif
  }
}

template <int CULL, bool COUNT, uint32_t STRIDE = 1>
HRT_LANE_FI void basic_box(const KParams& P, const G::Node* __restrict__ nodes, uint32_t& i, const TRay& r,
                           float closest, Counts& cn) {
  float4 a, b;
  load_node<STRIDE>(nodes, i, a, b);
  uint32_t skip = f2u(a.w);
#if defined(__HIP_DEVICE_COMPILE__)
  /* keep the skip link in the node's first 16-B load: left to itself the compiler narrows that load
   * to 12 B and fetches the link in a second, dependent LDS read on the fail path */
  asm("" : "+v"(skip));
#endif
  const uint32_t kp = f2u(b.w);
  if constexpr (COUNT) cn.nodes++;
  static_assert(CULL != G::CULL_EXACT, "CULL_EXACT walks the walk stream (walk_box)");
  const bool pass = box_hit<CULL>(a, b, r, P.t_min, closest) || ((kp >> 24) & G::KIND_MASK) == G::K_PRIM;
  const bool prim = (kp & (G::KIND_MASK << 24)) != 0u; /* K_BOX_PRIM or K_PRIM: a primitive to test */
  const uint32_t next = i + (prim ? STRIDE + WALK_PEND : STRIDE);
  i = pass ? next : skip;
}

/* i = the walk position with WALK_PEND set; clears it and tests the leaf (i - 1)'s primitive */
template <int CULL, bool COUNT, uint32_t STRIDE = 1>
HRT_LANE_FI void basic_prim(const KParams& P, const G::Node* __restrict__ nodes, const G::Prim* __restrict__ prims,
                            uint32_t& i, const TRay& r, float& closest, uint32_t& winner, Counts& cn) {
  i -= WALK_PEND;
  float4 a, b;
  load_node<STRIDE>(nodes, i - STRIDE, a, b);
  const uint32_t kp = f2u(b.w);
  const uint32_t payload = kp & 0xFFFFFFu;
  const G::Prim* pp = prims + payload;
  if constexpr (COUNT) cn.prims++;
  float t;
  if (sphere_root(pp, pp->km & 3u, r, P.t_min, closest, t, P.motion_uniform != 0)) {
    closest = t;
    winner = payload;
  }
}

/* both halves back to back (the host lane simulator's walk) */
template <int CULL, bool COUNT>
HRT_LANE_FI void basic_step(const KParams& P, const G::Node* __restrict__ nodes,
                                           const G::Prim* __restrict__ prims, uint32_t& i, const TRay& r,
                                           float& closest, uint32_t& winner, Counts& cn) {
  basic_box<CULL, COUNT>(P, nodes, i, r, closest, cn);
  if (walk_pending(i)) basic_prim<CULL, COUNT>(P, nodes, prims, i, r, closest, winner, cn);
}

/* The inflated test of CULL_EXACT on a box given by centre C and half-extent E (the walk stream's inner
 * boxes, which hold the reference boxes): false only if the box, widened by EXACT_MARGIN x D' (D' =
 * max_k |C_k - o_k| + E_k >= the L-inf distance of its farthest point from the origin), misses the ray
 * on [tmin, tmax].  Per axis the slab is m_k -+ t_k |inv_k| with m_k = (C_k - o_k) inv_k and
 * t_k = E_k + EXACT_MARGIN D', so the near/far swap of aabb.rs:28-29 disappears; each bound is one fma
 * (t_k by fmamk, the bounds by fma with |inv_k| as a source modifier).
 * HRT_BOX_FMA (default): m_k = fma(C_k, inv_k, -(o_k inv_k)) with the product kept per ray (TRay.noinv)
 * and |C_k - o_k| = |m_k| |d_k| folded into e_k = fma(|m_k|, |d_k|, E_k): two instructions per axis
 * instead of three (sub, mul, add).  Its extra error is the rounding of o_k inv_k, 2^-24 |o_k| in
 * position units; the stream's boxes keep max_k E_k >= 2^-12 max_k |C_k| (layout.h CE_FLOOR), so
 * |o_k| <= |C_k| + D' <= 4097 D' and that error stays below 2.5e-4 D'.  Rounding errors of the whole
 * computation stay below ~2.6e-4 D' |inv_k|, inside the slack of EXACT_MARGIN (layout.h: 4e-3 covers the
 * 2.4e-3 needed with 1.6e-3 to spare).  A NaN bound (the old form: inv_k = +-inf with C_k = o_k or
 * E_k = 0) is ignored by max3/min3: no constraint; a ray whose noinv is NaN (set_dir) passes every box.
 * An infinite box (E = +inf) always passes.  The hybrid LDS / global walk (WM_HYB, latency-bound) and the
 * sphere kernel's HEAVY instantiation keep the sub/mul/add form: the three more live registers cost them
 * 4.5% (C4 1/8 share) and 3% (C3), while the LDS walks gain 1.5-2% (C2: 14473 -> 14785 Mrays/s on the
 * r03v bench) from the two fewer instructions per axis.  tests/test_lane_sim.py checks both forms on
 * grazing, tiny-far and axis-aligned rays. */
#ifndef HRT_BOX_FMA
#define HRT_BOX_FMA 1
#endif
#ifndef HRT_BOX_FMA_ALL
#define HRT_BOX_FMA_ALL 0 /* 1: the hybrid walk and HEAVY use the fused form too */
#endif
/* NANG: the sub/mul/add form honours the ray's NaN mode (set_noinv; the fused form does by construction).
 * Only scenes with rects can produce the NaN hits that make it necessary; sphere kernels pass false. */
template <bool FMA = HRT_BOX_FMA, bool NANG = true>
HRT_LANE_FI bool box_ce(const float4& a, const float4& b, const TRay& r, float tmin, float tmax) {
  const float C[3] = {a.x, a.y, a.z}, E[3] = {b.x, b.y, b.z};
  const float inv[3] = {r.inv.x, r.inv.y, r.inv.z};
  float m[3], e[3];
  if constexpr (FMA) {
    const float noinv[3] = {r.noinv.x, r.noinv.y, r.noinv.z}, d[3] = {r.d.x, r.d.y, r.d.z};
#pragma unroll
    for (int k = 0; k < 3; k++) {
      float mk = fmaf(C[k], inv[k], noinv[k]);
#if defined(__HIP_DEVICE_COMPILE__)
      asm("" : "+v"(mk)); /* keep the axes scalar (no v_pk_*: see below) */
#endif
      m[k] = mk;
      e[k] = fmaf(fabsf(mk), fabsf(d[k]), E[k]);
    }
  } else {
    const float o[3] = {r.o.x, r.o.y, r.o.z};
#pragma unroll
    for (int k = 0; k < 3; k++) {
      float dc = C[k] - o[k];
#if defined(__HIP_DEVICE_COMPILE__)
      /* keep the three axes scalar: the SLP vectorizer would pair x and y into v_pk_* operations, which
       * issue no faster than two scalar ones on gfx950 and cost moves (measured 4% slower) */
      asm("" : "+v"(dc));
#endif
      m[k] = dc * inv[k];
      e[k] = fabsf(dc) + E[k];
    }
  }
  /* the farthest point's distance per axis: monotone under box inclusion, so a child's inflated box
   * lies in its parent's and every hierarchy over the same leaves tests the same leaves (max |dc| +
   * max E would save an instruction but is not monotone) */
  const float dist = fmaxf(fmaxf(e[0], e[1]), e[2]);
  float l[3], h[3];
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const float t = fmaf(dist, G::EXACT_MARGIN, E[k]);
    l[k] = fmaf(-t, fabsf(inv[k]), m[k]);
    h[k] = fmaf(t, fabsf(inv[k]), m[k]);
  }
  /* max(lo, tmin) <= min(hi, tmax) is !(hi < lo) & !(hi < tmin) & !(tmax < lo) when tmin <= tmax (a walk's
   * closest never drops below t_min; a NaN closest, G20, leaves min(hi, NaN) = hi: no bound from it, as the
   * three-comparison form) -- one comparison and no mask arithmetic.  A NaN lo / hi (all three axes NaN) is
   * no constraint either way. */
  const float lo = fmaxf(fmaxf(fmaxf(l[0], l[1]), l[2]), tmin);
  const float hi = fminf(fminf(fminf(h[0], h[1]), h[2]), tmax);
  if constexpr (!FMA && NANG) return !(hi < lo) | nan_mode(r);
  return !(hi < lo);
}

/* One node step: an inner node moves to pass / skip; a passed leaf parks the lane on it (WALK_PEND).  ls (the
 * walk kernels, HRT_KEEP_SKIP): the step's skip link, kept in a register of the lane's own.  A leaf's skip IS its
 * pre-order successor (layout.h), so a lane parked on a leaf continues there without reading the payload: in a
 * hybrid stream every payload is a global read, one dependent L2 round trip per leaf in the walk loop. */
/* FMA: box_ce's fused form (default except for the latency-bound hybrid walk; the sphere kernel's
 * HEAVY instantiation passes false: at its 128-VGPR cap the three more live registers cost 3% on C3) */
template <bool COUNT, int MEM, bool FMA = HRT_BOX_FMA && (MEM != WM_HYB || HRT_BOX_FMA_ALL), bool NANG = true,
          uint32_t HALF = 16, bool C16 = false>
HRT_LANE_FI void walk_box(const WalkSrc& src, uint32_t& i, const TRay& r, float tmin, float closest, Counts& cn,
                          uint32_t* ls = nullptr) {
  if constexpr (C16) { /* layout.h WALK_C16: position = node index, part at 16 i */
    const float4 q = wload_part16<MEM>(src, i << 4);
    const uint32_t w0 = f2u(q.x), w1 = f2u(q.y), w2 = f2u(q.z);
    uint32_t links = f2u(q.w);
#if defined(__HIP_DEVICE_COMPILE__)
    asm("" : "+v"(links));
#endif
    const float4 a = make_float4(h2f(w0 & 0xFFFFu), h2f(w0 >> 16), h2f(w1 & 0xFFFFu), 0.0f);
    const float4 b = make_float4(h2f(w1 >> 16), h2f(w2 & 0xFFFFu), h2f(w2 >> 16), 0.0f);
    if constexpr (COUNT) cn.nodes++;
    if (ls) *ls = links & 0xFFFFu;
    i = box_ce<FMA, NANG>(a, b, r, tmin, closest) ? links >> 16 : links & 0xFFFFu;
    return;
  }
  float4 a, b;
  wload_node<MEM, HALF>(src, i, a, b);
  uint32_t skip = f2u(a.w);
#if defined(__HIP_DEVICE_COMPILE__)
  asm("" : "+v"(skip)); /* keep the link in the first 16-B load (see basic_box) */
#if HRT_EXP_LDS2 /* timing experiment: one more 16-B LDS read per step (is the walk LDS-bound?) */
  { const float4 x = wload<MEM>(src, i + 32u); asm volatile("" :: "v"(x.x), "v"(x.y), "v"(x.z), "v"(x.w)); }
#endif
#endif
  if constexpr (COUNT) cn.nodes++;
  if (ls) *ls = skip;
  i = box_ce<FMA, NANG>(a, b, r, tmin, closest) ? f2u(b.w) : skip;
}

#ifndef HRT_LEAF_HOIST
#define HRT_LEAF_HOIST 0
#endif
/* The parked leaf's primitive: the reference test on its box (aabb.rs, monotone: leaves suffice, DESIGN
 * section 4), then the sphere test against the lane's closest; the walk continues behind the leaf. */
template <bool COUNT, int WMEM>
HRT_LANE_FI void walk_leaf_test(const KParams& P, const WalkSrc& src, uint32_t leaf, const TRay& r, float& closest,
                                uint32_t& winner, Counts& cn) {
  constexpr int MEM = payload_mem<WMEM>();
  const float4 bmn = wload<MEM>(src, leaf), bmx = wload<MEM>(src, leaf + 16u);
  /* a global payload (hybrid and buffer streams): the sphere's parts read with the box, one round trip instead
   * of up to three dependent ones (box -> centre -> motion; HRT_LEAF_HOIST: 1 the centre, 2 the motion too, which
   * 80% of the random scenes' spheres have).  Measured no faster on C4's 1/8 share (the other waves hide the
   * dependent reads; profiles/r06_leaf_hoist_ab.txt), so off by default. */
  constexpr bool HOIST = HRT_LEAF_HOIST && MEM == WM_BUF;
  float4 s0 = make_float4(0.0f, 0.0f, 0.0f, 0.0f), s1 = s0;
  if constexpr (HOIST) s0 = wload<MEM>(src, leaf + 32u);
  if constexpr (HOIST && HRT_LEAF_HOIST > 1) s1 = wload<MEM>(src, leaf + 48u);
  const uint32_t w = f2u(bmn.w);
  if (!(w & G::WL_NOBOX) && !box_ref(bmn, bmx, r, P.t_min, closest)) return;
  if constexpr (COUNT) cn.prims++;
  if constexpr (!HOIST) s0 = wload<MEM>(src, leaf + 32u);
  Vec3 c = v3(s0.x, s0.y, s0.z);
  if (w & G::WL_MOVING) { /* moving_sphere.rs:55-58 */
    if constexpr (!(HOIST && HRT_LEAF_HOIST > 1)) s1 = wload<MEM>(src, leaf + 48u);
    const float f = P.motion_uniform ? r.tau : (r.tau - s0.w) / s1.w; /* r.tau: the time (TRay) */
    c = c + f * v3(s1.x, s1.y, s1.z);
  }
  float t;
  if (sphere_root_at(c, bmx.w, r, P.t_min, closest, t)) {
    closest = t;
    winner = leaf; /* shade_walk reads the sphere and its material from the leaf */
  }
}

/* the leaf's pre-order successor, kept in its payload (w >> 2) */
template <int MEM>
HRT_LANE_FI uint32_t walk_successor(const WalkSrc& src, uint32_t leaf) { return f2u(wload<payload_mem<MEM>()>(src, leaf).w) >> 2; }

template <bool COUNT, int MEM, bool C16 = false>
HRT_LANE_FI void walk_prim(const KParams& P, const WalkSrc& src, uint32_t& i, const TRay& r, float& closest,
                           uint32_t& winner, Counts& cn) {
  const uint32_t leaf = pend_payload<C16>(P, i); /* the leaf's payload */
  i = walk_successor<MEM>(src, leaf); /* the walk goes on at the leaf's pre-order successor */
  walk_leaf_test<COUNT, MEM>(P, src, leaf, r, closest, winner, cn);
}

/* A one-node program (layout.h GL_ONE): trace_ray's body for a K_BOX_PRIM or K_PRIM node -- the node's
 * CULL_EXACT box test, then its rect or sphere against closest -- without the node loop and the dispatch over
 * every kind, whose code the wave otherwise runs for any lane that needs it.  Everything is addressed from
 * the payload (h.x the node, h.y its kind word, bmn.w the instance), so the node, its primitive and the
 * instance chain are loaded together, before the group box test: ONE memory round trip after the payload's
 * instead of up to three dependent ones (payload -> node -> primitive; payload -> chain -> its levels). */
#ifndef HRT_GWALK_ONE
#define HRT_GWALK_ONE 1
#endif
HRT_LANE_FI void chain_turn(const float4 c0, const float4 c1, const float4 c2, const float4* ch, Vec3& o, Vec3& d) {
  const uint32_t levels = f2u(c0.x); /* apply_chain_levels with the first two levels in registers */
  if (levels > 0u) chain_level(c1, o, d);
  if (levels > 1u) chain_level(c2, o, d);
  for (uint32_t l = 2; l < levels; l++) chain_level(ch[1 + l], o, d);
}

HRT_LANE_FI void chain_derived(uint32_t flags, TRay& lr) {
  /* 1/d and d.d of the turned direction where the program reads them (layout.h GL_INV / GL_DD) */
  if (flags & G::GL_INV) {
    lr.inv = inv_rn(lr.d);
    set_noinv(lr); /* NaN mode in the innermost frame (box_hit in the program) */
  }
  if (flags & G::GL_DD) {
    lr.dd = dot(lr.d, lr.d);
    lr.rdd = div_rn_y(lr.dd);
  }
}

template <bool COUNT>
HRT_LANE_FI void gwalk_one(const KParams& P, const G::Node* __restrict__ nodes, const G::Prim* __restrict__ prims,
                           uint32_t flags, const float4 h, const float4 bmn, const float4 bmx, const TRay& r,
                           float& closest, uint32_t& winner, uint32_t& gstate, Counts& cn) {
  const uint32_t i = f2u(h.x), kp = f2u(h.y);
  const G::Node* np = nodes + i;
  const float4 a = ld4(np->mn), b = ld4(np->mx);
  const G::Prim* pp = prims + (kp & 0xFFFFFFu);
  const float4 p0 = ld4(pp->p0), p1 = ld4(pp->p1), p2 = ld4(pp->p2);
  const bool inst = (flags & G::GL_INST) != 0u;
  const float4* ch = P.chains + (size_t)(inst ? f2u(bmn.w) : 0u) * G::CHAIN_F4;
  float4 c0 = p0, c1 = p0, c2 = p0;
  if (inst) {
    c0 = ch[0];
    c1 = ch[1];
    c2 = ch[2];
  }
  if (flags & G::GL_BOX) { /* the group's box: tested at the group's first leaf, the outcome kept (layout.h) */
    const uint32_t g = f2u(bmx.w);
    if ((gstate & 0x7FFFFFFFu) != g) gstate = g | (box_ref(bmn, bmx, r, P.t_min, closest) ? 0x80000000u : 0u);
    if (!(gstate >> 31)) return;
  }
  TRay lr = r;
  if (inst) {
    chain_turn(c0, c1, c2, ch, lr.o, lr.d);
    chain_derived(flags, lr);
#if HRT_EXP_CHAIN2 && defined(__HIP_DEVICE_COMPILE__) /* timing-only: the turn done twice (its cost, same images) */
    TRay l2 = r;
    float z = 0.0f;
    asm volatile("" : "+v"(z));
    l2.o.x += z;
    l2.d.x += z;
    chain_turn(c0, c1, c2, ch, l2.o, l2.d);
    chain_derived(flags, l2);
    asm volatile("" :: "v"(l2.o.x), "v"(l2.o.y), "v"(l2.o.z), "v"(l2.d.x), "v"(l2.d.y), "v"(l2.d.z), "v"(l2.inv.x),
                 "v"(l2.inv.y), "v"(l2.inv.z), "v"(l2.noinv.x), "v"(l2.noinv.y), "v"(l2.noinv.z), "v"(l2.dd), "v"(l2.rdd));
#endif
  }
  if constexpr (COUNT) cn.nodes++;
  if (((kp >> 24) & G::KIND_MASK) == G::K_BOX_PRIM &&
      !box_hit<G::CULL_EXACT>(a, b, lr, P.t_min, closest, (kp & G::NODE_REF_ONLY) != 0))
    return;
  const uint32_t km = f2u(p2.w);
  if constexpr (COUNT) cn.prims++;
  float t;
  bool hit;
  if ((km & 3u) == G::P_RECT) hit = rect_tv(p0, p1.x, (km >> 2) & 3u, lr, P.t_min, closest, t);
  else hit = sphere_root_v(p0, p1, p2.x, km & 3u, lr, P.t_min, closest, t, P.motion_uniform != 0);
  if (hit) {
    closest = t;
    winner = i;
  }
}

/* A passed leaf of the GENERAL walk stream (layout.h): the reference test of the enclosing BvhNode box
 * (box-less leaves, GL_BOX), then the leaf's program -- its range of the reference stream, whose first
 * node is the leaf's own box (the reference test at the leaf) -- from the world ray
 * against the lane's current closest.  The winner is a reference-stream node index (make_record<true>). */
/* A medium leaf over one sphere (layout.h GL_MED): trace_ray over its program [the ConstantMedium's box node,
 * its K_MEDIUM node] without the node loop, the box node, the medium record and the boundary sphere loaded
 * together (h.x the box node, h.y the medium, bmn.w the sphere) */
template <bool COUNT>
HRT_LANE_FI void gwalk_medium(const KParams& P, const G::Node* __restrict__ nodes, const G::Prim* __restrict__ prims,
                              uint32_t flags, const float4 h, const float4 bmn, const float4 bmx, const TRay& r,
                              float& closest, uint32_t& winner, uint32_t& gstate, const PathKey& pk, Counts& cn) {
  const uint32_t i = f2u(h.x);
  const G::Node* np = nodes + i;
  const float4 a = ld4(np->mn), b = ld4(np->mx);
  const G::Medium m = P.media[f2u(h.y)];
  const G::Prim* bp = prims + f2u(bmn.w);
  const float4 p0 = ld4(bp->p0), p1 = ld4(bp->p1), p2 = ld4(bp->p2);
  if (flags & G::GL_BOX) { /* as gwalk_one */
    const uint32_t g = f2u(bmx.w);
    if ((gstate & 0x7FFFFFFFu) != g) gstate = g | (box_ref(bmn, bmx, r, P.t_min, closest) ? 0x80000000u : 0u);
    if (!(gstate >> 31)) return;
  }
  if constexpr (COUNT) cn.nodes++;
  if (!box_hit<G::CULL_EXACT>(a, b, r, P.t_min, closest, (f2u(b.w) & G::NODE_REF_ONLY) != 0)) return;
  if constexpr (COUNT) cn.nodes++; /* the K_MEDIUM node */
  float c1 = u2f(0x7f800000u), c2 = c1;
  const int hits = medium_pair(P, p0, p1, p2.x, f2u(p2.w), r, c1, c2);
  if constexpr (COUNT) { /* the work counters of the two boundary walks it replaces (trace_ray) */
    cn.nodes += hits > 0 ? 2u : 1u;
    cn.prims += hits > 0 ? 2u : 1u;
  }
  if (hits < 2) return;
  medium_scatter(P, m, c1, c2, r, P.t_min, closest, winner, i + 1u, pk);
}

template <bool MEDIA, bool COUNT, int WMEM, bool PROG = true>
HRT_LANE_FI void gwalk_leaf_test(const KParams& P, const G::Node* __restrict__ nodes, const G::Prim* __restrict__ prims,
                                 const WalkSrc& src, uint32_t leaf, const TRay& r, float& closest, uint32_t& winner,
                                 uint32_t& gstate, const PathKey& pk, Counts& cn) {
  constexpr int MEM = payload_mem<WMEM>();
  const float4 h = wload<MEM>(src, leaf), bmn = wload<MEM>(src, leaf + 16u), bmx = wload<MEM>(src, leaf + 32u);
  const uint32_t flags = f2u(h.z);
  if (HRT_GWALK_ONE && (flags & G::GL_ONE)) {
    gwalk_one<COUNT>(P, nodes, prims, flags, h, bmn, bmx, r, closest, winner, gstate, cn);
    return;
  }
  if constexpr (MEDIA) {
    if (HRT_GWALK_ONE && (flags & G::GL_MED)) {
      gwalk_medium<COUNT>(P, nodes, prims, flags, h, bmn, bmx, r, closest, winner, gstate, pk, cn);
      return;
    }
  }
  if constexpr (!PROG && HRT_GWALK_ONE) return; /* (no such leaf: TRIM_PROGRAMS; GL_ONE leaves need the
                                                  * generic program when built without gwalk_one) */
  /* one call site for the program (the ray: the world ray, or the innermost instance frame's) */
  TRay lr = r;
  if (flags & G::GL_BOX) { /* as gwalk_one */
    const uint32_t g = f2u(bmx.w);
    if ((gstate & 0x7FFFFFFFu) != g) gstate = g | (box_ref(bmn, bmx, r, P.t_min, closest) ? 0x80000000u : 0u);
    if (!(gstate >> 31)) return;
  }
  if (flags & G::GL_INST) { /* (never with GL_MED: bmn.w is then the boundary sphere) */
    /* a leaf of a flattened instance chain (layout.h GL_INST): the ray in the innermost instance's frame,
     * as the reference's Translation / Rotation hits hand it down (apply_chain) */
    apply_chain(P, f2u(bmn.w), lr.o, lr.d);
    chain_derived(flags, lr);
  }
  const uint32_t begin = f2u(h.x); /* GL_ONE: h.y = the node's kind word; GL_MED: the medium (layout.h) */
  const uint32_t end = (flags & G::GL_ONE) ? begin + 1u : (flags & G::GL_MED) ? begin + 2u : f2u(h.y);
  trace_ray<G::CULL_EXACT, true, MEDIA, COUNT>(P, nodes, prims, begin, end, lr, P.t_min, closest, winner, pk, cn);
}

template <bool MEDIA, bool COUNT, int MEM>
HRT_LANE_FI void gwalk_prim(const KParams& P, const G::Node* __restrict__ nodes, const G::Prim* __restrict__ prims,
                            const WalkSrc& src, uint32_t& i, const TRay& r, float& closest, uint32_t& winner,
                            uint32_t& gstate, const PathKey& pk, Counts& cn) {
  const uint32_t leaf = i - WALK_PEND;
  i = walk_successor<MEM>(src, leaf);
  gwalk_leaf_test<MEDIA, COUNT, MEM>(P, nodes, prims, src, leaf, r, closest, winner, gstate, pk, cn);
}

/* both halves back to back (the host lane simulator's walk) */
template <bool COUNT, bool C16 = false>
HRT_LANE_FI void walk_step_host(const KParams& P, const WalkSrc& src, uint32_t& i, const TRay& r, float& closest,
                                uint32_t& winner, Counts& cn) {
  walk_box<COUNT, WM_HOST, HRT_BOX_FMA != 0, true, 16u, C16>(src, i, r, P.t_min, closest, cn);
  if (walk_pend<C16>(i)) walk_prim<COUNT, WM_HOST, C16>(P, src, i, r, closest, winner, cn);
}

/* The BASIC kernel (sphere scenes: the Random family), with POSTPONED shading.  A lane's walk state
 * (node, closest, winner, ray) lives across passes: the wave steps the walks of all its lanes one
 * node at a time and leaves the node loop only when at least P.postpone lanes have finished theirs
 * (or none is still walking); those lanes shade, start their next segment or sample, and the wave
 * goes back to stepping.  Every lane still runs exactly the reference's sequence of world.hit calls
 * and draws, so the image is the same as render_kernel's; only the wave's SIMD occupancy changes
 * (a wave no longer idles on its slowest lane's walk before every shading step). */
/* ------------------------------------------------------------------ general scenes, persistent walks */
/* Walk state of one lane in render_full_kernel: the main walk over [0, main_end), or one of the two
 * boundary walks of a ConstantMedium (constant_medium.rs:34-48: t in [-inf, inf], then [t1 + 1e-4, inf])
 * over its boundary subtree, after which the main walk resumes behind the medium node. */
struct FullWalk {
  uint32_t i, end;      /* active walk: next node, bound */
  uint32_t mode;        /* 0 main walk, 1 / 2 first / second boundary walk */
  uint32_t resume;      /* main-walk node after the medium node (mode != 0) */
  float tmin, cl;       /* active walk's t_min and closest */
  uint32_t wn;          /* active walk's winner: node index, NONE */
  float m_cl, c1;       /* main walk's closest while a boundary walk runs; the first boundary hit */
  uint32_t m_wn;
};

/* constant_medium.rs:50-76 after both boundary hits t1, t2: whether the ray scatters inside, and
 * where (`closest` in, the new closest out).  Out of line (f64 logarithm). */
HRT_LANE_NI bool medium_hit(const KParams& P, const G::Medium& m, float t1, float t2,
                                                     float closest, float dd, const PathKey& pk, float& t_out) {
  float r1 = t1, r2 = t2;
  if (r1 < P.t_min) r1 = P.t_min;
  if (r2 > closest) r2 = closest;
  if (r1 >= r2) return false;
  if (r1 < 0.0f) r1 = 0.0f;
  const float ray_length = sqrtf(dd);
  const float inside = (r2 - r1) * ray_length;
  const float xi = medium_xi(pk.pkey, pk.segment, m.medium_id);
  const float hit_distance = m.neg_inv_density * (ln_f(xi) / P.ln_e);
  if (hit_distance > inside) return false;
  t_out = r1 + hit_distance / ray_length;
  return true;
}

HRT_LANE_FI bool prim_hit(const KParams& P, const G::Prim* pp, const TRay& r, float tmin, float tmax,
                                         float& t) {
  const uint32_t km = pp->km;
  const uint32_t pkind = km & 3u;
  if (pkind == G::P_RECT) return rect_t(pp, (km >> 2) & 3u, r, tmin, tmax, t);
  return sphere_root(pp, pkind, r, tmin, tmax, t, P.motion_uniform != 0);
}

/* One node of a general walk (trace() as a resumable state machine).  `wo, wd` is the world ray:
 * INST_END rebuilds the parent frame's ray from it (apply_chain), so no per-lane ray stack is kept.
 * Media are only at world level here (plan() sends scenes with media inside instances to
 * render_kernel), so a boundary walk also starts from the world ray. */
template <int CULL, bool COUNT>
HRT_LANE_FI void full_step(const KParams& P, const G::Node* __restrict__ nodes,
                                          const G::Prim* __restrict__ prims, FullWalk& w, TRay& r, Vec3 wo, Vec3 wd,
                                          const PathKey& pk, Counts& cn) {
  const uint32_t here = w.i;
  const G::Node* np = nodes + here;
  const float4 a = ld4(np->mn);
  const float4 b = ld4(np->mx);
  const uint32_t kp = f2u(b.w);
  const uint32_t kind = (kp >> 24) & G::KIND_MASK;
  const uint32_t payload = kp & 0xFFFFFFu;
  if constexpr (COUNT) cn.nodes++;
  w.i = here + 1;
  if (kind <= G::K_PRIM) { /* K_BOX, K_BOX_PRIM, K_PRIM */
    const bool pass = kind == G::K_PRIM || box_hit<CULL>(a, b, r, w.tmin, w.cl, (kp & G::NODE_REF_ONLY) != 0);
    if (kind == G::K_BOX && !pass) w.i = umax(f2u(a.w), here + 1); /* skip links point forward */
    if (pass && kind != G::K_BOX) {
      if constexpr (COUNT) cn.prims++;
      float t;
      if (prim_hit(P, prims + payload, r, w.tmin, w.cl, t)) {
        w.cl = t;
        w.wn = here;
      }
    }
  } else if (kind == G::K_INST_BEGIN) {
    inst_enter(P.insts[payload], r);
  } else if (kind == G::K_INST_END) {
    inst_leave(P, P.insts[payload], r, wo, wd);
  } else if (kind == G::K_MEDIUM) { /* first boundary walk (constant_medium.rs:37) */
    const G::Medium& m = P.media[payload];
    w.resume = here + 1;
    w.m_cl = w.cl;
    w.m_wn = w.wn;
    w.mode = 1;
    w.i = m.bstart;
    w.end = m.bend;
    w.tmin = -u2f(0x7f800000u);
    w.cl = u2f(0x7f800000u);
    w.wn = G::NONE;
  }
  if (w.mode != 0 && w.i >= w.end) { /* a boundary walk ended */
    const uint32_t med_node = w.resume - 1;
    const G::Medium& m = P.media[nodes[med_node].kp & 0xFFFFFFu];
    bool back = w.wn == G::NONE; /* no boundary hit: the medium is missed */
    if (!back && w.mode == 1) {   /* second boundary walk (:42) */
      w.c1 = w.cl;
      w.mode = 2;
      w.i = m.bstart;
      w.tmin = w.c1 + 0.0001f;
      w.cl = u2f(0x7f800000u);
      w.wn = G::NONE;
    } else if (!back) {
      if (medium_hit(P, m, w.c1, w.cl, w.m_cl, r.dd, pk, w.m_cl)) w.m_wn = med_node;
      back = true;
    }
    if (back) {
      w.mode = 0;
      w.i = w.resume;
      w.end = P.main_end;
      w.tmin = P.t_min;
      w.cl = w.m_cl;
      w.wn = w.m_wn;
    }
  }
}


}  // namespace lane
}  // namespace hrt
