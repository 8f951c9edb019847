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
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "kernel_common.h"

using namespace hrt;
using namespace hrt::lane;
using namespace hrt::kern;

namespace {

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

/* The general kernel (every feature): each iteration of the wave loop advances every busy lane by
 * exactly one ray segment.  Lanes whose path ended start their next sample in the same iteration. */
#ifndef HRT_GEN_WAVES
#define HRT_GEN_WAVES 0 /* waves/SIMD cap of the general (FULL) segment kernel; 0 = compiler's choice */
#endif
template <bool FULL, bool LDS, bool FAST>
constexpr int general_min_waves() { return FULL && HRT_GEN_WAVES > 0 ? HRT_GEN_WAVES : 1; }

/* the FULL segment kernel needs ~140 VGPRs (3 waves/SIMD): 256-thread workgroups, so that three of
 * them (each with its own LDS copy of a small scene) fill a CU */
template <bool FULL, bool LDS, bool FAST>
constexpr int general_block_threads() { return FULL ? 256 : block_threads<LDS, FAST>(); }

/* GW > 0: this instantiation is built for GW waves/SIMD (plan() picks 4 for general scenes: +18% on
 * Cornell, +4% on Final; 3, the compiler's choice, for small noise-texture scenes, whose Perlin path
 * spills at 128 VGPRs) */
template <int CULL, bool FULL, bool COUNT, bool LDS, bool FAST, int GW = 0, int TRIM = 0>
__global__ __launch_bounds__((general_block_threads<FULL, LDS, FAST>()), (GW > 0 ? GW : general_min_waves<FULL, LDS, FAST>()))
void render_kernel(KParams P) {
  extern __shared__ float4 lds_scene[];
  const G::Node* nodes = P.nodes;
  const G::Prim* prims = P.prims;
  if constexpr (LDS) stage_scene(P, lds_scene, nodes, prims);
  const uint32_t lane = threadIdx.x & 63u;
  const float scale = 1.0f / (float)P.spp; /* application.rs:403 */

  bool has_item = false, exhausted = false, in_path = false;
  Item it{0u, 0u, 0u, 0u};
  WaveBlock wb{0u, 0u};
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
    claim_work(P, lane, has_item, exhausted, it, wb);
    if (!__any(has_item || !exhausted)) break;
    if (!has_item) continue;
    if (!in_path) {
      start_sample(P, ps, it.pxy & 0xFFFFu, it.pxy >> 16, it.sample);
      in_path = true;
    }
    const uint32_t nodes_before = cn.nodes;
    const bool done = segment<CULL, FULL, COUNT, FAST, TRIM>(P, nodes, prims, ps, cn, nullptr);
    if constexpr (COUNT) seg_nodes = cn.nodes - nodes_before;
    if (ps.traced) n_seg++;
    if (done) {
      in_path = false;
      finish_sample(P, it, sum, ps.rad, scale, has_item, n_samples, n_pixels);
    }
  }
  flush_stats(P, n_seg, n_samples, n_pixels, cn, COUNT);
}

/* The general kernel with persistent walks and postponed shading (render_basic_kernel's structure;
 * see there).  Rects, instances, media and every texture. */
template <int CULL, bool COUNT, bool LDS>
__global__ __launch_bounds__((basic_block_threads<LDS, FULL_WAVES>()), FULL_WAVES)
void render_full_kernel(KParams P) {
  extern __shared__ float4 lds_scene[];
  const G::Node* nodes = P.nodes;
  const G::Prim* prims = P.prims;
  if constexpr (LDS) stage_scene(P, lds_scene, nodes, prims);
  const uint32_t lane = threadIdx.x & 63u;
  const float scale = 1.0f / (float)P.spp; /* application.rs:403 */
  const float inf = __uint_as_float(0x7f800000u);
  const uint32_t need = P.postpone;

  bool has_item = false, exhausted = false;
  bool walking = false;
  Item it{0u, 0u, 0u, 0u};
  WaveBlock wb{0u, 0u};
  Vec3 sum = v3(0.0f, 0.0f, 0.0f);
  PathState ps;
  init_path_state(ps);
  TRay r;
  set_ray(r, ps.ro, ps.rd, 0.0f, P);
  Vec3 wo = ps.ro, wd = ps.rd;
  FullWalk w{G::NONE, 0u, 0u, 0u, 0.0f, inf, G::NONE, inf, 0.0f, G::NONE};
  uint32_t n_seg = 0, n_samples = 0, n_pixels = 0;
  Counts cn{0u, 0u, 0u, 0u, 0u, 0u};

  auto begin_walk = [&]() {
    wo = ps.ro;
    wd = ps.rd;
    w.i = 0u;
    w.end = P.main_end;
    w.mode = 0u;
    w.tmin = P.t_min;
    w.cl = inf;
    w.wn = G::NONE;
  };

  for (;;) {
    claim_work(P, lane, has_item, exhausted, it, wb);
    if (!__any(has_item || !exhausted)) break;
    if (has_item && !walking) {
      start_sample(P, ps, it.pxy & 0xFFFFu, it.pxy >> 16, it.sample);
      walking = true;
      set_ray(r, ps.ro, ps.rd, ps.rtime, P);
      begin_walk();
      if (ps.depth_left == 0) w.i = G::NONE; /* max_depth 0: black without a world.hit (:478-480) */
    }
    if constexpr (COUNT) cn.shade_slots++;
    const unsigned long long walkers = __ballot(walking);
    uint32_t iters = 0;
    bool stuck = false;
    for (;;) {
#pragma unroll
      for (int u = 0; u < WALK_UNROLL; u++) {
        if constexpr (COUNT) cn.walk_slots++;
        if (w.i < w.end) full_step<CULL, COUNT>(P, nodes, prims, w, r, wo, wd, ps.pk, cn);
      }
      const unsigned long long live = __ballot(w.i < w.end);
      if (!live || (uint32_t)__popcll(walkers & ~live) >= need) break;
      if (++iters > P.walk_cap) { stuck = true; break; }
    }
    if (stuck) { /* a walk that cannot end (corrupt scene data): report it, retire the wave */
      if (lane == 0) atomicOr(&P.stats[12], 1ull);
      exhausted = true;
      has_item = false;
      walking = false;
      w.i = G::NONE;
      w.end = 0u;
    }
    const bool shading = walking && w.i >= w.end;
    const bool traced = shading && w.i != G::NONE;
    bool sample_done = false, chunk_done = false;
    if (shading) {
      bool done = true;
      if (traced) {
        ps.pk.segment++;
        done = shade<true, COUNT>(P, ps, w.wn, w.cl, wo, wd, r.time, r.tau, cn) || ps.depth_left == 0;
      }
      if (done) {
        walking = false;
        w.i = G::NONE;
        w.end = 0u;
        sum = sum + ps.rad;
        sample_done = true;
        if (++it.sample == it.sample_end) {
          if (P.n_chunks == 1)
            P.out[it.slot] = make_float4(sqrtf(sum.x * scale), sqrtf(sum.y * scale), sqrtf(sum.z * scale), 1.0f);
          else
            P.partial[it.slot] = make_float4(sum.x, sum.y, sum.z, 0.0f);
          chunk_done = true;
          has_item = false;
          sum = v3(0.0f, 0.0f, 0.0f);
        }
      } else {
        set_dir(r, ps.ro, ps.rd); /* the scattered ray keeps the sample's shutter time */
        begin_walk();
      }
    }
    n_seg += (uint32_t)__popcll(__ballot(traced));
    n_samples += (uint32_t)__popcll(__ballot(sample_done));
    n_pixels += (uint32_t)__popcll(__ballot(chunk_done && it.sample_end <= P.chunk));
  }
  if (lane == 0) {
    atomicAdd(&P.stats[0], (unsigned long long)n_seg);
    atomicAdd(&P.stats[1], (unsigned long long)n_samples);
    atomicAdd(&P.stats[2], (unsigned long long)n_pixels);
  }
  if constexpr (COUNT) flush_counts(P, cn);
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
    case 7: r = div_rn(a, b, div_rn_y(b)); break; /* the walk's division by dot(d, d) */
    case 8: r = __int_as_float(sat_f2i32(a)); break; /* Rust `as i32` (the Perlin lattice): the bits */
    case 9: r = __uint_as_float(sat_f2u32(a)); break; /* Rust `as u32` (image texel indices): the bits */
  }
  out[i] = r;
}

/* hrt_debug_box_test: the walk's inflated box test (lane.h box_ce) on (box, ray) pairs, the same code on the
 * device and on the host (this file's host compilation of lane.h) */
template <bool FMA>
HRT_LANE_FI uint8_t box_pair(const float* boxes, const float* rays, uint32_t b, uint32_t q, float tmin, float tmax) {
  TRay r;
  set_dir(r, v3(rays[6 * q], rays[6 * q + 1], rays[6 * q + 2]), v3(rays[6 * q + 3], rays[6 * q + 4], rays[6 * q + 5]));
  const float4 c = make_float4(boxes[8 * b], boxes[8 * b + 1], boxes[8 * b + 2], 0.0f);
  const float4 e = make_float4(boxes[8 * b + 4], boxes[8 * b + 5], boxes[8 * b + 6], 0.0f);
  return box_ce<FMA>(c, e, r, tmin, tmax) ? 1u : 0u;
}

__global__ void box_test_kernel(int form, const float* boxes, uint32_t nb, const float* rays, uint32_t nr, float tmin,
                                float tmax, uint8_t* out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (uint64_t)nb * nr) return;
  const uint32_t b = (uint32_t)(i / nr), q = (uint32_t)(i % nr);
  out[i] = form ? box_pair<true>(boxes, rays, b, q, tmin, tmax) : box_pair<false>(boxes, rays, b, q, tmin, tmax);
}

/* ------------------------------------------------------------------ host helpers */
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

constexpr size_t SLOT_HDR = 256; /* work counter (8 B), stats words 0-11, error word 12, stats words 13-16 */

constexpr const char* SLOT_ERROR_MSG =
    "a render launch on this scene stopped walks that did not terminate (corrupt scene data); its frame is incomplete";

/* Render parameters every kernel entry point accepts: 2 <= W, H <= 65535 (start_sample's camera
 * divisions use host reciprocals proven exact there, lane.h), spp > 0, known flags, a shutter interval. */
void check_render_args(const hrt_camera* cam, const hrt_render_params* p) {
  if (p->width < 2 || p->height < 2 || p->width > 65535 || p->height > 65535 || p->samples == 0 ||
      (p->flags & ~(uint32_t)(HRT_RENDER_COUNT_WORK | HRT_RENDER_NO_LDS | HRT_RENDER_REFERENCE_CULL |
                              HRT_RENDER_FAST_CULL | HRT_RENDER_SAH)) != 0)
    throw HipError{HRT_ERR_INVALID_ARG, "bad render params (2 <= width, height <= 65535, samples > 0, known flags)"};
  if (!(cam->time0 < cam->time1)) throw HipError{HRT_ERR_INVALID_ARG, "camera time0 must be < time1"};
}

/* The watchdog's error word of a slot's finished launch (pinned copy, word 12): report it once. */
void take_slot_error(hrt_scene::Slot& sl) {
  unsigned long long* h = (unsigned long long*)sl.h_tiles;
  if (h && h[12] != 0) {
    const unsigned long long e = h[12];
    h[12] = 0;
    if (e & 2ull) throw HipError{HRT_ERR_STATE, "the sphere kernel's LDS did not start at address 0 (walk stream not staged)"};
    throw HipError{HRT_ERR_STATE, SLOT_ERROR_MSG};
  }
}


template <int CULL, bool FULL, bool COUNT, bool LDS, bool FAST, int GW = 0, int TRIM = 0>
void launch(const KParams& kp, int device, hipStream_t stream, size_t smem) {
  const void* fn = (const void*)render_kernel<CULL, FULL, COUNT, LDS, FAST, GW, TRIM>;
  const int block = general_block_threads<FULL, LDS, FAST>();
  const int grid = resident_grid(fn, block, device, LDS ? smem : 0, LDS, __PRETTY_FUNCTION__);
  hipLaunchKernelGGL((render_kernel<CULL, FULL, COUNT, LDS, FAST, GW, TRIM>), dim3(grid), dim3(block), LDS ? smem : 0,
                     stream, kp);
  hip_check(hipGetLastError(), "render_kernel launch");
}

template <int CULL, bool COUNT, bool LDS>
void launch_full(const KParams& kp, int device, hipStream_t stream, size_t smem) {
  const void* fn = (const void*)render_full_kernel<CULL, COUNT, LDS>;
  const int block = basic_block_threads<LDS, FULL_WAVES>();
  const int grid = resident_grid(fn, block, device, LDS ? smem : 0, LDS, __PRETTY_FUNCTION__);
  hipLaunchKernelGGL((render_full_kernel<CULL, COUNT, LDS>), dim3(grid), dim3(block), LDS ? smem : 0, stream, kp);
  hip_check(hipGetLastError(), "render_full_kernel launch");
}

/* LDS residency: the scene a sphere-kernel workgroup stages (the walk stream, or the reference-order
 * stream) must fit twice per CU (two workgroups of the 160 KiB), the 8 SAH octant streams once (one
 * 1024-thread workgroup). */
constexpr size_t LDS_SCENE_MAX = G::LDS_SCENE_MAX_BYTES;
constexpr size_t LDS_FAST_MAX = 150 * 1024;
constexpr size_t LDS_GEN_MAX = 48 * 1024;

struct Plan {
  bool full, fast, lds;
  bool heavy;    /* sphere scene with noise / image textures on the sphere kernel (HEAVY instantiation) */
  bool perlin_lds; /* the Perlin tables staged in LDS (sphere HEAVY and gwalk kernels) */
  bool gwalk;    /* general scene on render_gwalk_kernel (the general walk stream, render_general.hip) */
  int gwalk_mem; /* its walk-stream placement: WM_LDS / WM_HYB / WM_BUF */
  bool gwalk_lref; /* ... with the reference stream and primitives staged in LDS too */
  bool gwalk_packet; /* ... walked by the wave as one packet (a small stream staged whole in LDS) */
  bool sphere_packet; /* sphere kernel: a tiny walk stream staged whole in LDS walked as one packet */
  int gen_waves; /* general scenes under CULL_EXACT: the render_kernel<FULL> instantiation (3 or 4 waves/SIMD) */
  int trim;      /* general scenes: features compiled out of render_kernel (lane.h TRIM_*) */
  bool general; /* sphere scene forced onto the general kernel (diagnostics: HRT_KERNEL=general) */
  int cull;
  size_t smem;
};

Plan plan(const hrt_scene* s, const hrt_camera* cam, uint32_t flags) {
  Plan pl;
  /* a sphere scene whose walk stream is the GENERAL one (a List inside a BvhNode leaf: scene.cpp build_walk)
   * runs the general kernels: the sphere kernel would read its 48-B leaf programs as sphere payloads */
  pl.full = (s->feature_mask & ~G::F_BASIC) != 0 || s->w_general;
  pl.heavy = false;
  pl.perlin_lds = false;
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
                    : (s->g_nodes.size() * sizeof(G::Node) + s->g_prims.size() * sizeof(G::Prim));
  /* the sphere kernel under CULL_EXACT stages the walk stream (layout.h) instead: whole, or its top
   * levels (w_hot) when it exceeds the LDS budget */
  if (!pl.full && !pl.fast && pl.cull == G::CULL_EXACT) pl.smem = s->w_hot ? s->w_hot : s->w_end;
  pl.lds = (flags & HRT_RENDER_NO_LDS) == 0 && pl.smem <= (pl.fast ? LDS_FAST_MAX : LDS_SCENE_MAX);
  const char* k = knob_env("HRT_KERNEL");
  /* General scenes run the segment-at-a-time kernel by default; render_full_kernel (persistent walks)
   * is opt-in (HRT_KERNEL=persistent) until it has been measured and validated on the GPU.  Sphere
   * scenes can be sent to the segment kernel for diagnostics (HRT_KERNEL=general). */
  const bool persistent = k && strcmp(k, "persistent") == 0;
  pl.general = (k && strcmp(k, "general") == 0) || s->media_nested || (pl.full && !persistent);
  /* render_kernel<FULL>: node stream + primitives in LDS when they fit three 256-thread workgroups per
   * CU (HRT_GEN_LDS=0: global memory, for A/B) */
  const char* gl = knob_env("HRT_GEN_LDS");
  if (pl.general && pl.full && (pl.smem > LDS_GEN_MAX || (gl && strcmp(gl, "0") == 0))) pl.lds = false;
  const char* gw = knob_env("HRT_GEN_WAVES_RT"); /* A/B override: 3 or 4 */
  pl.gen_waves = gw ? (strcmp(gw, "3") == 0 ? 3 : 4) : ((s->feature_mask & G::F_NOISE) && pl.lds ? 3 : 4);
  const char* lt = knob_env("HRT_GEN_TRIM"); /* A/B knob: "0" keeps the all-feature instantiation */
  /* instantiated: all features (0), no noise / image textures (HEAVY_TEX: Cornell-smoke 124 VGPRs, no
   * spills, +1.9%), neither those nor media (Cornell: 92 VGPRs, 5 waves/SIMD, +19%).  Trimming the
   * medium branch alone measured -0.6 / -1% (Earth+Perlin, simple-light), so it is not built. */
  /* sphere scenes with noise / image textures (Earth + Perlin) under exact culling: the sphere kernel's
   * HEAVY instantiation over the sphere walk stream (HRT_KERNEL=segment keeps the segment kernel) */
  const bool seg = k && strcmp(k, "segment") == 0;
  if (pl.full && (s->feature_mask & ~(G::F_BASIC | G::F_HEAVY_TEX)) == 0 && pl.cull == G::CULL_EXACT && !s->w_general &&
      s->w_end > 0 && !seg && !(k && strcmp(k, "general") == 0) && !(k && strcmp(k, "persistent") == 0)) {
    pl.full = false;
    pl.heavy = true;
    pl.general = false;
    pl.smem = s->w_hot ? s->w_hot : s->w_end;
    pl.lds = (flags & HRT_RENDER_NO_LDS) == 0 && pl.smem <= LDS_SCENE_MAX;
    const size_t perlin = s->perlin.size() * sizeof(G::Perlin);
    const char* pe = knob_env("HRT_PERLIN_LDS"); /* A/B knob: "0" keeps the Perlin tables in global memory */
    const size_t at = (pl.smem + G::PERLIN_LDS_ALIGN - 1) / G::PERLIN_LDS_ALIGN * G::PERLIN_LDS_ALIGN; /* stage_perlin */
    pl.perlin_lds = pl.lds && perlin > 0 && at + perlin <= LDS_SCENE_MAX && !(pe && strcmp(pe, "0") == 0);
    if (pl.perlin_lds) pl.smem = at + perlin;
  }
  /* the sphere kernel's packet walk (render_sphere.hip PACKET) for streams of at most SPHERE_PACKET_NODES node parts */
  {
    const char* sp = knob_env("HRT_SPHERE_PACKET"); /* A/B knob: "0" keeps the per-lane walk, "1" forces the packet */
    pl.sphere_packet = !pl.full && !pl.fast && pl.lds && pl.cull == G::CULL_EXACT && !s->w_hot && !s->w_general &&
                       (sp ? strcmp(sp, "1") == 0 : s->w_nodes <= G::SPHERE_PACKET_NODES);
  }
  pl.trim = 0;
  if ((s->feature_mask & (G::F_NOISE | G::F_IMAGE)) == 0)
    pl.trim = TRIM_HEAVY_TEX | ((s->feature_mask & G::F_MEDIUM) == 0 && !s->media_nested ? TRIM_MEDIA : 0);
  if (lt && strcmp(lt, "0") == 0) pl.trim = 0;
  /* General scenes under exact culling: render_gwalk_kernel over the general walk stream (persistent
   * walks, postponed shading, batched leaf programs) unless HRT_KERNEL asks for a segment kernel. */
  pl.gwalk = pl.full && s->w_general && s->w_end > 0 && pl.cull == G::CULL_EXACT && !s->media_nested &&
             !(k && (strcmp(k, "general") == 0 || strcmp(k, "persistent") == 0 || strcmp(k, "segment") == 0));
  pl.gwalk_mem = WM_BUF;
  pl.gwalk_lref = false;
  pl.gwalk_packet = false;
  if (pl.gwalk) {
    pl.general = false;
    const size_t walk = s->w_hot ? s->w_hot : s->w_end;
    /* everything leaf programs and shading read, but the Perlin tables and images */
    const size_t ref = s->g_nodes.size() * sizeof(G::Node) + s->g_prims.size() * sizeof(G::Prim) +
                       s->g_insts.size() * sizeof(G::Inst) + s->g_media.size() * sizeof(G::Medium) +
                       s->g_mats.size() * sizeof(G::Mat) + s->g_texs.size() * sizeof(G::Tex) +
                       s->g_chains.size() * sizeof(float);
    const bool no_lds = (flags & HRT_RENDER_NO_LDS) != 0;
    /* a hybrid general stream's staged part may take one 1024-thread workgroup's LDS (GWALK_LDS_BIG_BYTES) */
    pl.gwalk_mem = no_lds || walk > (s->w_hot ? (size_t)G::GWALK_LDS_BIG_BYTES : LDS_SCENE_MAX) ? WM_BUF
                                                                                             : (s->w_hot ? WM_HYB : WM_LDS);
    const char* lr = knob_env("HRT_GWALK_LREF"); /* A/B knob: "0" keeps the reference stream in global memory */
    pl.gwalk_lref = pl.gwalk_mem == WM_LDS && walk + ref <= LDS_SCENE_MAX && !(lr && strcmp(lr, "0") == 0);
    pl.smem = pl.gwalk_mem == WM_BUF ? 0 : walk + (pl.gwalk_lref ? ref : 0);
    const size_t perlin = s->perlin.size() * sizeof(G::Perlin);
    const char* pe = knob_env("HRT_PERLIN_LDS");
    const size_t at = (pl.smem + G::PERLIN_LDS_ALIGN - 1) / G::PERLIN_LDS_ALIGN * G::PERLIN_LDS_ALIGN; /* stage_perlin */
    pl.perlin_lds = pl.gwalk_lref && perlin > 0 && at + perlin <= LDS_SCENE_MAX && !(pe && strcmp(pe, "0") == 0);
    if (pl.perlin_lds) pl.smem = at + perlin;
    pl.lds = pl.gwalk_mem != WM_BUF;
    /* the packet walk (render_general.hip) for streams of at most GWALK_PACKET_NODES node parts staged whole in
     * LDS with their reference arrays whose leaves run generic programs (s->w_generic: Cornell-smoke's media in
     * rotated boxes): a wave's lanes visit at most that many nodes together per segment */
    const char* pk = knob_env("HRT_GWALK_PACKET"); /* A/B knob: "0" keeps the per-lane speculative walk, "1" forces it */
    pl.gwalk_packet = pl.gwalk_lref && s->w_nodes <= G::GWALK_PACKET_NODES &&
                      (pk ? strcmp(pk, "1") == 0 : s->w_generic);
    pl.trim = ((s->feature_mask & (G::F_NOISE | G::F_IMAGE)) == 0 ? TRIM_HEAVY_TEX : 0) |
              ((s->feature_mask & G::F_MEDIUM) == 0 ? TRIM_MEDIA : 0);
    const char* tp = knob_env("HRT_GWALK_TRIMP"); /* A/B knob: "0" keeps trace_ray's generic program compiled in */
    if (!s->w_generic && !(tp && strcmp(tp, "0") == 0)) pl.trim |= TRIM_PROGRAMS;
    if (lt && strcmp(lt, "0") == 0) pl.trim = 0;
    if (pl.trim & TRIM_PROGRAMS) pl.gwalk_packet = false; /* instantiated with the generic program only */
  }
  return pl;
}

template <bool COUNT>
void launch_any(const hrt_scene* s, const Plan& pl, const KParams& kp, hipStream_t stream) {
  const size_t smem = pl.lds ? pl.smem : 0;
  if (pl.gwalk) {
    /* every chunk one sample (head of 1-sample chunks, no tail): render_gwalk_kernel's ONE instantiation */
    const char* o1 = knob_env("HRT_GWALK_ONE"); /* A/B knob: "0" keeps the general chunk loop */
    const bool one = kp.chunk == 1u && kp.chunk_first == 1u && kp.n_chunks == kp.chunk_head && !(o1 && strcmp(o1, "0") == 0);
    launch_gwalk(COUNT, pl.gwalk_mem, pl.gwalk_lref, pl.trim, one, pl.gwalk_packet, kp, s->device, stream, smem);
    return;
  }
  if (pl.fast) {
    if (pl.lds) launch<G::CULL_SLAB, false, COUNT, true, true>(kp, s->device, stream, smem);
    else launch<G::CULL_SLAB, false, COUNT, false, true>(kp, s->device, stream, 0);
  } else if (pl.general) {
    const int c = pl.cull;
    if (pl.full) {
      if (c == G::CULL_EXACT && pl.gen_waves == 4 && pl.trim != 0) {
        if (pl.trim == (TRIM_MEDIA | TRIM_HEAVY_TEX))
          pl.lds ? launch<G::CULL_EXACT, true, COUNT, true, false, 4, TRIM_MEDIA | TRIM_HEAVY_TEX>(kp, s->device, stream, smem)
                 : launch<G::CULL_EXACT, true, COUNT, false, false, 4, TRIM_MEDIA | TRIM_HEAVY_TEX>(kp, s->device, stream, 0);
        else
          pl.lds ? launch<G::CULL_EXACT, true, COUNT, true, false, 4, TRIM_HEAVY_TEX>(kp, s->device, stream, smem)
                 : launch<G::CULL_EXACT, true, COUNT, false, false, 4, TRIM_HEAVY_TEX>(kp, s->device, stream, 0);
      } else if (c == G::CULL_EXACT && pl.gen_waves == 4)
        pl.lds ? launch<G::CULL_EXACT, true, COUNT, true, false, 4>(kp, s->device, stream, smem)
               : launch<G::CULL_EXACT, true, COUNT, false, false, 4>(kp, s->device, stream, 0);
      else if (c == G::CULL_EXACT) pl.lds ? launch<G::CULL_EXACT, true, COUNT, true, false>(kp, s->device, stream, smem)
                                          : launch<G::CULL_EXACT, true, COUNT, false, false>(kp, s->device, stream, 0);
      else if (c == G::CULL_SLAB) pl.lds ? launch<G::CULL_SLAB, true, COUNT, true, false>(kp, s->device, stream, smem)
                                         : launch<G::CULL_SLAB, true, COUNT, false, false>(kp, s->device, stream, 0);
      else pl.lds ? launch<G::CULL_REFERENCE, true, COUNT, true, false>(kp, s->device, stream, smem)
                  : launch<G::CULL_REFERENCE, true, COUNT, false, false>(kp, s->device, stream, 0);
      return;
    }
    if (c == G::CULL_EXACT) pl.lds ? launch<G::CULL_EXACT, false, COUNT, true, false>(kp, s->device, stream, smem)
                                   : launch<G::CULL_EXACT, false, COUNT, false, false>(kp, s->device, stream, 0);
    else if (c == G::CULL_SLAB) pl.lds ? launch<G::CULL_SLAB, false, COUNT, true, false>(kp, s->device, stream, smem)
                                       : launch<G::CULL_SLAB, false, COUNT, false, false>(kp, s->device, stream, 0);
    else pl.lds ? launch<G::CULL_REFERENCE, false, COUNT, true, false>(kp, s->device, stream, smem)
                : launch<G::CULL_REFERENCE, false, COUNT, false, false>(kp, s->device, stream, 0);
  } else if (pl.cull == G::CULL_EXACT) {
    if (pl.full) pl.lds ? launch_full<G::CULL_EXACT, COUNT, true>(kp, s->device, stream, smem)
                        : launch_full<G::CULL_EXACT, COUNT, false>(kp, s->device, stream, 0);
    else launch_sphere(G::CULL_EXACT, COUNT, pl.lds, pl.heavy, pl.sphere_packet, kp, s->device, stream, smem);
  } else if (pl.cull == G::CULL_SLAB) {
    if (pl.full) pl.lds ? launch_full<G::CULL_SLAB, COUNT, true>(kp, s->device, stream, smem)
                        : launch_full<G::CULL_SLAB, COUNT, false>(kp, s->device, stream, 0);
    else launch_sphere(G::CULL_SLAB, COUNT, pl.lds, false, false, kp, s->device, stream, smem);
  } else {
    if (pl.full) pl.lds ? launch_full<G::CULL_REFERENCE, COUNT, true>(kp, s->device, stream, smem)
                        : launch_full<G::CULL_REFERENCE, COUNT, false>(kp, s->device, stream, 0);
    else launch_sphere(G::CULL_REFERENCE, COUNT, pl.lds, false, false, kp, s->device, stream, smem);
  }
}

/* BASIC-kernel tuning knob, 1..64 lanes (read per launch; any value gives the same image):
 *   HRT_POSTPONE   a wave leaves the walk to shade once this many lanes have finished theirs;
 *   HRT_PRIM_BATCH the wave runs its primitive tests once this many lanes wait for one. */
uint32_t env_knob(const char* name, uint32_t dflt) {
  const char* e = knob_env(name);
  const long x = e ? strtol(e, nullptr, 10) : 0;
  return (uint32_t)(x >= 1 && x <= 64 ? x : dflt);
}

/* A render's sample chunks (lane.h frame_chunks): its inputs are the spp, the scene's class, the full image
 * size and the scene's options (hrt_scene_options), never the environment. */
void chunk_schedule(const hrt_scene* s, const hrt_render_params* p, uint32_t& chunk, uint32_t& n_head, uint32_t& first,
                    uint32_t& n_tail) {
  frame_chunks(p->samples, chunk_class(s->feature_mask, s->main_end), p->width, p->height, s->opts.chunk_min,
               s->opts.chunk_max, s->opts.chunk_uniform ? 0u : 32u, chunk, n_head, first, n_tail);
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
  kp.chains = (const float4*)(base + s->off_chains);
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
  set_pixel_rcp(kp);
  kp.spp = p->samples;
  kp.max_depth = p->max_depth;
  kp.sample_offset = p->sample_offset;
  kp.t_min = p->t_min;
  kp.background = v3(p->background[0], p->background[1], p->background[2]);
  kp.seed = p->seed;
  kp.n_nodes = pl.fast ? 8 * s->f_stream_len : (uint32_t)s->g_nodes.size(); /* main stream + medium boundary subtrees */
  kp.n_prims = (uint32_t)(pl.fast ? s->f_prims.size() : s->g_prims.size());
  kp.n_insts = (uint32_t)s->g_insts.size();
  kp.n_media = (uint32_t)s->g_media.size();
  kp.n_mats = (uint32_t)s->g_mats.size();
  kp.n_texs = (uint32_t)s->g_texs.size();
  kp.n_perlin = (uint32_t)s->perlin.size();
  kp.perlin_lds = pl.perlin_lds ? 1u : 0u;
  kp.stream_len = pl.fast ? s->f_stream_len : 0;
  /* the sphere kernel's speculative walk (render_sphere.hip SPEC) blocks lanes less often: it runs best
   * with smaller batches; deep streams (top levels in LDS, w_hot: long walks) shade earlier (r02z sweep
   * of postpone {40..56} x batch {4, 6, 8}: C2 best at 52-56 / 4, random-10k at 44 / 4, +1.8% over 48 / 6;
   * DESIGN.md section 10) */
  const bool spec = !pl.full && !pl.general && !pl.fast && pl.cull == G::CULL_EXACT;
  /* gwalk (r04 sweeps, one box): streams in LDS (Cornell 1/8 share, 1250 spp) batch 16 / 32 = 14183 / 14014;
   * deep streams staged in part (Final 800^2 x 64: many leaf programs per ray) batch 32 / 16 / 8 / 4 = 1258 /
   * 1373 / 1430 / 1389, postpone 52 / 44 / 32 = 1131 / 1188 / 1385 (batch 32) */
  const bool deep = pl.gwalk && pl.gwalk_mem != WM_LDS;
  kp.postpone = env_knob("HRT_POSTPONE", pl.gwalk ? (deep ? 32 : 44) : (spec ? (s->w_hot ? 44 : 52) : 56));
  kp.prim_batch = env_knob("HRT_PRIM_BATCH", pl.gwalk ? (deep ? 8 : 16) : (spec ? 4 : 8));
  /* a walk visits each node at most once, a medium's boundary subtree at most twice per medium node */
  kp.walk_cap = 3u * (uint32_t)s->g_nodes.size() + 64u;
  kp.motion_uniform = s->motion_uniform ? 1u : 0u;
  kp.motion_t0 = s->motion_t0;
  kp.motion_span = s->motion_span;
  kp.walk = base + s->off_walk;
  kp.walk_bytes = s->w_end;
  kp.walk_end = s->w_c16 ? s->w_nodes : s->w_end; /* layout.h WALK_C16: positions are node indices */
  kp.walk_c16 = s->w_c16 ? 1u : 0u;
  kp.walk_pbase = s->w_pbase;
  kp.walk_hot = (pl.gwalk && pl.gwalk_mem == WM_HYB) || (pl.lds && !pl.full && !pl.fast && pl.cull == G::CULL_EXACT)
                    ? s->w_hot : 0;
  kp.walk_half = s->w_half;
  return kp;
}

}  // namespace

/* ============================================================================ device runtime */
namespace {
/* hrt_render's device output buffers (scene_internal.h out_pool): taken and given back under the pool's
 * mutex; a buffer too small for a call is freed and replaced */
struct OutBuf {
  void* ptr;
  size_t cap;
};
struct OutPool {
  std::mutex mu;
  std::vector<OutBuf> free;
};
OutBuf out_pool_take(hrt_scene* s, size_t bytes) {
  OutPool* pool = static_cast<OutPool*>(s->out_pool);
  OutBuf b{nullptr, 0};
  {
    std::lock_guard<std::mutex> lk(pool->mu);
    if (!pool->free.empty()) {
      b = pool->free.back();
      pool->free.pop_back();
    }
  }
  if (b.cap < bytes) {
    if (b.ptr) hip_check(hipFree(b.ptr), "hipFree(out)");
    b = OutBuf{nullptr, 0};
    hip_check(hipMalloc(&b.ptr, bytes), "hipMalloc(out)");
    b.cap = bytes;
  }
  return b;
}
void out_pool_give(hrt_scene* s, OutBuf b) {
  if (!b.ptr) return;
  OutPool* pool = static_cast<OutPool*>(s->out_pool);
  std::lock_guard<std::mutex> lk(pool->mu);
  pool->free.push_back(b);
}
}  // namespace

namespace hrt {

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw HipError{HRT_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e)};
}

namespace {
struct GridKey {
  const void* fn;
  int device;
  size_t smem;
  hrt_launch_info info;
};
thread_local hrt_launch_info t_last_launch;
thread_local bool t_has_launch = false;

/* "void ns::launch_basic(...) [CULL = 2, COUNT = false, ...]" -> "launch_basic[CULL = 2, COUNT = false, ...]" */
void launch_name(const char* pretty, char* out, size_t cap) {
  std::string s(pretty ? pretty : "?");
  for (size_t a; (a = s.find("(anonymous namespace)")) != std::string::npos;) s.erase(a, 21);
  const size_t paren = s.find('(');
  std::string head = s.substr(0, paren);
  const size_t sp = head.find_last_of(" :");
  head = sp == std::string::npos ? head : head.substr(sp + 1);
  const size_t br = s.find('[');
  std::string name = head + (br == std::string::npos ? std::string() : s.substr(br));
  snprintf(out, cap, "%s", name.c_str());
}
}  // namespace

/* The knobs this launch ran with: those set now (read by the launch) and those set when its scene
 * was committed (placement knobs, "commit:NAME=value"), snapshotted into the thread's launch record, so a knob
 * set for the commit and unset before the launch is still reported. */
void launch_knobs(const hrt_scene* s) {
  std::string k = knobs_in_effect();
  size_t a = 0;
  const std::string& c = s->commit_knobs;
  while (a < c.size()) {
    size_t b = c.find(';', a);
    if (b == std::string::npos) b = c.size();
    if (!k.empty()) k += ';';
    k += "commit:" + c.substr(a, b - a);
    a = b + 1;
  }
  snprintf(t_last_launch.knobs, sizeof(t_last_launch.knobs), "%s", k.c_str());
}

int resident_grid(const void* fn, int block, int device, size_t smem, bool lds, const char* name) {
  static std::mutex mu;
  static std::vector<GridKey> cache;
  std::lock_guard<std::mutex> lk(mu);
  for (const GridKey& k : cache)
    if (k.fn == fn && k.device == device && k.smem == smem) {
      t_last_launch = k.info;
      t_has_launch = true;
      return (int)k.info.grid;
    }
  if (lds) hip_check(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem),
                     "hipFuncSetAttribute(LDS)");
  int per_cu = 0;
  hip_check(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, block, smem),
            "hipOccupancyMaxActiveBlocksPerMultiprocessor");
  hipDeviceProp_t prop;
  hip_check(hipGetDeviceProperties(&prop, device), "hipGetDeviceProperties");
  hipFuncAttributes fa;
  memset(&fa, 0, sizeof(fa));
  hip_check(hipFuncGetAttributes(&fa, fn), "hipFuncGetAttributes");
  const int g = std::max(1, per_cu) * prop.multiProcessorCount;
  hrt_launch_info li;
  memset(&li, 0, sizeof(li));
  launch_name(name, li.kernel, sizeof(li.kernel));
  li.grid = (uint32_t)g;
  li.block = (uint32_t)block;
  li.blocks_per_cu = (uint32_t)std::max(0, per_cu);
  li.cus = (uint32_t)prop.multiProcessorCount;
  li.waves_per_simd = li.blocks_per_cu * (uint32_t)block / 64u / 4u;
  li.vgprs = (uint32_t)fa.numRegs;
  li.scratch_bytes = (uint32_t)fa.localSizeBytes;
  li.lds_bytes = (uint32_t)smem;
  cache.push_back(GridKey{fn, device, smem, li});
  t_last_launch = li;
  t_has_launch = true;
  return g;
}


hrt_status device_upload(hrt_scene* s, int device) {
  return hguard([&] {
    if (device < 0) hip_check(hipGetDevice(&device), "hipGetDevice");
    DeviceGuard dg(device);
    device_release(s);
    /* the walk stream's re-grouped hierarchy built on the device (build_walk.hip; the host
     * build's hierarchy node for node), for the scenes build_walk left to it (HRT_WALK_BUILD = host |
     * device | auto: the device for scenes of at least 32768 leaves) */
    if (s->w_regroup_pending) {
      std::vector<host::WNode> T;
      const std::vector<host::WalkLeaf> leaves = walk_leaves(s, nullptr, nullptr);
      const auto t0 = std::chrono::steady_clock::now();
      device_walk_regroup(leaves, T, device);
      s->w_build_us = (uint32_t)std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count();
      s->w_regroup_pending = false; /* placed and written as the host build's hierarchy is (16-B parts included) */
      walk_place_and_write(s, T, leaves);
      s->w_device_built = true;
      s->w_regrouped = true;
    }
    std::vector<uint8_t> blob = build_blob(s);
    const size_t off = blob.size();
    s->device = device; /* from here on device_release() cleans up whatever was allocated */
    hip_check(hipMalloc(&s->d_blob, off), "hipMalloc(scene)");
    hip_check(hipMemcpy(s->d_blob, blob.data(), off, hipMemcpyHostToDevice), "hipMemcpy(scene)");
    s->slot_mutex = new std::mutex();
    s->out_pool = new OutPool();
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
  if (OutPool* pool = static_cast<OutPool*>(s->out_pool)) {
    for (const OutBuf& b : pool->free) (void)hipFree(b.ptr);
    delete pool;
  }
  s->out_pool = nullptr;
  if (s->d_blob) (void)hipFree(s->d_blob);
  s->d_blob = nullptr;
  if (prev >= 0) (void)hipSetDevice(prev);
  s->device = -1;
}

}  // namespace hrt

namespace hrt {
/* a device buffer freed on every exit path (the debug entry points throw through hip_check) */
template <typename T>
struct DevBuf {
  T* p = nullptr;
  explicit DevBuf(size_t bytes) { hip_check(hipMalloc((void**)&p, bytes), "hipMalloc(debug)"); }
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
};

}  // namespace hrt

extern "C" {

hrt_status hrt_render_tiles_device(hrt_scene* s, const hrt_camera* cam, const hrt_render_params* p,
                                   const hrt_tile* tiles, uint32_t n_tiles, float* d_rgba, void* stream_,
                                   hrt_render_stats* stats) {
  return hguard([&] {
    if (!s || !cam || !p || !tiles || !d_rgba || n_tiles == 0)
      throw HipError{HRT_ERR_INVALID_ARG, "hrt_render_tiles_device: null argument"};
    if (!s->committed || !s->d_blob) throw HipError{HRT_ERR_STATE, "scene not committed"};
    check_render_args(cam, p);
    /* sample chunks (lane.h sample_chunk): they bound the frame's tail: the last items of a launch run
     * alone, and a pixel whose paths bounce 50 times makes a long item (a 1/8-frame share of C2: chunks
     * of 8 / 16 / 24 / 32 / 63 samples gave 12590 / 12330 / 11628 / 10796 / 9270 Mrays/s; the whole
     * frame 14243 / 14489 / 14489 / 14338 / 13930).  The rule depends on spp and
     * the scene's feature class only, so every tile split sums a pixel's samples in the same chunks. */
    const uint32_t spp = p->samples;
    uint32_t chunk = 0, n_head = 0, first = 0, n_tail = 0;
    chunk_schedule(s, p, chunk, n_head, first, n_tail);
    const uint32_t n_chunks = n_head + n_tail;
    std::vector<G::TileDev> td(n_tiles);
    uint64_t pad = 0, outp = 0;
    for (uint32_t i = 0; i < n_tiles; i++) {
      const hrt_tile& t = tiles[i];
      if (t.w == 0 || t.h == 0 || (uint64_t)t.x + t.w > p->width || (uint64_t)t.y + t.h > p->height)
        throw HipError{HRT_ERR_INVALID_ARG, "tile outside the image"};
      uint32_t bw = (t.w + 7) / 8, bh = (t.h + 7) / 8;
      td[i] = G::TileDev{t.x, t.y, t.w, t.h, bw, (uint32_t)pad, (uint32_t)outp, 0};
      pad += (uint64_t)bw * bh * 64; /* padded pixels (items: pad x n_chunks, chunk-major) */
      outp += (uint64_t)t.w * t.h;
    }
    /* Many tiles (a rank's share of the 16-px grid: 4080 tiles at 2 GPUs): a claim's binary search over
     * the tile table was a dozen dependent global loads.  When padding every tile to the largest one's
     * item count costs at most 1/8 more (idle) items, tile = item / stride instead (share of 2 / 8 on C2:
     * DESIGN.md section 6.1). */
    uint32_t stride = 0;
    if (n_tiles > 1) {
      uint64_t mx = 0;
      for (uint32_t i = 0; i < n_tiles; i++) mx = std::max<uint64_t>(mx, (uint64_t)((td[i].w + 7) / 8) * ((td[i].h + 7) / 8) * 64);
      const char* ts = knob_env("HRT_TILE_STRIDE"); /* A/B knob: "0" keeps the binary search */
      if (mx * n_tiles <= pad + pad / 8 && mx * n_tiles * n_chunks < 0xF0000000ull && !(ts && strcmp(ts, "0") == 0)) {
        stride = (uint32_t)mx;
        for (uint32_t i = 0; i < n_tiles; i++) td[i].pad_start = i * stride;
        pad = mx * n_tiles;
      }
    }
    /* work items and Item.slot (pixel x n_chunks + chunk < pad x n_chunks) are 32-bit */
    /* headroom: waves claim blocks of CLAIM_BLOCK items past the end before they retire */
    if (pad * n_chunks >= 0xF0000000ull) throw HipError{HRT_ERR_UNSUPPORTED, "more than 3.75G pixel x sample-chunk items in one call"};
    hipStream_t stream = (hipStream_t)stream_;
    DeviceGuard dg(s->device);
    /* scratch slot: device [counter u32 | pad | stats 8 x u64 | pad to HDR | tiles], pinned host [stats | tiles] */
    std::lock_guard<std::mutex> lock(*static_cast<std::mutex*>(s->slot_mutex));
    /* an earlier launch whose walks the watchdog killed is reported by the first call that sees its
     * copied-back error word (every launch copies it, with or without stats) */
    for (auto& other : s->slots)
      if (other.used && hipEventQuery((hipEvent_t)other.event) == hipSuccess) take_slot_error(other);
    hrt_scene::Slot& sl = s->slots[s->next_slot++ % hrt_scene::N_SLOTS];
    if (sl.used) {
      hip_check(hipEventSynchronize((hipEvent_t)sl.event), "hipEventSynchronize(slot)");
      take_slot_error(sl);
    }
    size_t tiles_bytes = n_tiles * sizeof(G::TileDev);
    const size_t partial_bytes = n_chunks > 1 ? (size_t)n_chunks * outp * sizeof(float4) : 0;
    auto grow = [&](hrt_scene::Slot& g, bool partial) {
      if (tiles_bytes > g.tiles_cap) {
        if (g.d_mem) hip_check(hipFree(g.d_mem), "hipFree(slot)");
        if (g.h_tiles) hip_check(hipHostFree(g.h_tiles), "hipHostFree(slot)");
        g.d_mem = g.h_tiles = nullptr;
        g.tiles_cap = 0;
        size_t cap = std::max<size_t>(tiles_bytes, 64 * sizeof(G::TileDev));
        hip_check(hipMalloc(&g.d_mem, SLOT_HDR + cap), "hipMalloc(slot)");
        hip_check(hipHostMalloc(&g.h_tiles, SLOT_HDR + cap, hipHostMallocDefault), "hipHostMalloc(slot)");
        g.tiles_cap = cap;
      }
      if (partial && partial_bytes > g.partial_cap) {
        if (g.d_partial) hip_check(hipFree(g.d_partial), "hipFree(partial)");
        g.d_partial = nullptr;
        g.partial_cap = 0;
        hip_check(hipMalloc(&g.d_partial, partial_bytes), "hipMalloc(partial)");
        g.partial_cap = partial_bytes;
      }
    };
    /* slots never launched are grown with this one, so the next calls (e.g. a timed loop that keeps
     * several launches in flight) do not allocate pinned and device memory between launches.  Their
     * partial-sum buffers (a pixel's chunk sums: 1 GB for C2's 32 chunks) only when this call is
     * asynchronous (no stats): a synchronous caller (hrt_render, a progressive batch with stats) never
     * has a second launch in flight, and would otherwise hold N_SLOTS such buffers. */
    const bool first_growth = tiles_bytes > sl.tiles_cap || partial_bytes > sl.partial_cap;
    grow(sl, true);
    if (first_growth)
      for (auto& other : s->slots)
        if (&other != &sl && !other.used) grow(other, stats == nullptr);
    void* scratch = sl.d_mem;
    memcpy((uint8_t*)sl.h_tiles + SLOT_HDR, td.data(), tiles_bytes);
    hip_check(hipMemsetAsync(scratch, 0, SLOT_HDR, stream), "hipMemsetAsync");
    hip_check(hipMemcpyAsync((uint8_t*)scratch + SLOT_HDR, (uint8_t*)sl.h_tiles + SLOT_HDR, tiles_bytes, hipMemcpyHostToDevice,
                             stream), "hipMemcpyAsync(tiles)");
    const Plan pl = plan(s, cam, p->flags);
    KParams kp = scene_params(s, cam, p, pl);
    kp.tiles = (const G::TileDev*)((uint8_t*)scratch + SLOT_HDR);
    kp.n_tiles = n_tiles;
    kp.total_work = (uint32_t)(pad * n_chunks);
    kp.pad_px = (uint32_t)pad;
    kp.head_items = (uint32_t)(pad * n_head);
    kp.tile_stride = stride;
    /* the sphere kernel claims blocks of items to the end: its passes are short, and per-lane claims
     * made them wait on the contended counter (r02y: +12% on C2; per-lane claims for the last 0.26 /
     * 1 / 4 M items measured +0.7 / -0.5 / -3% on C2 and -1 / -9 / -6% on a 1/8-frame share).  The
     * segment kernels claim per lane: a segment iteration is long, claims are rare, and with few items
     * per lane (Cornell 1024^2 x 128: 2) blocks unbalance the waves (-6%).
     * HRT_CLAIM_FINE (A/B knob): claim the last that many items per lane, in every kernel */
    const bool sphere_kernel = (!pl.full && !pl.fast && !pl.general) || pl.gwalk; /* block claims */
    const char* cf = knob_env("HRT_CLAIM_FINE");
    const uint64_t work = pad * n_chunks;
    const uint64_t fine = cf ? strtoull(cf, nullptr, 10) : (sphere_kernel ? 0u : work);
    kp.claim_fine = (uint32_t)(work > fine ? work - fine : 0);
    kp.out = (float4*)d_rgba;
    kp.counter = (uint32_t*)scratch;
    kp.stats = (unsigned long long*)((uint8_t*)scratch + 8);
    kp.chunk = chunk;
    kp.n_chunks = n_chunks;
    kp.chunk_head = n_head;
    kp.chunk_first = first;
    kp.n_out = (uint32_t)outp;
    kp.partial = (float4*)sl.d_partial;
    if (p->flags & HRT_RENDER_COUNT_WORK) launch_any<true>(s, pl, kp, stream);
    else launch_any<false>(s, pl, kp, stream);
    launch_knobs(s);
    if (n_chunks > 1) {
      uint32_t blocks = (uint32_t)std::min<uint64_t>((outp + 255) / 256, 4096);
      hipLaunchKernelGGL(reduce_chunks, dim3(blocks), dim3(256), 0, stream, (const float4*)sl.d_partial,
                         (float4*)d_rgba, (uint32_t)outp, n_chunks, spp);
      hip_check(hipGetLastError(), "reduce_chunks launch");
    }
    /* the stats words and the watchdog's error word (h[12]) come back after EVERY launch, so a killed
     * frame is reported even when the caller asked for no stats (take_slot_error) */
    unsigned long long* h = (unsigned long long*)sl.h_tiles;
    hip_check(hipMemcpyAsync(h, (uint8_t*)scratch + 8, 136, hipMemcpyDeviceToHost, stream), "hipMemcpyAsync(stats)");
    hip_check(hipEventRecord((hipEvent_t)sl.event, stream), "hipEventRecord(slot)");
    sl.used = true;
    if (stats) {
      hip_check(hipEventSynchronize((hipEvent_t)sl.event), "hipEventSynchronize(stats)");
      take_slot_error(sl);
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
      stats->park_slots = h[13];
      stats->wait_slots = h[14];
      stats->leaf_cycles = h[15];
      stats->walk_steps = h[16];
    }
  });
}

hrt_status hrt_scene_synchronize(hrt_scene* s) {
  return hguard([&] {
    if (!s) throw HipError{HRT_ERR_INVALID_ARG, "hrt_scene_synchronize: null scene"};
    if (!s->committed || !s->slot_mutex) return;
    DeviceGuard dg(s->device);
    std::lock_guard<std::mutex> lock(*static_cast<std::mutex*>(s->slot_mutex));
    bool failed = false;
    for (auto& sl : s->slots) {
      if (!sl.used) continue;
      hip_check(hipEventSynchronize((hipEvent_t)sl.event), "hipEventSynchronize(slot)");
      try {
        take_slot_error(sl);
      } catch (const HipError&) {
        failed = true; /* keep draining the other slots, report once */
      }
    }
    if (failed) throw HipError{HRT_ERR_STATE, SLOT_ERROR_MSG};
  });
}

hrt_status hrt_debug_poke_blob(hrt_scene* s, uint64_t offset, const void* data, uint64_t n) {
  return hguard([&] {
    if (!s || !data) throw HipError{HRT_ERR_INVALID_ARG, "hrt_debug_poke_blob: null argument"};
    if (!s->committed || !s->d_blob) throw HipError{HRT_ERR_STATE, "scene not committed"};
    if (offset > s->blob_bytes || n > s->blob_bytes - offset)
      throw HipError{HRT_ERR_INVALID_ARG, "hrt_debug_poke_blob: range outside the scene blob"};
    DeviceGuard dg(s->device);
    hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    hip_check(hipMemcpy((uint8_t*)s->d_blob + offset, data, n, hipMemcpyHostToDevice), "hipMemcpy(poke)");
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
  /* the device output buffer comes from the scene's pool (allocated once, reused by every later call,
   * e.g. one call per tile of a frame; concurrent calls take different buffers) */
  OutBuf buf{nullptr, 0};
  const size_t bytes = (size_t)w * h * 16 + 16;
  hrt_status st = hguard([&] {
    DeviceGuard dg(s->device);
    buf = out_pool_take(s, bytes);
  });
  if (st != HRT_OK) return st;
  hrt_render_stats local;
  st = hrt_render_device(s, cam, p, x0, y0, w, h, (float*)buf.ptr, nullptr, stats ? stats : &local);
  if (st == HRT_OK) {
    st = hguard([&] {
      DeviceGuard dg(s->device);
      hip_check(hipMemcpy(rgba_out, buf.ptr, (size_t)w * h * 16, hipMemcpyDeviceToHost), "hipMemcpy(out)");
    });
  }
  out_pool_give(s, buf);
  return st;
}

/* Application::render with progressive tile delivery (application.rs:393-475, the Tile messages of
 * :45-52 / :461-472): the rank's share of the tile grid is rendered in launches of `batch` tiles on a
 * stream of its own; while batch k+1 renders, batch k (copied to pinned memory) is handed to `fn` tile
 * by tile in grid order.  With `stats` each batch's counters are read as it completes (the host then
 * waits for every launch before consuming the previous batch). */
hrt_status hrt_render_progressive(hrt_scene* s, const hrt_camera* cam, const hrt_render_params* p,
                                  uint32_t tile_size, uint32_t rank, uint32_t world, uint32_t batch,
                                  hrt_tile_fn fn, void* user, hrt_render_stats* stats) {
  if (!s || !cam || !p || !fn || tile_size == 0 || batch == 0 || world == 0 || rank >= world) {
    set_error("hrt_render_progressive: bad argument");
    return HRT_ERR_INVALID_ARG;
  }
  if (!s->committed) {
    set_error("scene not committed");
    return HRT_ERR_STATE;
  }
  uint32_t n = 0;
  hrt_status st = hrt_tile_grid(p->width, p->height, tile_size, rank, world, nullptr, 0, &n);
  if (st != HRT_OK) return st;
  std::vector<hrt_tile> tiles(n);
  st = hrt_tile_grid(p->width, p->height, tile_size, rank, world, tiles.data(), n, &n);
  if (st != HRT_OK) return st;
  if (stats) memset(stats, 0, sizeof(*stats));
  const size_t slot_floats = (size_t)batch * tile_size * tile_size * 4;
  float* d_buf[2] = {nullptr, nullptr};
  float* h_buf[2] = {nullptr, nullptr};
  hipStream_t stream = nullptr;
  hipEvent_t ev[2] = {nullptr, nullptr};
  st = hguard([&] {
    DeviceGuard dg(s->device);
    hip_check(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking), "hipStreamCreate");
    for (int k = 0; k < 2; k++) {
      hip_check(hipMalloc((void**)&d_buf[k], slot_floats * sizeof(float)), "hipMalloc(progressive)");
      hip_check(hipHostMalloc((void**)&h_buf[k], slot_floats * sizeof(float), hipHostMallocDefault),
                "hipHostMalloc(progressive)");
      hip_check(hipEventCreateWithFlags(&ev[k], hipEventDisableTiming), "hipEventCreate");
    }
    const uint32_t n_batches = (n + batch - 1) / batch;
    for (uint32_t b = 0; b <= n_batches; b++) {
      if (b < n_batches) { /* render batch b into slot b % 2, copy it back, mark it */
        const uint32_t first = b * batch, cnt = std::min(batch, n - first);
        hrt_render_stats bs;
        const hrt_status r = hrt_render_tiles_device(s, cam, p, tiles.data() + first, cnt, d_buf[b % 2], stream,
                                                     stats ? &bs : nullptr);
        if (r != HRT_OK) throw HipError{r, hrt_last_error()};
        size_t px = 0;
        for (uint32_t t = 0; t < cnt; t++) px += (size_t)tiles[first + t].w * tiles[first + t].h;
        hip_check(hipMemcpyAsync(h_buf[b % 2], d_buf[b % 2], px * 16, hipMemcpyDeviceToHost, stream),
                  "hipMemcpyAsync(progressive)");
        hip_check(hipEventRecord(ev[b % 2], stream), "hipEventRecord(progressive)");
        if (stats) {
          stats->segments += bs.segments;
          stats->samples += bs.samples;
          stats->pixels += bs.pixels;
          stats->node_visits += bs.node_visits;
          stats->prim_tests += bs.prim_tests;
          stats->tex_evals += bs.tex_evals;
        }
      }
      if (b >= 1) { /* hand batch b-1 over, tile by tile */
        const uint32_t k = b - 1, first = k * batch, cnt = std::min(batch, n - first);
        hip_check(hipEventSynchronize(ev[k % 2]), "hipEventSynchronize(progressive)");
        size_t off = 0;
        for (uint32_t t = 0; t < cnt; t++) {
          const hrt_tile& tl = tiles[first + t];
          hrt_tile_pixels tp{tl.x / tile_size, tl.y / tile_size, tl.w, tl.h, h_buf[k % 2] + off * 4};
          fn(&tp, user);
          off += (size_t)tl.w * tl.h;
        }
      }
    }
  });
  {
    int prev = -1;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(s->device);
    if (stream) (void)hipStreamSynchronize(stream);
    for (int k = 0; k < 2; k++) {
      if (ev[k]) (void)hipEventDestroy(ev[k]);
      if (d_buf[k]) (void)hipFree(d_buf[k]);
      if (h_buf[k]) (void)hipHostFree(h_buf[k]);
    }
    if (stream) (void)hipStreamDestroy(stream);
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
    check_render_args(cam, p);
    if (x >= p->width || y >= p->height) throw HipError{HRT_ERR_INVALID_ARG, "pixel outside the image"};
    DeviceGuard dg(s->device);
    const Plan pl = plan(s, cam, p->flags);
    KParams kp = scene_params(s, cam, p, pl);
    size_t bytes = (9 * (size_t)max_segments + 3) * sizeof(float);
    DevBuf<float> out_buf(bytes);
    DevBuf<uint32_t> n_buf(4);
    float* d_out = out_buf.p;
    uint32_t* d_n = n_buf.p;
    if (pl.fast) hipLaunchKernelGGL((debug_path_kernel<G::CULL_SLAB, false, true>), dim3(1), dim3(64), 0, 0, kp, x, y, sample, d_out, max_segments, d_n);
    else if ((pl.full || pl.heavy) && pl.cull == G::CULL_EXACT) hipLaunchKernelGGL((debug_path_kernel<G::CULL_EXACT, true, false>), dim3(1), dim3(64), 0, 0, kp, x, y, sample, d_out, max_segments, d_n);
    else if (pl.cull == G::CULL_EXACT) hipLaunchKernelGGL((debug_path_kernel<G::CULL_EXACT, false, false>), dim3(1), dim3(64), 0, 0, kp, x, y, sample, d_out, max_segments, d_n);
    else if (pl.full && pl.cull == G::CULL_SLAB) hipLaunchKernelGGL((debug_path_kernel<G::CULL_SLAB, true, false>), dim3(1), dim3(64), 0, 0, kp, x, y, sample, d_out, max_segments, d_n);
    else if (pl.full) hipLaunchKernelGGL((debug_path_kernel<G::CULL_REFERENCE, true, false>), dim3(1), dim3(64), 0, 0, kp, x, y, sample, d_out, max_segments, d_n);
    else if (pl.cull == G::CULL_SLAB) hipLaunchKernelGGL((debug_path_kernel<G::CULL_SLAB, false, false>), dim3(1), dim3(64), 0, 0, kp, x, y, sample, d_out, max_segments, d_n);
    else hipLaunchKernelGGL((debug_path_kernel<G::CULL_REFERENCE, false, false>), dim3(1), dim3(64), 0, 0, kp, x, y, sample, d_out, max_segments, d_n);
    hip_check(hipGetLastError(), "debug_path_kernel launch");
    hip_check(hipMemcpy(out, d_out, bytes, hipMemcpyDeviceToHost), "hipMemcpy");
    hip_check(hipMemcpy(n_segments, d_n, 4, hipMemcpyDeviceToHost), "hipMemcpy");
  });
}

hrt_status hrt_debug_box_test(int32_t form, int32_t on_device, const float* boxes, uint32_t n_boxes, const float* rays,
                              uint32_t n_rays, float tmin, float tmax, uint8_t* out) {
  return hguard([&] {
    if (!boxes || !rays || !out || form < 0 || form > 1 || (uint64_t)n_boxes * n_rays >= (1ull << 31))
      throw HipError{HRT_ERR_INVALID_ARG, "hrt_debug_box_test: bad argument"};
    const uint64_t n = (uint64_t)n_boxes * n_rays;
    if (n == 0) return;
    if (!on_device) {
      for (uint32_t b = 0; b < n_boxes; b++)
        for (uint32_t q = 0; q < n_rays; q++)
          out[(uint64_t)b * n_rays + q] = form ? box_pair<true>(boxes, rays, b, q, tmin, tmax)
                                               : box_pair<false>(boxes, rays, b, q, tmin, tmax);
      return;
    }
    /* on the calling thread's current device (hipSetDevice / torch.cuda.set_device), like hrt_debug_device_math */
    DevBuf<float> b_buf((size_t)n_boxes * 32), r_buf((size_t)n_rays * 24);
    DevBuf<uint8_t> o_buf(n);
    float *db = b_buf.p, *dr = r_buf.p;
    uint8_t* dout = o_buf.p;
    hip_check(hipMemcpy(db, boxes, (size_t)n_boxes * 32, hipMemcpyHostToDevice), "hipMemcpy");
    hip_check(hipMemcpy(dr, rays, (size_t)n_rays * 24, hipMemcpyHostToDevice), "hipMemcpy");
    hipLaunchKernelGGL(box_test_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, 0, form, db, n_boxes, dr, n_rays,
                       tmin, tmax, dout);
    hip_check(hipGetLastError(), "box_test_kernel launch");
    hip_check(hipMemcpy(out, dout, n, hipMemcpyDeviceToHost), "hipMemcpy");
  });
}

hrt_status hrt_debug_sample_chunks(hrt_scene* s, const hrt_render_params* p, uint32_t* out4) {
  return hguard([&] {
    if (!s || !p || !out4) throw HipError{HRT_ERR_INVALID_ARG, "hrt_debug_sample_chunks: null argument"};
    if (p->samples == 0) throw HipError{HRT_ERR_INVALID_ARG, "hrt_debug_sample_chunks: no samples"};
    /* the schedule needs the scene's class only (feature mask, main stream length): an uncommitted scene is
     * flattened without its walk streams (no view pass, no re-grouping) */
    if (!s->committed) flatten_scene_reference(s);
    chunk_schedule(s, p, out4[0], out4[1], out4[2], out4[3]);
  });
}

hrt_status hrt_last_launch(hrt_launch_info* out) {
  return hguard([&] {
    if (!out) throw HipError{HRT_ERR_INVALID_ARG, "hrt_last_launch: null pointer"};
    if (!t_has_launch) throw HipError{HRT_ERR_STATE, "hrt_last_launch: no launch on this thread yet"};
    *out = t_last_launch; /* knobs: the snapshot taken at that launch (launch_knobs) */
  });
}

hrt_status hrt_debug_device_math(int32_t op, const float* x, const float* y, float* out, uint32_t n) {
  return hguard([&] {
    if (!x || !out || op < 0 || op > 9) throw HipError{HRT_ERR_INVALID_ARG, "bad argument"};
    if (n == 0) return;
    DevBuf<float> x_buf((size_t)n * 4), o_buf((size_t)n * 4), y_buf(y ? (size_t)n * 4 : 4);
    float *dx = x_buf.p, *dy = y ? y_buf.p : nullptr, *dout = o_buf.p;
    hip_check(hipMemcpy(dx, x, n * 4, hipMemcpyHostToDevice), "hipMemcpy");
    if (y) hip_check(hipMemcpy(dy, y, n * 4, hipMemcpyHostToDevice), "hipMemcpy");
    hipLaunchKernelGGL(math_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, op, dx, dy, dout, n);
    hip_check(hipGetLastError(), "math_kernel launch");
    hip_check(hipMemcpy(out, dout, n * 4, hipMemcpyDeviceToHost), "hipMemcpy");
  });
}

}  // extern "C"
