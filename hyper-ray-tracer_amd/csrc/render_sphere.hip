/*
 * render_sphere.hip — the sphere-scene kernel (render_basic_kernel): scenes within F_BASIC (spheres,
 * moving spheres, Lambertian / Metal / Dielectric, solid and checker textures), among them the
 * BASELINE headline scene.  Persistent walks over the walk stream (layout.h) with postponed shading;
 * DESIGN.md section 6.1.  Built on its own translation unit (see kernel_common.h).
 */
#include "kernel_common.h"

using namespace hrt;
using namespace hrt::lane;
using namespace hrt::kern;

#ifndef HRT_SPEC
#define HRT_SPEC 1 /* speculative walk of the walk stream (0: lanes park on every passed leaf, for A/B) */
#endif

#ifndef HRT_KEEP_SKIP
#define HRT_KEEP_SKIP 1 /* a parked lane continues at the skip kept from its leaf's step (lane.h walk_box), not at the
                           successor read from the leaf's payload (0: the payload read, for A/B) */
#endif
#ifndef HRT_HEAVY_WAVES
#define HRT_HEAVY_WAVES 4 /* HEAVY: the out-of-line texture calls spill live registers at 80 VGPRs (6 waves) */
#endif

namespace {

template <bool HEAVY>
constexpr int sphere_waves() { return HEAVY ? HRT_HEAVY_WAVES : BASIC_WAVES; }

/* HYB (CULL_EXACT with LDS): the walk stream exceeds the LDS budget; its first P.walk_hot bytes (the
 * hierarchy's top levels) are staged, the rest is read through the buffer descriptor (layout.h) */
/* SPLIT: the stream's node parts are split (layout.h WALK_SPLIT_HALF; hybrid streams: WALK_SPLIT_HALF_HYB) */
/* C16: 16-B node parts (layout.h WALK_C16; hybrid streams): walk positions are node indices */
/* PACKET: a tiny stream staged whole in LDS (at most SPHERE_PACKET_NODES node parts: Earth + Perlin, the two-sphere
 * scenes) walked by the wave as one packet (render_general.hip PACKET): every lane's segment ends in one pass */
template <int CULL, bool COUNT, bool LDS, bool HYB = false, bool HEAVY = false, bool SPLIT = false, bool C16 = false,
          bool PACKET = false>
__global__ __launch_bounds__((basic_block_threads<LDS, sphere_waves<HEAVY>()>()), sphere_waves<HEAVY>())
void render_basic_kernel(KParams P) {
  extern __shared__ float4 lds_scene[];
  const G::Node* nodes = P.nodes;
  const G::Prim* prims = P.prims;
  /* CULL_EXACT walks the walk stream (layout.h; positions are byte offsets, in LDS or through a buffer
   * descriptor); the other modes walk the reference node stream (with the scene in LDS the walk
   * position is the node's LDS byte address, basic_box STRIDE) */
  constexpr bool WS = CULL == G::CULL_EXACT;
  constexpr bool SPEC = WS && HRT_SPEC;
  constexpr int WMEM = HYB ? WM_HYB : (LDS ? WM_LDS : WM_BUF);
  constexpr uint32_t STRIDE = LDS ? (uint32_t)sizeof(G::Node) : 1u;
  const uint32_t lds_base = (uint32_t)(size_t)(__attribute__((address_space(3))) float4*)lds_scene;
  const uint32_t root = WS || !LDS ? 0u : lds_base;
  WalkSrc ws;
  ws.base = P.walk;
  ws.hot = P.walk_hot;
#if defined(__HIP_DEVICE_COMPILE__)
  ws.rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)P.walk, 0, (int)P.walk_bytes, 0x00020000);
#endif
  /* Q: the scene as shading reads it; HEAVY with perlin_lds: the Perlin tables (turbulence gathers 7 x 8
   * permutation and gradient entries per noise texture call) staged in LDS behind the walk stream */
  KParams Q = P;
  if constexpr (WS && LDS) { /* the stream at LDS address 0: its offsets are LDS addresses */
    const float4* g = reinterpret_cast<const float4*>(P.walk);
    const uint32_t staged = HYB ? P.walk_hot : P.walk_bytes;
    for (uint32_t k = threadIdx.x; k < staged / 16u; k += blockDim.x) lds_scene[k] = g[k];
    if constexpr (HEAVY) {
      if (P.perlin_lds) /* at the next 4-KB boundary (render.hip plan sizes the LDS so) */
        Q.perlin = stage_perlin(lds_align(lds_scene + staged / 16u, G::PERLIN_LDS_ALIGN), P.perlin, P.n_perlin);
    }
    __syncthreads();
    if (lds_base != 0u) { /* no static LDS in this kernel, so this cannot happen: report, do nothing */
      if (threadIdx.x == 0) atomicOr(&P.stats[12], 2ull);
      return;
    }
  } else if constexpr (LDS) {
    stage_scene<true>(P, lds_scene, nodes, prims, root);
  }
  /* the lane's Item.slot lives in LDS: a register kept across the whole item would be spilled at the
   * 80-VGPR cap (scratch written at every claim and chunk end) */
  uint32_t* const slot_lds = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(lds_scene) + P.lane_lds) + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63u;
  const float scale = 1.0f / (float)P.spp; /* application.rs:403 */
  const float inf = __uint_as_float(0x7f800000u);
  const uint32_t end = WS ? P.walk_end : root + P.main_end * STRIDE;
  /* t_min canonicalised once: box_ce's fmaxf against it then needs no per-step quieting */
  const float tmin_c = __builtin_canonicalizef(P.t_min);
  const uint32_t need = P.postpone;
  const uint32_t batch = P.prim_batch;
  /* watchdog: a lane's walk is at most walk_cap steps; waiting for a batch can stretch a pass to the
   * lanes' total work (each iteration steps or tests for at least one lane) */
  const uint32_t cap = P.walk_cap * 128u;

  bool has_item = false, exhausted = false;
  bool walking = false; /* a segment is in flight (walk running, or finished and waiting to shade) */
  bool setup = false;   /* the lane's next segment needs its ray set up (a new sample, or a scattered ray) */
  Item it{0u, 0u, 0u, 0u};
  WaveBlock wb{0u, 0u};
  Vec3 sum = v3(0.0f, 0.0f, 0.0f);
  PathState ps;
  init_path_state(ps);
  TRay r;
  set_ray(r, ps.ro, ps.rd, 0.0f, P);
  uint32_t node = G::NONE, winner = G::NONE; /* node: walk position (basic_box: index | WALK_PEND, or NONE) */
  /* every stream: in a hybrid one the payload read is a dependent global read (C4's 1/8 share +2.7%); from LDS it
   * is a dependent LDS read, and the register is worth more than the 16 B of scratch it adds (C2 +1.8%, C3 +0.7%,
   * profiles/r05_keep_skip_ab.txt) */
  constexpr bool KEEP_SKIP = HRT_KEEP_SKIP != 0;
  uint32_t nskip = G::NONE; /* KEEP_SKIP: the skip link of the lane's last node step */
  /* SPEC: a passed leaf whose test waits for the wave's next primitive block while the lane walks on
   * (speculative traversal: the walk runs ahead with a closest that the pending test may still shrink,
   * so it visits a superset of the nodes; the leaf tests, each with the reference box test against the
   * current closest, keep their order and outcomes: DESIGN.md section 4) */
  uint32_t pend = G::NONE;
  float closest = inf;
  uint32_t n_seg = 0, n_samples = 0, n_pixels = 0; /* wave totals (uniform) */
  Counts cn{0u, 0u, 0u, 0u, 0u, 0u};
  PhaseClock pc{{0ull, 0ull, 0ull}, 0ull, 0ull};
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
    const bool had_item = has_item;
    claim_work(P, lane, has_item, exhausted, it, wb);
    if (has_item && !had_item) *slot_lds = it.slot;
    if (!__any(has_item || !exhausted)) break;
    if (has_item && !walking) {
      start_sample(P, ps, it.pxy & 0xFFFFu, it.pxy >> 16, it.sample);
      walking = true;
      setup = true;
    }
    if (setup) { /* new samples and scattered rays share one pass through the ray setup (1/d, d.d) */
#if HRT_RAY_REDERIVE_SPHERE
      r.o = ps.ro;
      r.d = ps.rd;
      set_time(r, ps.rtime, P); /* a scattered ray keeps the sample's shutter time */
#else
      set_ray(r, ps.ro, ps.rd, ps.rtime, P);
#endif
      closest = inf;
      winner = G::NONE;
      node = ps.depth_left == 0 ? G::NONE : root; /* max_depth 0: black without a world.hit (:478-480) */
      setup = false;
    }
#if HRT_RAY_REDERIVE_SPHERE
    set_dir(r, r.o, r.d); /* every lane: dead across shading (kernel_common.h) */
#endif
    /* step the walks until enough lanes have finished (lanes not walking hold node >= end).  A lane
     * whose leaf box passed holds WALK_PEND in `node` and waits; the wave runs the sphere block
     * once `batch` lanes wait (or no lane can step), instead of for every lane that needs it. */
    if constexpr (COUNT) cn.shade_slots++;
    stamp(0);
    const unsigned long long walkers = __ballot(walking);
    uint32_t iters = 0;
    bool stuck = false;
    if constexpr (PACKET) {
      /* the packet walk (render_general.hip PACKET): the wave at ONE position u, the lanes whose own position is u
       * active; a leaf's test runs at once for the lanes that pass its box, so each lane tests exactly its own
       * walk's leaves, in order, with its own closest, and every lane's walk ends in this pass */
      if (__ballot(node < end)) {
        uint32_t u = 0u;
        while (u < end) {
          if constexpr (COUNT) cn.walk_slots++;
          const float4 a = wload<WM_LDS>(ws, u), b = wload<WM_LDS>(ws, u + 16u);
          const uint32_t skip = (uint32_t)__builtin_amdgcn_readfirstlane((int)f2u(a.w));
          const uint32_t pass = (uint32_t)__builtin_amdgcn_readfirstlane((int)f2u(b.w));
          const bool act = node == u;
          bool p = false;
          if (act) {
            if constexpr (COUNT) {
              cn.nodes++;
              cn.steps++;
            }
            p = box_ce<HRT_BOX_FMA && !HEAVY, false>(a, b, r, tmin_c, closest);
          }
          uint32_t nu;
          if (walk_pend<false>(pass)) { /* a leaf (uniform) */
            if (p) walk_leaf_test<COUNT, WMEM>(P, ws, pass - WALK_PEND, r, closest, winner, cn);
            if (act) node = skip;
            nu = skip;
          } else {
            if (act) node = p ? pass : skip;
            nu = __ballot(p) ? pass : skip;
          }
          if (nu <= u) { /* links point forward in a stream staged whole: a corrupt one is reported */
            stuck = true;
            break;
          }
          u = nu;
        }
      }
    } else {
    for (;;) {
#pragma unroll
      for (int u = 0; u < WALK_UNROLL; u++) {
        if constexpr (COUNT) cn.walk_slots++;
        if (node < end) {
          if constexpr (COUNT) cn.steps++;
          if constexpr (WS) walk_box<COUNT, WMEM, HRT_BOX_FMA && ((WMEM != WM_HYB && !HEAVY) || HRT_BOX_FMA_ALL), false,
                                    SPLIT ? (HYB ? G::WALK_SPLIT_HALF_HYB : G::WALK_SPLIT_HALF) : 16u, C16>(ws, node, r, tmin_c, closest, cn,
                                                                             KEEP_SKIP && SPEC ? &nskip : nullptr); /* no rects: no NaN hits (lane.h set_noinv) */
          else basic_box<CULL, COUNT, STRIDE>(P, nodes, node, r, closest, cn);
        } else if constexpr (COUNT) {
          if (walk_pend<C16>(node)) cn.park_slots++;
          else if (walking) cn.wait_slots++;
        }
        if ((u + 1) % PRIM_EVERY != 0) continue;
        if constexpr (SPEC) {
          /* a lane parked on a leaf with no test pending makes the leaf's test pending and walks on behind
           * it; a lane parks for good (blocked) only on a second leaf, or at the end of its walk */
          if (walk_pend<C16>(node) && pend == G::NONE) {
            pend = pend_payload<C16>(P, node);
            node = KEEP_SKIP ? nskip : walk_successor<WMEM>(ws, pend);
          }
          const bool waiting = pend != G::NONE && !(node < end);
          const unsigned long long pm = __ballot(waiting);
          if (pm && ((uint32_t)__popcll(pm) >= batch || !__ballot(node < end))) {
            const unsigned long long t_leaf = COUNT ? __builtin_amdgcn_s_memtime() : 0ull;
            if constexpr (COUNT) cn.prim_slots++;
            if (pend != G::NONE) { /* the pending tests of every lane, walking or blocked, in walk order */
              walk_leaf_test<COUNT, WMEM>(P, ws, pend, r, closest, winner, cn);
              pend = G::NONE;
              if (walk_pend<C16>(node)) { /* blocked: its leaf's test becomes the pending one */
                pend = pend_payload<C16>(P, node);
                node = KEEP_SKIP ? nskip : walk_successor<WMEM>(ws, pend);
              }
            }
            if constexpr (COUNT) pc.leaf += __builtin_amdgcn_s_memtime() - t_leaf;
          }
          continue;
        }
        const bool waiting = walk_pend<C16>(node);
        const unsigned long long pm = __ballot(waiting);
        if (pm && ((uint32_t)__popcll(pm) >= batch || !__ballot(node < end))) {
          if constexpr (COUNT) cn.prim_slots++;
          if (waiting) {
            if constexpr (WS) walk_prim<COUNT, WMEM, C16>(P, ws, node, r, closest, winner, cn);
            else basic_prim<CULL, COUNT, STRIDE>(P, nodes, prims, node, r, closest, winner, cn);
          }
        }
      }
      const unsigned long long live = __ballot(node < end || walk_pend<C16>(node) || (SPEC && pend != G::NONE));
      if (!live || (uint32_t)__popcll(walkers & ~live) >= need) break;
      if (++iters > cap) { stuck = true; break; }
    }
    }
    if (stuck) { /* a walk that cannot end (corrupt scene data): report it, retire the wave */
      if (lane == 0) atomicOr(&P.stats[12], 1ull);
      exhausted = true;
      has_item = false;
      walking = false;
      node = G::NONE;
      pend = G::NONE;
    }
    stamp(1);
    /* shade the finished segments (application.rs:483-494) */
    const bool shading = walking && node >= end && !walk_pend<C16>(node) && (!SPEC || pend == G::NONE);
    const bool traced = shading && node != G::NONE;
    bool sample_done = false, chunk_done = false;
    if (shading) {
      bool done = true;
      if (traced) {
        if constexpr (WS) done = shade_walk<COUNT, WMEM, HEAVY>(Q, ws, ps, winner, closest, r.o, r.d, r.tau, r.tau, sum, cn);
        else done = shade<false, COUNT>(P, ps, winner, closest, r.o, r.d, r.tau, r.tau, cn); /* time = r.tau unless uniform (TRay) */
        done = done || ps.depth_left == 0;
      }
      if (done) {
        /* application.rs:448: samples of a chunk summed in order */
        walking = false;
        node = G::NONE;
        if constexpr (!WS) sum = sum + ps.rad; /* shade_walk added a miss's radiance already */
        sample_done = true;
        if (++it.sample == it.sample_end) {
          if (P.n_chunks == 1) /* sqrt(sum / spp), alpha 1 (:451-456) */
            P.out[*slot_lds] = make_float4(sqrtf(sum.x * scale), sqrtf(sum.y * scale), sqrtf(sum.z * scale), 1.0f);
          else
            P.partial[*slot_lds] = make_float4(sum.x, sum.y, sum.z, 0.0f);
          chunk_done = true;
          has_item = false;
          sum = v3(0.0f, 0.0f, 0.0f);
        }
      } else {
        setup = true; /* the scattered ray (depth_left > 0) is set up with the next pass's new samples */
        node = G::NONE;
      }
    }
    n_seg += (uint32_t)__popcll(__ballot(traced));
    n_samples += (uint32_t)__popcll(__ballot(sample_done));
    n_pixels += (uint32_t)__popcll(__ballot(chunk_done && it.sample_end <= P.chunk));
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
    if (lane == 0) atomicAdd(&P.stats[15], pc.leaf);
  }
}


template <int CULL, bool COUNT, bool LDS, bool HYB = false, bool HEAVY = false, bool SPLIT = false, bool C16 = false,
          bool PACKET = false>
void launch_basic(const KParams& kp, int device, hipStream_t stream, size_t smem) {
  const void* fn = (const void*)render_basic_kernel<CULL, COUNT, LDS, HYB, HEAVY, SPLIT, C16, PACKET>;
  const int block = basic_block_threads<LDS, sphere_waves<HEAVY>()>();
  /* LDS: the staged scene, then one u32 result slot per thread (layout.h LDS_SCENE_MAX_BYTES leaves
   * room for both, twice per CU) */
  KParams p = kp;
  p.lane_lds = LDS ? (uint32_t)((smem + 15) & ~(size_t)15) : 0u;
  const size_t total = p.lane_lds + (size_t)block * sizeof(uint32_t);
  const int grid = resident_grid(fn, block, device, total, true, __PRETTY_FUNCTION__);
  hipLaunchKernelGGL((render_basic_kernel<CULL, COUNT, LDS, HYB, HEAVY, SPLIT, C16, PACKET>), dim3(grid), dim3(block), total, stream, p);
  hip_check(hipGetLastError(), "render_basic_kernel launch");
}


}  // namespace

namespace hrt {

void launch_sphere(int cull, bool count, bool lds, bool heavy, bool packet, const KParams& kp, int device, hipStream_t stream,
                   size_t smem) {
  if (packet && lds && cull == G::CULL_EXACT && kp.walk_hot == 0 && kp.walk_half == 16u && !kp.walk_c16) {
    if (heavy) count ? launch_basic<G::CULL_EXACT, true, true, false, true, false, false, true>(kp, device, stream, smem)
                     : launch_basic<G::CULL_EXACT, false, true, false, true, false, false, true>(kp, device, stream, smem);
    else count ? launch_basic<G::CULL_EXACT, true, true, false, false, false, false, true>(kp, device, stream, smem)
               : launch_basic<G::CULL_EXACT, false, true, false, false, false, false, true>(kp, device, stream, smem);
    return;
  }
  if (heavy) { /* noise / image textures (exact culling only: plan()) */
    if (lds && kp.walk_hot > 0) { /* a stream beyond the LDS budget: its staged part in LDS, the rest global */
      count ? launch_basic<G::CULL_EXACT, true, true, true, true>(kp, device, stream, smem)
            : launch_basic<G::CULL_EXACT, false, true, true, true>(kp, device, stream, smem);
      return;
    }
    if (count) lds ? launch_basic<G::CULL_EXACT, true, true, false, true>(kp, device, stream, smem)
                   : launch_basic<G::CULL_EXACT, true, false, false, true>(kp, device, stream, 0);
    else lds ? launch_basic<G::CULL_EXACT, false, true, false, true>(kp, device, stream, smem)
             : launch_basic<G::CULL_EXACT, false, false, false, true>(kp, device, stream, 0);
    return;
  }
  if (cull == G::CULL_EXACT && kp.walk_c16) { /* 16-B node parts (layout.h WALK_C16: hybrid streams only) */
    if (lds) count ? launch_basic<G::CULL_EXACT, true, true, true, false, false, true>(kp, device, stream, smem)
                   : launch_basic<G::CULL_EXACT, false, true, true, false, false, true>(kp, device, stream, smem);
    else count ? launch_basic<G::CULL_EXACT, true, false, false, false, false, true>(kp, device, stream, 0)
               : launch_basic<G::CULL_EXACT, false, false, false, false, false, true>(kp, device, stream, 0);
  } else if (cull == G::CULL_EXACT && lds && kp.walk_hot > 0) { /* top levels in LDS, the rest in global memory */
    if (kp.walk_half != 16u) { /* split node parts (layout.h WALK_SPLIT_HALF_HYB, opt-in) */
      if (count) launch_basic<G::CULL_EXACT, true, true, true, false, true>(kp, device, stream, smem);
      else launch_basic<G::CULL_EXACT, false, true, true, false, true>(kp, device, stream, smem);
    } else if (count) launch_basic<G::CULL_EXACT, true, true, true>(kp, device, stream, smem);
    else launch_basic<G::CULL_EXACT, false, true, true>(kp, device, stream, smem);
  } else if (cull == G::CULL_EXACT && kp.walk_half != 16u) { /* split node parts (layout.h; F_BASIC scenes) */
    if (count) lds ? launch_basic<G::CULL_EXACT, true, true, false, false, true>(kp, device, stream, smem)
                   : launch_basic<G::CULL_EXACT, true, false, false, false, true>(kp, device, stream, 0);
    else lds ? launch_basic<G::CULL_EXACT, false, true, false, false, true>(kp, device, stream, smem)
             : launch_basic<G::CULL_EXACT, false, false, false, false, true>(kp, device, stream, 0);
  } else if (cull == G::CULL_EXACT) {
    if (count) lds ? launch_basic<G::CULL_EXACT, true, true>(kp, device, stream, smem)
                   : launch_basic<G::CULL_EXACT, true, false>(kp, device, stream, 0);
    else lds ? launch_basic<G::CULL_EXACT, false, true>(kp, device, stream, smem)
             : launch_basic<G::CULL_EXACT, false, false>(kp, device, stream, 0);
  } else if (cull == G::CULL_SLAB) {
    if (count) lds ? launch_basic<G::CULL_SLAB, true, true>(kp, device, stream, smem)
                   : launch_basic<G::CULL_SLAB, true, false>(kp, device, stream, 0);
    else lds ? launch_basic<G::CULL_SLAB, false, true>(kp, device, stream, smem)
             : launch_basic<G::CULL_SLAB, false, false>(kp, device, stream, 0);
  } else {
    if (count) lds ? launch_basic<G::CULL_REFERENCE, true, true>(kp, device, stream, smem)
                   : launch_basic<G::CULL_REFERENCE, true, false>(kp, device, stream, 0);
    else lds ? launch_basic<G::CULL_REFERENCE, false, true>(kp, device, stream, smem)
             : launch_basic<G::CULL_REFERENCE, false, false>(kp, device, stream, 0);
  }
}

}  // namespace hrt
