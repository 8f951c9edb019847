/*
 * render_general.hip — the general-scene kernel with persistent walks (render_gwalk_kernel): rects,
 * instances, media, lights and every texture (Cornell, Cornell-smoke, Final, Earth+Perlin, ...).
 *
 * It is render_basic_kernel's schedule (render_sphere.hip) over the GENERAL walk
 * stream (layout.h): the wave steps its lanes' walks one node at a time over a re-grouped hierarchy of the
 * reference's leaf objects, leaves a passed leaf's test pending while the lane walks on (speculative walk),
 * runs the pending tests of many lanes in one batched block, and shades once enough lanes have finished.
 * A leaf's test is its PROGRAM: the leaf's range of the reference node stream (its BvhNode box, instance
 * brackets, a Cuboid's or a List's primitives, a ConstantMedium's boundary walks) run by lane.h trace_ray
 * from the world ray against the lane's closest, so every state that instances and media need lives inside
 * that block and the walk loop keeps the sphere kernel's registers.  Shading is the segment kernels'
 * shade<true> (hit record through the instance chain, emission, scatter, textures).
 *
 * Each lane runs exactly the reference's sequence of world.hit calls and RNG draws (a lane's tests are in
 * the reference's leaf order with its closest; tests/test_lane_sim.py holds the lane to the oracle and to
 * render_full_kernel's lane bit for bit), so the image is the segment kernel's.
 */
#include "kernel_common.h"

using namespace hrt;
using namespace hrt::lane;
using namespace hrt::kern;

#ifndef HRT_GWALK_WAVES
#define HRT_GWALK_WAVES 4
#endif

namespace {

constexpr int GWALK_WAVES = HRT_GWALK_WAVES;
#ifndef HRT_GWALK_KEEP_SKIP
#define HRT_GWALK_KEEP_SKIP 1 /* a parked lane continues at the skip kept from its leaf's step (lane.h walk_box)
                                 instead of the successor read from the payload (hybrid streams: a global read,
                                 Final +2.9%; in LDS: C5's share +1.8%, profiles/r05_keep_skip_ab.txt) */
#endif
#ifndef HRT_GWALK_RECOMPUTE
#define HRT_GWALK_RECOMPUTE 1 /* kernel_common.h claim_work<RECOMPUTE> */
#endif

/* WMEM: where the walk stream is read (WM_LDS: staged whole; WM_HYB: its top levels staged, the rest
 * through the buffer descriptor; WM_BUF: global memory).  LREF: the reference node stream and the
 * primitives that leaf programs read are staged in LDS behind the walk stream. */
/* BIG: one 1024-thread workgroup per CU (a hybrid stream's staged part beyond LDS_SCENE_MAX_BYTES).
 * ONE: every chunk of the schedule is one sample (deep general scenes up to 64 spp, lane.h sample_chunk):
 * a lane's work item is dead once its sample has started and its partial sum is that sample's radiance, so
 * neither the item nor the chunk's running sum lives across the walk and shading (Final: 48 -> 32 B of
 * scratch per lane; the spills that were left were per-segment writes, 3.9 GB per launch). */
/* PACKET: the wave walks a small stream staged whole in LDS, whose leaves run generic programs (Cornell-smoke's
 * media in rotated boxes), as one packet: see below */
template <bool COUNT, int WMEM, bool LREF, int TRIM, bool BIG, bool ONE, bool PACKET>
__global__ __launch_bounds__((BIG ? 256 : 128) * GWALK_WAVES, GWALK_WAVES)
void render_gwalk_kernel(KParams P) {
  extern __shared__ float4 lds_scene[];
  constexpr bool MEDIA = !(TRIM & TRIM_MEDIA);
  constexpr bool PROG = !(TRIM & TRIM_PROGRAMS);
  const G::Node* nodes = P.nodes;
  const G::Prim* prims = P.prims;
  const uint32_t lds_base = (uint32_t)(size_t)(__attribute__((address_space(3))) float4*)lds_scene;
  WalkSrc ws;
  ws.base = P.walk;
  ws.hot = P.walk_hot;
#if defined(__HIP_DEVICE_COMPILE__)
  ws.rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)P.walk, 0, (int)P.walk_bytes, 0x00020000);
#endif
  uint32_t staged = 0; /* bytes of the walk stream in LDS, at LDS address 0 */
  if constexpr (WMEM == WM_LDS || WMEM == WM_HYB) {
    staged = WMEM == WM_HYB ? P.walk_hot : P.walk_bytes;
    const float4* g = reinterpret_cast<const float4*>(P.walk);
    for (uint32_t k = threadIdx.x; k < staged / 16u; k += blockDim.x) lds_scene[k] = g[k];
  }
  /* Q: the parameters leaf programs and shading read the scene through.  LREF: every record they read
   * but the Perlin tables and images (reference stream, primitives, instances, media, materials,
   * textures) staged in LDS behind the walk stream (all 16-B records), so a leaf's instance chain and a
   * hit record's node -> primitive -> instance -> material -> texture reads are LDS reads instead of
   * dependent global loads */
  KParams Q = P;
  if constexpr (LREF) {
    float4* dst = lds_scene + staged / 16u;
    auto stage = [&](const void* src, uint32_t records, uint32_t bytes) {
      float4* at = dst;
      const float4* g = reinterpret_cast<const float4*>(src);
      const uint32_t n4 = records * (bytes / 16u);
      for (uint32_t k = threadIdx.x; k < n4; k += blockDim.x) at[k] = g[k];
      dst += n4;
      return (const void*)at;
    };
    Q.nodes = static_cast<const G::Node*>(stage(P.nodes, P.n_nodes, sizeof(G::Node)));
    Q.prims = static_cast<const G::Prim*>(stage(P.prims, P.n_prims, sizeof(G::Prim)));
    Q.insts = static_cast<const G::Inst*>(stage(P.insts, P.n_insts, sizeof(G::Inst)));
    Q.media = static_cast<const G::Medium*>(stage(P.media, P.n_media, sizeof(G::Medium)));
    Q.mats = static_cast<const G::Mat*>(stage(P.mats, P.n_mats, sizeof(G::Mat)));
    Q.texs = static_cast<const G::Tex*>(stage(P.texs, P.n_texs, sizeof(G::Tex)));
    Q.chains = static_cast<const float4*>(stage(P.chains, P.n_insts, G::CHAIN_F4 * 16u));
    if (P.perlin_lds) Q.perlin = stage_perlin(lds_align(dst, G::PERLIN_LDS_ALIGN), P.perlin, P.n_perlin); /* render.hip plan */
    nodes = Q.nodes;
    prims = Q.prims;
  }
  __syncthreads();
  if ((WMEM == WM_LDS || WMEM == WM_HYB) && lds_base != 0u) { /* stream offsets are LDS addresses */
    if (threadIdx.x == 0) atomicOr(&P.stats[12], 2ull);
    return;
  }
  uint32_t* const slot_lds = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(lds_scene) + P.lane_lds) + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63u;
  const float scale = 1.0f / (float)P.spp; /* application.rs:403 */
  const float inf = __uint_as_float(0x7f800000u);
  const uint32_t end = P.walk_end;
  const float tmin_c = __builtin_canonicalizef(P.t_min);
  const uint32_t need = P.postpone;
  const uint32_t batch = P.prim_batch;
  const uint32_t cap = P.walk_cap * 128u;

  bool has_item = false, exhausted = false;
  bool walking = false, setup = false;
  Item it{0u, 0u, 0u, 0u};
  WaveBlock wb{0u, 0u};
  Vec3 sum = v3(0.0f, 0.0f, 0.0f);
  PathState ps;
  init_path_state(ps);
  TRay r;
  set_ray(r, ps.ro, ps.rd, 0.0f, P);
  uint32_t node = G::NONE, winner = G::NONE, pend = G::NONE;
  constexpr bool KEEP_SKIP = HRT_GWALK_KEEP_SKIP != 0;
  uint32_t nskip = G::NONE; /* KEEP_SKIP: the skip link of the lane's last node step */
  uint32_t gstate = G::NONE; /* the last leaf group whose box this walk tested, and its outcome (bit 31) */
  float closest = inf;
  uint32_t n_seg = 0, n_samples = 0, n_pixels = 0;
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
    const bool had_item = has_item;
    claim_work<HRT_GWALK_RECOMPUTE != 0>(P, lane, has_item, exhausted, it, wb);
    if (has_item && !had_item) *slot_lds = it.slot;
    if (!__any(has_item || !exhausted)) break;
    if (has_item && !walking) {
      start_sample(P, ps, it.pxy & 0xFFFFu, it.pxy >> 16, it.sample);
      walking = true;
      setup = true;
      if constexpr (ONE) n_pixels += it.sample == 0u ? 1u : 0u; /* lane-local: a pixel's first chunk */
    }
    if constexpr (ONE) it = Item{0u, 0u, 0u, 0u}; /* every started item: nothing of it is read again */
    if (setup) {
#if HRT_RAY_REDERIVE
      r.o = ps.ro;
      r.d = ps.rd;
      set_time(r, ps.rtime, P);
#else
      set_ray(r, ps.ro, ps.rd, ps.rtime, P);
#endif
      closest = inf;
      winner = G::NONE;
      gstate = G::NONE & 0x7FFFFFFFu;
      node = ps.depth_left == 0 ? G::NONE : 0u; /* max_depth 0: black without a world.hit (:478-480) */
      setup = false;
    }
#if HRT_RAY_REDERIVE
    set_dir(r, r.o, r.d); /* every lane: dead across shading (kernel_common.h) */
#endif
    if constexpr (COUNT) cn.shade_slots++;
    stamp(0);
    const unsigned long long walkers = __ballot(walking);
    uint32_t iters = 0;
    bool stuck = false;
    if constexpr (PACKET) {
      /* The packet walk (small streams staged whole in LDS with generic leaf programs).  The wave keeps ONE walk
       * position u (wave-uniform) and every lane its own: a lane is active at u when its position is u.  At an
       * inner node the active lanes run the inflated test and move to `pass` or `skip`; the wave goes to `pass`
       * if any lane passed, else to `skip`.  At a leaf the passing lanes run the leaf's program at once, all of
       * them together (one leaf, one kind: the program's code is uniform), and every active lane moves to the
       * leaf's skip.  In pre-order a lane's own position is always u or beyond u's subtree, so every lane
       * visits exactly the nodes of its own stackless walk, in the same order and with the same closest (the
       * non-speculative walk: each leaf tested as it is reached), and all lanes end their segment together:
       * no parked lanes, no postponed shading, one uniform node read (an LDS broadcast) per step.  The price: the
       * wave visits the union of its lanes' nodes.  Measured (profiles/r06_packet_ab.txt): Cornell-smoke +14%
       * (its leaf programs, two media in rotated boxes, run once for all the lanes that need them instead of
       * parking lanes in batches); Cornell -42% and simple-light -11% (one-node programs: the per-lane walk's
       * batches cost less than visiting the union), so those keep the per-lane walk. */
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
            p = box_ce<HRT_BOX_FMA != 0, true>(a, b, r, tmin_c, closest);
          }
          uint32_t nu;
          if (walk_pending(pass)) { /* a leaf (uniform): its program for the lanes that passed, now */
            if (p) gwalk_leaf_test<MEDIA, COUNT, WMEM, PROG>(Q, nodes, prims, ws, pass - WALK_PEND, r, closest, winner, gstate,
                                                             ps.pk, cn);
            if (act) node = skip;
            nu = skip;
          } else {
            if (act) node = p ? pass : skip;
            nu = __ballot(p) ? pass : skip;
          }
          if (nu <= u) { /* links point forward in a valid stream: a corrupt one is reported, not walked */
            stuck = true;
            break;
          }
          u = nu;
        }
      }
    } else {
    for (;;) {
      /* the node steps unrolled on their own, the leaf block after every PRIM_EVERY of them: unrolling
       * the block with them made the loop too large for the unroller */
      for (int v = 0; v < WALK_UNROLL / PRIM_EVERY; v++) {
#pragma unroll
        for (int u = 0; u < PRIM_EVERY; u++) {
          if constexpr (COUNT) cn.walk_slots++;
          if (node < end) {
            walk_box<COUNT, WMEM>(ws, node, r, tmin_c, closest, cn, KEEP_SKIP ? &nskip : nullptr);
            if constexpr (COUNT) cn.steps++;
          } else if constexpr (COUNT) {
            if (walk_pending(node)) cn.park_slots++;
            else if (walking) cn.wait_slots++;
          }
        }
        /* speculative walk (render_sphere.hip): a passed leaf's program waits in `pend` while the lane
         * walks on; the wave runs the pending programs once `batch` lanes are blocked or none can step */
        if (walk_pending(node) && pend == G::NONE) {
          pend = node - WALK_PEND;
          node = KEEP_SKIP ? nskip : walk_successor<WMEM>(ws, pend);
        }
        const bool waiting = pend != G::NONE && !(node < end);
        const unsigned long long pm = __ballot(waiting);
        if (pm && ((uint32_t)__popcll(pm) >= batch || !__ballot(node < end))) {
          const unsigned long long t_leaf = COUNT ? __builtin_amdgcn_s_memtime() : 0ull;
          if constexpr (COUNT) cn.prim_slots++;
          if (pend != G::NONE) {
            const float before = closest;
            gwalk_leaf_test<MEDIA, COUNT, WMEM, PROG>(Q, nodes, prims, ws, pend, r, closest, winner, gstate, ps.pk, cn);
            if (closest != closest && before == before) {
              /* the leaf accepted a NaN t (rect.rs 0 / 0, lane.h set_noinv; in an instance's frame the world
               * ray need not be in NaN mode): the reference now passes every box and accepts the next hit at
               * any t, but the walk ran ahead culling with the old closest -- walk again from the leaf's
               * successor (a leaf this lane was blocked on is reached again) */
              node = walk_successor<WMEM>(ws, pend);
              pend = G::NONE;
            }
            pend = G::NONE;
            if (walk_pending(node)) {
              pend = node - WALK_PEND;
              node = KEEP_SKIP ? nskip : walk_successor<WMEM>(ws, pend);
            }
          }
          if constexpr (COUNT) pc.leaf += __builtin_amdgcn_s_memtime() - t_leaf;
        }
      }
      const unsigned long long live = __ballot(node < end || walk_pending(node) || pend != G::NONE);
      if (!live || (uint32_t)__popcll(walkers & ~live) >= need) break;
      if (++iters > cap) { stuck = true; break; }
    }
    }
    if (stuck) {
      if (lane == 0) atomicOr(&P.stats[12], 1ull);
      exhausted = true;
      has_item = false;
      walking = false;
      node = G::NONE;
      pend = G::NONE;
    }
    stamp(1);
    /* shade the finished segments (application.rs:483-494) */
    const bool shading = walking && node >= end && !walk_pending(node) && pend == G::NONE;
    const bool traced = shading && node != G::NONE;
    bool sample_done = false, chunk_done = false;
    if (shading) {
      bool done = true;
      if (traced) {
        ps.pk.segment++;
        /* without media nothing but the motion factor reads the ray's time: r.tau holds it (lane.h TRay),
         * so r.time is dead in the media-free instantiations (one register fewer) */
        done = shade<true, COUNT, TRIM>(Q, ps, winner, closest, r.o, r.d, MEDIA ? r.time : r.tau, r.tau, cn) ||
               ps.depth_left == 0;
      }
      if (done && ONE) {
        walking = false;
        node = G::NONE;
        sample_done = true;
        const Vec3 c = v3(0.0f, 0.0f, 0.0f) + ps.rad; /* the chunk's sum, as the general case forms it */
        if (P.n_chunks == 1)
          P.out[*slot_lds] = make_float4(sqrtf(c.x * scale), sqrtf(c.y * scale), sqrtf(c.z * scale), 1.0f);
        else
          P.partial[*slot_lds] = make_float4(c.x, c.y, c.z, 0.0f);
        chunk_done = true;
        has_item = false;
      } else if (done) {
        walking = false;
        node = G::NONE;
        sum = sum + ps.rad; /* application.rs:448: samples of a chunk summed in order */
        sample_done = true;
        if (++it.sample == it.sample_end) {
          if (P.n_chunks == 1)
            P.out[*slot_lds] = make_float4(sqrtf(sum.x * scale), sqrtf(sum.y * scale), sqrtf(sum.z * scale), 1.0f);
          else
            P.partial[*slot_lds] = make_float4(sum.x, sum.y, sum.z, 0.0f);
          chunk_done = true;
          has_item = false;
          sum = v3(0.0f, 0.0f, 0.0f);
        }
      } else {
        setup = true; /* the scattered ray keeps the sample's shutter time */
        node = G::NONE;
      }
    }
    n_seg += (uint32_t)__popcll(__ballot(traced));
    n_samples += (uint32_t)__popcll(__ballot(sample_done));
    if constexpr (!ONE) n_pixels += (uint32_t)__popcll(__ballot(chunk_done && it.sample_end <= P.chunk));
    stamp(2);
  }
  if constexpr (ONE) { /* n_pixels counted per lane: the wave's sum */
    for (int o = 32; o >= 1; o >>= 1) n_pixels += (uint32_t)__shfl_xor((int)n_pixels, o);
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

template <bool COUNT, int WMEM, bool LREF, int TRIM, bool BIG = false, bool ONE = false, bool PACKET = false>
void launch_g(const KParams& kp, int device, hipStream_t stream, size_t smem) {
  const void* fn = (const void*)render_gwalk_kernel<COUNT, WMEM, LREF, TRIM, BIG, ONE, PACKET>;
  const int block = (BIG ? 256 : 128) * GWALK_WAVES;
  KParams p = kp;
  p.lane_lds = (uint32_t)((smem + 15) & ~(size_t)15);
  const size_t total = p.lane_lds + (size_t)block * sizeof(uint32_t);
  const int grid = resident_grid(fn, block, device, total, true, __PRETTY_FUNCTION__);
  hipLaunchKernelGGL((render_gwalk_kernel<COUNT, WMEM, LREF, TRIM, BIG, ONE, PACKET>), dim3(grid), dim3(block), total, stream, p);
  hip_check(hipGetLastError(), "render_gwalk_kernel launch");
}

template <bool COUNT, int TRIM>
void launch_g_mem(int wmem, bool lref, bool one, bool packet, const KParams& kp, int device, hipStream_t stream, size_t smem) {
  if constexpr (!(TRIM & TRIM_PROGRAMS)) /* packet walks: streams with generic leaf programs (render.hip plan) */
    if (wmem == WM_LDS && lref && packet) return launch_g<COUNT, WM_LDS, true, TRIM, false, false, true>(kp, device, stream, smem);
  if (wmem == WM_LDS) lref ? launch_g<COUNT, WM_LDS, true, TRIM>(kp, device, stream, smem)
                           : launch_g<COUNT, WM_LDS, false, TRIM>(kp, device, stream, smem);
  else if (wmem == WM_HYB && smem > G::LDS_SCENE_MAX_BYTES) {
    one ? launch_g<COUNT, WM_HYB, false, TRIM, true, true>(kp, device, stream, smem)
        : launch_g<COUNT, WM_HYB, false, TRIM, true, false>(kp, device, stream, smem);
  }
  else if (wmem == WM_HYB) launch_g<COUNT, WM_HYB, false, TRIM>(kp, device, stream, smem);
  else launch_g<COUNT, WM_BUF, false, TRIM>(kp, device, stream, smem);
}

}  // namespace

namespace hrt {

void launch_gwalk(bool count, int wmem, bool lref, int trim, bool one, bool packet, const KParams& kp, int device,
                  hipStream_t stream, size_t smem) {
  /* instantiated trims: none, media, heavy textures, both; TRIM_PROGRAMS with none (Final) or both (Cornell) */
  if (trim & TRIM_PROGRAMS) {
    const int base = trim & ~TRIM_PROGRAMS;
    if (base != 0 && base != (TRIM_MEDIA | TRIM_HEAVY_TEX)) trim = base;
  }
  if (count) {
    if (trim == (TRIM_MEDIA | TRIM_HEAVY_TEX | TRIM_PROGRAMS)) launch_g_mem<true, TRIM_MEDIA | TRIM_HEAVY_TEX | TRIM_PROGRAMS>(wmem, lref, one, packet, kp, device, stream, smem);
    else if (trim == (TRIM_MEDIA | TRIM_HEAVY_TEX)) launch_g_mem<true, TRIM_MEDIA | TRIM_HEAVY_TEX>(wmem, lref, one, packet, kp, device, stream, smem);
    else if (trim == TRIM_MEDIA) launch_g_mem<true, TRIM_MEDIA>(wmem, lref, one, packet, kp, device, stream, smem);
    else if (trim == TRIM_HEAVY_TEX) launch_g_mem<true, TRIM_HEAVY_TEX>(wmem, lref, one, packet, kp, device, stream, smem);
    else if (trim == TRIM_PROGRAMS) launch_g_mem<true, TRIM_PROGRAMS>(wmem, lref, one, packet, kp, device, stream, smem);
    else launch_g_mem<true, 0>(wmem, lref, one, packet, kp, device, stream, smem);
  } else {
    if (trim == (TRIM_MEDIA | TRIM_HEAVY_TEX | TRIM_PROGRAMS)) launch_g_mem<false, TRIM_MEDIA | TRIM_HEAVY_TEX | TRIM_PROGRAMS>(wmem, lref, one, packet, kp, device, stream, smem);
    else if (trim == (TRIM_MEDIA | TRIM_HEAVY_TEX)) launch_g_mem<false, TRIM_MEDIA | TRIM_HEAVY_TEX>(wmem, lref, one, packet, kp, device, stream, smem);
    else if (trim == TRIM_MEDIA) launch_g_mem<false, TRIM_MEDIA>(wmem, lref, one, packet, kp, device, stream, smem);
    else if (trim == TRIM_HEAVY_TEX) launch_g_mem<false, TRIM_HEAVY_TEX>(wmem, lref, one, packet, kp, device, stream, smem);
    else if (trim == TRIM_PROGRAMS) launch_g_mem<false, TRIM_PROGRAMS>(wmem, lref, one, packet, kp, device, stream, smem);
    else launch_g_mem<false, 0>(wmem, lref, one, packet, kp, device, stream, smem);
  }
}

}  // namespace hrt
