/*
 * lane_sim.hip — TEST INFRASTRUCTURE: runs the kernels' per-lane code (hyper-ray-tracer_amd/csrc/lane.h)
 * on the host, one lane at a time, over the flattened scene of hrt_debug_scene_blob.
 *
 * A GPU lane of render_basic_kernel / render_full_kernel executes, for each of its samples, exactly:
 * start_sample -> { walk to the end with walk_box/walk_prim (the sphere kernel under CULL_EXACT, over the
 * walk stream), basic_step or full_step; shade } until the path ends, and
 * sums the samples of a chunk in order (reduce_chunks then adds the chunk sums in chunk order).
 * Which lanes step together, and when a wave stops to shade, never changes a lane's own sequence of
 * tests and draws.  So this harness reproduces what the kernels compute per pixel, and
 * tests/test_lane_sim.py checks it against the CPU oracle (oracle/) without a GPU.  It is built by the
 * tests (host-only compile) and is not part of libhrt.
 */
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <vector>

#include "lane.h"
#include "walk_box.h"

using namespace hrt;
using namespace hrt::lane;

namespace {

/* ---- pricing a 4-wide walk, host only ----
 * The sphere walk stream's binary hierarchy (re-grouped over the reference leaf order) collapsed one level:
 * a wide record holds the boxes of a node's grandchildren (a leaf child is kept as it is), at most 4, in leaf
 * order.  A lane visiting a record tests all its child boxes at once (the inflated test box_ce with its
 * current closest) into a pass mask, then takes the passed children in order: a leaf gets its test right
 * away (walk_leaf_test: the reference box test and the sphere against the current closest), an inner child is
 * descended into with the rest of the mask kept on a per-level trail; a record whose mask runs out climbs
 * to its parent (a dependent load of the parent's links).  Leaves are tested in the reference's order, each
 * with the reference test, and every culled box holds its leaves, so the result must equal the binary walk's
 * bit for bit (checked per segment).  Counted per segment: binary node steps and leaf tests; wide records,
 * climbs, box tests, leaf tests; and per (8x8 block, sample, segment index) group the lockstep maxima. */
struct WideTree {
  struct N {
    float4 a, b;
    bool leaf;
    uint32_t payload;
    int kid[2];
    int wk[4];
    int nwk;
    double key; /* the builder's staging priority: the parent box's half area (scene.cpp walk_place_and_write) */
    int depth;
  };
  std::vector<N> T;
  int root = -1;
  /* hot[b][n]: node n staged in LDS under staging budget b (HOT_BUDGETS node parts) */
  std::vector<std::vector<char>> hot;
};
/* staged node parts: 77 KB of 32-B parts (today's sphere kernel), of 16-B parts (a compressed format in the
 * same LDS), 152 KB of 32-B parts (one 1024-thread workgroup per CU) */
constexpr uint32_t HOT_BUDGETS[3] = {77u * 1024u / 32u, 77u * 1024u / 16u, 152u * 1024u / 32u};
struct WideStats {
  uint64_t segs, bin_steps, bin_leaf, wide_records, wide_climbs, wide_tests, wide_leaf, mismatch;
  uint64_t depth_max;
  uint64_t lock_steps, lock_global[3]; /* lockstep binary steps; those where some lane reads a non-staged part */
};
WideTree* g_wide = nullptr;
/* segment recorder (scripts/price_hierarchy.py): origin, direction, final closest of every sphere-lane segment */
std::vector<float>* g_segs = nullptr;
int g_wide_arity = 4; /* 2: a record holds its node's two child boxes (no collapse) */
WideStats g_ws;
struct LockKey {
  uint32_t block, sample, seg;
  bool operator<(const LockKey& o) const {
    return block != o.block ? block < o.block : (sample != o.sample ? sample < o.sample : seg < o.seg);
  }
};
struct LockVal {
  uint32_t bin_max, wide_max, n;
  uint64_t bin_sum, wide_sum;
  std::vector<uint8_t> global; /* per binary step index: bit b set when some lane's node is cold under budget b */
};
std::map<LockKey, LockVal>* g_lock = nullptr;
std::map<uint64_t, uint32_t>* g_segidx = nullptr; /* (pixel, sample) -> segments so far */

int wide_parse(const WalkSrc& src, uint32_t off, WideTree& W, double key = 1e300, int depth = 0) {
  const float4 a = wload<WM_HOST>(src, off), b = wload<WM_HOST>(src, off + src.half);
  const int id = (int)W.T.size();
  W.T.push_back(WideTree::N{a, b, false, 0u, {-1, -1}, {-1, -1, -1, -1}, 0, key, depth});
  const uint32_t pass = f2u(b.w);
  if (walk_pending(pass)) {
    W.T[id].leaf = true;
    W.T[id].payload = pass - WALK_PEND;
    return id;
  }
  const double ha = 4.0 * ((double)b.x * b.y + (double)b.y * b.z + (double)b.z * b.x); /* half area of [C - E, C + E] */
  const int c0 = wide_parse(src, pass, W, ha, depth + 1);
  const int c1 = wide_parse(src, f2u(W.T[c0].a.w), W, ha, depth + 1); /* the first child's skip: its next sibling */
  W.T[id].kid[0] = c0;
  W.T[id].kid[1] = c1;
  int n = 0;
  for (int k : {c0, c1}) {
    if (W.T[k].leaf || g_wide_arity == 2) W.T[id].wk[n++] = k;
    else {
      W.T[id].wk[n++] = W.T[k].kid[0];
      W.T[id].wk[n++] = W.T[k].kid[1];
    }
  }
  W.T[id].nwk = n;
  return id;
}

/* the binary walk again over the parsed tree (the kernel's walk without speculation: the same node
 * sequence as walk_step_host), recording the nodes it visits */
void bin_walk_nodes(const KParams& P, const WalkSrc& src, const TRay& r, int n, float& closest, uint32_t& winner,
                    std::vector<int>& seq) {
  const WideTree& W = *g_wide;
  Counts cn{0u, 0u, 0u, 0u, 0u, 0u};
  seq.push_back(n);
  if (!box_ce<HRT_BOX_FMA != 0, false>(W.T[n].a, W.T[n].b, r, P.t_min, closest)) return;
  if (W.T[n].leaf) {
    walk_leaf_test<true, WM_HOST>(P, src, W.T[n].payload, r, closest, winner, cn);
    return;
  }
  bin_walk_nodes(P, src, r, W.T[n].kid[0], closest, winner, seq);
  bin_walk_nodes(P, src, r, W.T[n].kid[1], closest, winner, seq);
}

void wide_price_segment(const KParams& P, const WalkSrc& src, const TRay& r, float bin_closest, uint32_t bin_winner,
                        uint32_t bin_steps, uint32_t bin_leaf, uint32_t px, uint32_t py, uint32_t sample) {
  const WideTree& W = *g_wide;
  Counts cn{0u, 0u, 0u, 0u, 0u, 0u};
  float closest = u2f(0x7f800000u);
  uint32_t winner = G::NONE;
  uint64_t records = 0, climbs = 0, tests = 0;
  struct Lv {
    int node;
    uint32_t mask;
  } st[96];
  int depth = 0;
  auto visit = [&](int n) {
    records++;
    uint32_t m = 0;
    const WideTree::N& N = W.T[n];
    for (int j = 0; j < N.nwk; j++) {
      const WideTree::N& K = W.T[N.wk[j]];
      tests++;
      if (box_ce<HRT_BOX_FMA != 0, false>(K.a, K.b, r, P.t_min, closest)) m |= 1u << j;
    }
    st[depth++] = Lv{n, m};
    if ((uint64_t)depth > g_ws.depth_max) g_ws.depth_max = depth;
  };
  const WideTree::N& R = W.T[W.root];
  if (R.leaf) {
    tests++;
    if (box_ce<HRT_BOX_FMA != 0, false>(R.a, R.b, r, P.t_min, closest)) walk_leaf_test<true, WM_HOST>(P, src, R.payload, r, closest, winner, cn);
  } else {
    visit(W.root);
    while (depth > 0) {
      Lv& top = st[depth - 1];
      if (top.mask == 0) {
        depth--;
        if (depth > 0) climbs++;
        continue;
      }
      const int j = __builtin_ctz(top.mask);
      top.mask &= top.mask - 1u;
      const int k = W.T[top.node].wk[j];
      if (W.T[k].leaf) walk_leaf_test<true, WM_HOST>(P, src, W.T[k].payload, r, closest, winner, cn);
      else visit(k);
    }
  }
  g_ws.segs++;
  g_ws.bin_steps += bin_steps;
  g_ws.bin_leaf += bin_leaf;
  g_ws.wide_records += records;
  g_ws.wide_climbs += climbs;
  g_ws.wide_tests += tests;
  g_ws.wide_leaf += cn.prims;
  if (f2u(closest) != f2u(bin_closest) || winner != bin_winner) g_ws.mismatch++;
  /* lockstep groups: the 64 lanes of an 8x8 block at one sample and one segment index */
  const uint64_t key = ((uint64_t)(py * P.W + px) << 20) | sample;
  const uint32_t seg = (*g_segidx)[key]++;
  LockVal& v = (*g_lock)[LockKey{(py / 8u) * 4096u + px / 8u, sample, seg}];
  const uint32_t wide_dep = (uint32_t)(records + climbs);
  {
    std::vector<int> seq;
    float cl = u2f(0x7f800000u);
    uint32_t wn = G::NONE;
    bin_walk_nodes(P, src, r, W.root, cl, wn, seq);
    if (f2u(cl) != f2u(bin_closest) || wn != bin_winner) g_ws.mismatch++;
    if (v.global.size() < seq.size()) v.global.resize(seq.size(), 0);
    for (size_t k = 0; k < seq.size(); k++)
      for (int b = 0; b < 3; b++)
        if (!W.hot[b][seq[k]]) v.global[k] |= (uint8_t)(1u << b);
  }
  v.bin_max = std::max(v.bin_max, bin_steps);
  v.wide_max = std::max(v.wide_max, wide_dep);
  v.bin_sum += bin_steps;
  v.wide_sum += wide_dep;
  v.n++;
}

/* KIND 0: render_basic_kernel's lane, 1: render_full_kernel's lane, 2: render_kernel's (segment()),
 * 3: render_gwalk_kernel's (the general walk stream) */
template <int CULL, int KIND>
void render_pixel(const KParams& P, uint32_t px, uint32_t py, float* rgba, uint64_t* cnt) {
  constexpr bool FULL = KIND == 1;
  const uint32_t spp = P.spp;
  const uint32_t n_chunks = P.n_chunks; /* render.hip: lane.h sample_chunk + chunk_plan, set by the caller */
  const float inf = u2f(0x7f800000u);
  Counts cn{0u, 0u, 0u, 0u, 0u, 0u};
  Vec3 total = v3(0.0f, 0.0f, 0.0f);
  for (uint32_t c = 0; c < n_chunks; c++) {
    Vec3 sum = v3(0.0f, 0.0f, 0.0f);
    uint32_t s_begin, s_end;
    chunk_range(P, c, s_begin, s_end);
    for (uint32_t sample = s_begin; sample < s_end; sample++) {
      PathState ps;
      init_path_state(ps);
      start_sample(P, ps, px, py, sample);
      if constexpr (KIND == 2) { /* one world.hit per segment() call (render_kernel) */
        for (;;) {
          const bool done = segment<CULL, true, true, false>(P, P.nodes, P.prims, ps, cn, nullptr);
          if (ps.traced) cnt[0]++;
          if (done) break;
        }
        sum = sum + ps.rad;
        cnt[1]++;
        continue;
      }
      TRay r;
      set_ray(r, ps.ro, ps.rd, ps.rtime, P);
      Vec3 wo = ps.ro, wd = ps.rd;
      for (;;) {
        bool traced, done;
        if constexpr (KIND == 3) { /* render_gwalk_kernel: the general walk stream, leaf programs, shade<true> */
          uint32_t node = ps.depth_left == 0 ? G::NONE : 0u, winner = G::NONE, gstate = 0x7FFFFFFFu;
          float closest = inf;
          WalkSrc src;
          src.base = P.walk;
          src.half = P.walk_half;
          uint32_t last_chain = G::NONE; /* pricing: instance-chain leaves and repeats of the previous chain */
          while (node < P.walk_end) {
            walk_box<true, WM_HOST>(src, node, r, P.t_min, closest, cn);
            if (walk_pending(node)) {
              const uint32_t leaf = node - G::WALK_PEND;
              const float4 h = wload<WM_HOST>(src, leaf), bmn = wload<WM_HOST>(src, leaf + 16u);
              if (f2u(h.z) & G::GL_INST) {
                cnt[5]++;                                    /* cnt[5]: leaf tests of instance-chain leaves */
                if (f2u(bmn.w) == last_chain) cnt[6]++;      /* cnt[6]: ... whose chain the previous one shared */
                last_chain = f2u(bmn.w);
              }
              gwalk_prim<true, true, WM_HOST>(P, P.nodes, P.prims, src, node, r, closest, winner, gstate, ps.pk, cn);
            }
          }
          traced = node != G::NONE;
          done = true;
          if (traced) {
            ps.pk.segment++;
            done = shade<true, true>(P, ps, winner, closest, r.o, r.d, r.time, r.tau, cn) || ps.depth_left == 0;
          }
        } else if constexpr (FULL) {
          FullWalk w{0u, P.main_end, 0u, 0u, P.t_min, inf, G::NONE, inf, 0.0f, G::NONE};
          if (ps.depth_left == 0) w.i = G::NONE;
          while (w.i < w.end) full_step<CULL, true>(P, P.nodes, P.prims, w, r, wo, wd, ps.pk, cn);
          traced = w.i != G::NONE;
          done = true;
          if (traced) {
            ps.pk.segment++;
            done = shade<true, true>(P, ps, w.wn, w.cl, wo, wd, r.time, r.tau, cn) || ps.depth_left == 0;
          }
        } else {
          uint32_t node = ps.depth_left == 0 ? G::NONE : 0u, winner = G::NONE;
          float closest = inf;
          if constexpr (CULL == G::CULL_EXACT) { /* the walk stream (layout.h), as the kernel walks it */
            WalkSrc src;
            src.base = P.walk;
          src.half = P.walk_half;
            const uint32_t nodes0 = cn.nodes, prims0 = cn.prims;
            if (P.walk_c16)
              while (node < P.walk_end) walk_step_host<true, true>(P, src, node, r, closest, winner, cn);
            else
              while (node < P.walk_end) walk_step_host<true>(P, src, node, r, closest, winner, cn);
            if (g_wide && node != G::NONE) wide_price_segment(P, src, r, closest, winner, cn.nodes - nodes0, cn.prims - prims0, px, py, sample);
            if (g_segs && node != G::NONE)
              g_segs->insert(g_segs->end(), {r.o.x, r.o.y, r.o.z, r.d.x, r.d.y, r.d.z, closest});
          } else {
            while (node < P.main_end) basic_step<CULL, true>(P, P.nodes, P.prims, node, r, closest, winner, cn);
          }
          traced = node != G::NONE;
          if constexpr (CULL == G::CULL_EXACT) {
            WalkSrc src;
            src.base = P.walk;
          src.half = P.walk_half;
            done = !traced || shade_walk<true, WM_HOST, true>(P, src, ps, winner, closest, r.o, r.d, r.time, r.tau, sum, cn) ||
                   ps.depth_left == 0;
          } else {
            done = !traced ||
                   shade<false, true>(P, ps, winner, closest, r.o, r.d, r.time, r.tau, cn) || ps.depth_left == 0;
          }
        }
        if (traced) cnt[0]++;
        if (done) break;
        set_dir(r, ps.ro, ps.rd); /* the scattered ray keeps the sample's shutter time */
        wo = ps.ro;
        wd = ps.rd;
      }
      sum = sum + ps.rad;
      cnt[1]++;
    }
    total = c == 0 ? sum : total + sum;
  }
  const float scale = 1.0f / (float)spp;
  rgba[0] = sqrtf(total.x * scale);
  rgba[1] = sqrtf(total.y * scale);
  rgba[2] = sqrtf(total.z * scale);
  rgba[3] = 1.0f;
  cnt[2] += cn.nodes;
  cnt[3] += cn.prims;
  cnt[4] += cn.tex;
}

}  // namespace

extern "C" {

/* the sample chunks of a pixel (lane.h chunk_plan / chunk_range): ranges[2k], ranges[2k+1] = [s0, s1) of
 * chunk k; returns the number of chunks (the caller's cap permitting) */
int lane_sim_chunks(uint32_t spp, uint32_t cls, int tail, uint32_t* ranges, uint32_t cap) {
  KParams P;
  memset(&P, 0, sizeof(P));
  P.spp = spp;
  P.chunk = sample_chunk(spp, cls);
  uint32_t nh = 0, first = 0, nt = 0;
  chunk_plan(spp, P.chunk, tail, nh, first, nt);
  P.chunk_head = nh;
  P.chunk_first = first;
  P.n_chunks = nh + nt;
  for (uint32_t k = 0; k < P.n_chunks && k < cap; k++) chunk_range(P, k, ranges[2 * k], ranges[2 * k + 1]);
  return (int)P.n_chunks;
}

/* kernel: 0 = render_basic_kernel's lane, 1 = render_full_kernel's, 2 = render_kernel's (segment
 * at a time), 3 = render_gwalk_kernel's (general walk stream; CULL_EXACT); cull: layout.h CULL_*.
 * cnt[0..4] += segments, samples, node visits, primitive tests, texture evaluations. */
int lane_sim_render(const void* blob, const hrt_blob_info* bi, const hrt_camera* cam, const hrt_render_params* p,
                    int kernel, int cull, uint32_t x0, uint32_t y0, uint32_t w, uint32_t h, float* rgba,
                    uint64_t* cnt) {
  const uint8_t* base = (const uint8_t*)blob;
  KParams P;
  memset(&P, 0, sizeof(P));
  P.nodes = (const G::Node*)(base + bi->off_nodes);
  P.prims = (const G::Prim*)(base + bi->off_prims);
  P.insts = (const G::Inst*)(base + bi->off_insts);
  P.media = (const G::Medium*)(base + bi->off_media);
  P.mats = (const G::Mat*)(base + bi->off_mats);
  P.texs = (const G::Tex*)(base + bi->off_texs);
  P.perlin = (const G::Perlin*)(base + bi->off_perlin);
  P.images = base + bi->off_images;
  P.chains = (const float4*)(base + bi->off_chains);
  P.main_end = bi->main_end;
  P.ln_e = bi->ln_e;
  P.motion_uniform = bi->motion_uniform;
  P.motion_t0 = bi->motion_t0;
  P.motion_span = bi->motion_span;
  P.walk = base + bi->off_walk;
  P.walk_bytes = bi->walk_bytes;
  P.walk_end = bi->walk_c16 ? bi->walk_nodes : bi->walk_bytes; /* layout.h WALK_C16: node indices */
  P.walk_hot = bi->walk_hot;
  P.walk_half = bi->walk_half ? bi->walk_half : 16u;
  P.walk_c16 = bi->walk_c16;
  P.walk_pbase = bi->walk_pbase;
  P.cam_origin = v3(cam->origin[0], cam->origin[1], cam->origin[2]);
  P.cam_llc = v3(cam->lower_left_corner[0], cam->lower_left_corner[1], cam->lower_left_corner[2]);
  P.cam_h = v3(cam->horizontal[0], cam->horizontal[1], cam->horizontal[2]);
  P.cam_v = v3(cam->vertical[0], cam->vertical[1], cam->vertical[2]);
  P.cam_u = v3(cam->u[0], cam->u[1], cam->u[2]);
  P.cam_vv = v3(cam->v[0], cam->v[1], cam->v[2]);
  P.lens_radius = cam->lens_radius;
  P.time0 = cam->time0;
  P.time1 = cam->time1;
  P.W = p->width;
  P.H = p->height;
  set_pixel_rcp(P);
  P.spp = p->samples;
  {
    uint32_t nh = 0, first = 0, nt = 0; /* the default scene options (hrt_scene_options all zero) */
    frame_chunks(P.spp, chunk_class(bi->feature_mask, bi->main_end), P.W, P.H, 0u, 0u, 32u, P.chunk, nh, first, nt);
    P.chunk_head = nh;
    P.chunk_first = first;
    P.n_chunks = nh + nt;
  }
  P.max_depth = p->max_depth;
  P.sample_offset = p->sample_offset;
  P.t_min = p->t_min;
  P.background = v3(p->background[0], p->background[1], p->background[2]);
  P.seed = p->seed;
  if (kernel == 0 && (bi->feature_mask & ~(G::F_BASIC | G::F_HEAVY_TEX)) != 0) return 1; /* not a sphere scene */
  if (kernel == 3 && (bi->walk_bytes == 0 || !bi->walk_general)) return 1; /* no general stream */
  if (kernel == 0 && bi->walk_general && cull == G::CULL_EXACT) return 1;      /* no sphere stream */
  for (uint32_t y = 0; y < h; y++)
    for (uint32_t x = 0; x < w; x++) {
      float* o = rgba + 4 * ((size_t)y * w + x);
      if (kernel == 0) {
        if (cull == G::CULL_EXACT) render_pixel<G::CULL_EXACT, 0>(P, x0 + x, y0 + y, o, cnt);
        else if (cull == G::CULL_SLAB) render_pixel<G::CULL_SLAB, 0>(P, x0 + x, y0 + y, o, cnt);
        else render_pixel<G::CULL_REFERENCE, 0>(P, x0 + x, y0 + y, o, cnt);
      } else if (kernel == 1) {
        if (cull == G::CULL_EXACT) render_pixel<G::CULL_EXACT, 1>(P, x0 + x, y0 + y, o, cnt);
        else if (cull == G::CULL_SLAB) render_pixel<G::CULL_SLAB, 1>(P, x0 + x, y0 + y, o, cnt);
        else render_pixel<G::CULL_REFERENCE, 1>(P, x0 + x, y0 + y, o, cnt);
      } else if (kernel == 3) {
        render_pixel<G::CULL_EXACT, 3>(P, x0 + x, y0 + y, o, cnt);
      } else {
        if (cull == G::CULL_EXACT) render_pixel<G::CULL_EXACT, 2>(P, x0 + x, y0 + y, o, cnt);
        else if (cull == G::CULL_SLAB) render_pixel<G::CULL_SLAB, 2>(P, x0 + x, y0 + y, o, cnt);
        else render_pixel<G::CULL_REFERENCE, 2>(P, x0 + x, y0 + y, o, cnt);
      }
    }
  return 0;
}


/* Price the 4-wide walk over the sphere scene's walk stream on a region (render_basic_kernel's lane, EXACT):
 * renders the region as lane_sim_render (rgba, cnt), and for every segment walks the wide hierarchy too.
 * out[0..15]: segments, binary node steps, binary leaf tests, wide records, wide climbs, wide box tests, wide
 * leaf tests, segments whose wide result differs (must be 0), deepest trail, lockstep groups, sum over groups
 * of 64 x the binary max steps, of 64 x the wide max dependent loads (records + climbs), lockstep binary steps,
 * and those of them where some lane reads a node part not staged in LDS under each of HOT_BUDGETS.  arity 2: records of
 * the two child boxes of a node (no collapse), 4: of its grandchildren. */
int lane_sim_wide_price(const void* blob, const hrt_blob_info* bi, const hrt_camera* cam, const hrt_render_params* p,
                        uint32_t x0, uint32_t y0, uint32_t w, uint32_t h, float* rgba, uint64_t* cnt, uint64_t* out,
                        int arity) {
  if (bi->walk_bytes == 0 || bi->walk_general || bi->walk_c16 || (arity != 2 && arity != 4)) return 1;
  g_wide_arity = arity;
  WideTree W;
  WalkSrc src;
  src.base = (const uint8_t*)blob + bi->off_walk;
  src.half = bi->walk_half ? bi->walk_half : 16u;
  W.root = wide_parse(src, 0u, W);
  { /* the staged sets under each budget, by the builder's rule (largest parent box first, then depth) */
    std::vector<int> order(W.T.size());
    for (size_t i = 0; i < order.size(); i++) order[i] = (int)i;
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) {
      return W.T[x].key != W.T[y].key ? W.T[x].key > W.T[y].key : W.T[x].depth < W.T[y].depth;
    });
    W.hot.assign(3, std::vector<char>(W.T.size(), 0));
    for (int b = 0; b < 3; b++)
      for (size_t k = 0; k < order.size() && k < HOT_BUDGETS[b]; k++) W.hot[b][order[k]] = 1;
  }
  std::map<LockKey, LockVal> lock;
  std::map<uint64_t, uint32_t> segidx;
  g_wide = &W;
  g_lock = &lock;
  g_segidx = &segidx;
  memset(&g_ws, 0, sizeof(g_ws));
  const int rc = lane_sim_render(blob, bi, cam, p, 0, G::CULL_EXACT, x0, y0, w, h, rgba, cnt);
  g_wide = nullptr;
  g_lock = nullptr;
  g_segidx = nullptr;
  uint64_t groups = 0, bmax = 0, wmax = 0, lsteps = 0, lglob[3] = {0, 0, 0};
  for (const auto& kv : lock) {
    groups++;
    bmax += 64ull * kv.second.bin_max;
    wmax += 64ull * kv.second.wide_max;
    lsteps += kv.second.global.size();
    for (uint8_t g : kv.second.global)
      for (int b = 0; b < 3; b++) lglob[b] += (g >> b) & 1u;
  }
  const uint64_t v[16] = {g_ws.segs, g_ws.bin_steps, g_ws.bin_leaf, g_ws.wide_records, g_ws.wide_climbs, g_ws.wide_tests,
                          g_ws.wide_leaf, g_ws.mismatch, g_ws.depth_max, groups, bmax, wmax, lsteps, lglob[0], lglob[1], lglob[2]};
  memcpy(out, v, sizeof(v));
  return rc;
}

/* For every range [i, j) of a leaf sequence (boxes n x (mn, mx)), how many of the rays (m x (o, d, closest))
 * pass the walk's inflated test (lane.h box_ce, fused form) of the range's union box on [tmin, closest]:
 * out[i * (n + 1) + j].  Pricing hierarchies over a fixed leaf order (scripts/price_hierarchy.py). */
int lane_sim_range_pass(const float* boxes, uint32_t n, const float* rays, uint32_t m, float tmin, uint32_t* out) {
  std::vector<TRay> R(m);
  std::vector<float> cl(m);
  for (uint32_t q = 0; q < m; q++) {
    set_dir(R[q], v3(rays[7 * q], rays[7 * q + 1], rays[7 * q + 2]), v3(rays[7 * q + 3], rays[7 * q + 4], rays[7 * q + 5]));
    cl[q] = rays[7 * q + 6];
  }
  for (uint32_t i = 0; i < n; i++) {
    float mn[3] = {boxes[6 * i], boxes[6 * i + 1], boxes[6 * i + 2]}, mx[3] = {boxes[6 * i + 3], boxes[6 * i + 4], boxes[6 * i + 5]};
    for (uint32_t j = i + 1; j <= n; j++) {
      if (j > i + 1)
        for (int k = 0; k < 3; k++) {
          mn[k] = std::min(mn[k], boxes[6 * (j - 1) + k]);
          mx[k] = std::max(mx[k], boxes[6 * (j - 1) + 3 + k]);
        }
      float C[3], E[3], fmn[3], fmx[3];
      walkbox::ce_floored(mn, mx, C, E, fmn, fmx);
      const float4 a = make_float4(C[0], C[1], C[2], 0.0f), b = make_float4(E[0], E[1], E[2], 0.0f);
      uint32_t c = 0;
      for (uint32_t q = 0; q < m; q++) c += box_ce<true, false>(a, b, R[q], tmin, cl[q]) ? 1u : 0u;
      out[(size_t)i * (n + 1) + j] = c;
    }
  }
  return 0;
}

/* Every segment of a region's sphere-lane render (EXACT): out[7 k ..] = origin, direction, final closest (+inf on a
 * miss); returns the number of segments (all of them are counted; at most cap are written). */
int lane_sim_segments(const void* blob, const hrt_blob_info* bi, const hrt_camera* cam, const hrt_render_params* p,
                      uint32_t x0, uint32_t y0, uint32_t w, uint32_t h, float* out, uint32_t cap) {
  std::vector<float> segs;
  std::vector<float> rgba((size_t)w * h * 4);
  uint64_t cnt[8] = {0};
  g_segs = &segs;
  const int rc = lane_sim_render(blob, bi, cam, p, 0, G::CULL_EXACT, x0, y0, w, h, rgba.data(), cnt);
  g_segs = nullptr;
  if (rc) return -1;
  const size_t n = segs.size() / 7;
  memcpy(out, segs.data(), std::min<size_t>(n, cap) * 7 * sizeof(float));
  return (int)n;
}

/* The culling property behind CULL_EXACT on single spheres: whenever the reference's
 * sphere test (sphere.rs:38-55, lane.h sphere_root_at) accepts a root in [tmin, tmax], the walk's inflated
 * test (lane.h box_ce, both forms) on the sphere's box as the stream builder encodes it (walk_box.h
 * ce_floored over sphere.rs's bounding box) must pass.  sph: n x (cx, cy, cz, r); rays: m x (o, d).
 * cnt: [pairs accepted, accepted outside the sphere's box (grazing false hits), culled by the fused form,
 * culled by the sub/mul/add form, boxes raised by the floor, rays in NaN mode] */
int lane_sim_cull_property(const float* sph, uint32_t n_sph, const float* rays, uint32_t n_rays, float tmin,
                           float tmax, uint64_t* cnt) {
  for (uint32_t q = 0; q < n_rays; q++) {
    TRay r;
    set_dir(r, v3(rays[6 * q], rays[6 * q + 1], rays[6 * q + 2]), v3(rays[6 * q + 3], rays[6 * q + 4], rays[6 * q + 5]));
    if (r.noinv.x != r.noinv.x) cnt[5]++;
  }
  for (uint32_t i = 0; i < n_sph; i++) {
    const Vec3 c = v3(sph[4 * i], sph[4 * i + 1], sph[4 * i + 2]);
    const float rad = sph[4 * i + 3];
    const Vec3 rv = v3(rad, rad, rad);
    const Vec3 bmn = c - rv, bmx = c + rv; /* sphere.rs bounding_box */
    const float mn[3] = {bmn.x, bmn.y, bmn.z}, mx[3] = {bmx.x, bmx.y, bmx.z};
    float C[3], E[3], fmn[3], fmx[3];
    if (walkbox::ce_floored(mn, mx, C, E, fmn, fmx)) cnt[4]++;
    const float4 a = make_float4(C[0], C[1], C[2], 0.0f), b = make_float4(E[0], E[1], E[2], 0.0f);
    for (uint32_t q = 0; q < n_rays; q++) {
      TRay r;
      set_dir(r, v3(rays[6 * q], rays[6 * q + 1], rays[6 * q + 2]), v3(rays[6 * q + 3], rays[6 * q + 4], rays[6 * q + 5]));
      float t;
      if (!sphere_root_at(c, rad, r, tmin, tmax, t)) continue;
      cnt[0]++;
      const Vec3 p = r.o + t * r.d;
      if (p.x < mn[0] || p.x > mx[0] || p.y < mn[1] || p.y > mx[1] || p.z < mn[2] || p.z > mx[2]) cnt[1]++;
      if (!box_ce<true>(a, b, r, tmin, tmax)) cnt[2]++;
      if (!box_ce<false>(a, b, r, tmin, tmax)) cnt[3]++;
    }
  }
  return 0;
}

/* the one-quadratic medium boundary (lane.h sphere_pair_at, what medium_pair / GL_MED leaves use)
 * against the two boundary queries of constant_medium.rs:37-48 as the sphere test makes them
 * (sphere_root_at over (-inf, inf), then over (t1 + 0.0001, inf)).  sph: n x (c, r); rays: m x (o, d).
 * out[6 * (i * m + q) ..]: pair hits, t1, t2, two-call hits, t1, t2 (t = +inf where there is no hit). */
int lane_sim_sphere_pair(const float* sph, uint32_t n_sph, const float* rays, uint32_t n_rays, float* out) {
  const float inf = u2f(0x7f800000u);
  for (uint32_t i = 0; i < n_sph; i++) {
    const Vec3 c = v3(sph[4 * i], sph[4 * i + 1], sph[4 * i + 2]);
    const float rad = sph[4 * i + 3];
    for (uint32_t q = 0; q < n_rays; q++) {
      const Vec3 o = v3(rays[6 * q], rays[6 * q + 1], rays[6 * q + 2]), d = v3(rays[6 * q + 3], rays[6 * q + 4], rays[6 * q + 5]);
      float* w = out + 6 * ((size_t)i * n_rays + q);
      float p1 = inf, p2 = inf;
      w[0] = (float)sphere_pair_at(c, rad, o, d, p1, p2);
      w[1] = p1;
      w[2] = p2;
      TRay r;
      set_dir(r, o, d);
      float t1 = inf, t2 = inf;
      int hits = 0;
      if (sphere_root_at(c, rad, r, -inf, inf, t1)) {
        hits = 1;
        if (sphere_root_at(c, rad, r, t1 + 0.0001f, inf, t2)) hits = 2;
      }
      w[3] = (float)hits;
      w[4] = hits > 0 ? t1 : inf;
      w[5] = hits > 1 ? t2 : inf;
    }
  }
  return 0;
}

}  // extern "C"

extern "C" {
/* One path of render_kernel's lane (segment at a time) with culling `cull`: out[9 * k ..] = origin,
 * direction, time, closest, winner (bits) of segment k; returns the number of segments (diagnostics). */
int lane_sim_path(const void* blob, const hrt_blob_info* bi, const hrt_camera* cam, const hrt_render_params* p,
                  int cull, uint32_t px, uint32_t py, uint32_t sample, float* out, uint32_t cap) {
  std::vector<float> img(4);
  KParams P;
  memset(&P, 0, sizeof(P));
  const uint8_t* base = (const uint8_t*)blob;
  P.nodes = (const G::Node*)(base + bi->off_nodes);
  P.prims = (const G::Prim*)(base + bi->off_prims);
  P.insts = (const G::Inst*)(base + bi->off_insts);
  P.media = (const G::Medium*)(base + bi->off_media);
  P.mats = (const G::Mat*)(base + bi->off_mats);
  P.texs = (const G::Tex*)(base + bi->off_texs);
  P.perlin = (const G::Perlin*)(base + bi->off_perlin);
  P.images = base + bi->off_images;
  P.chains = (const float4*)(base + bi->off_chains);
  P.main_end = bi->main_end;
  P.ln_e = bi->ln_e;
  P.motion_uniform = bi->motion_uniform;
  P.motion_t0 = bi->motion_t0;
  P.motion_span = bi->motion_span;
  P.cam_origin = v3(cam->origin[0], cam->origin[1], cam->origin[2]);
  P.cam_llc = v3(cam->lower_left_corner[0], cam->lower_left_corner[1], cam->lower_left_corner[2]);
  P.cam_h = v3(cam->horizontal[0], cam->horizontal[1], cam->horizontal[2]);
  P.cam_v = v3(cam->vertical[0], cam->vertical[1], cam->vertical[2]);
  P.cam_u = v3(cam->u[0], cam->u[1], cam->u[2]);
  P.cam_vv = v3(cam->v[0], cam->v[1], cam->v[2]);
  P.lens_radius = cam->lens_radius;
  P.time0 = cam->time0;
  P.time1 = cam->time1;
  P.W = p->width;
  P.H = p->height;
  set_pixel_rcp(P);
  P.spp = p->samples;
  P.max_depth = p->max_depth;
  P.sample_offset = p->sample_offset;
  P.t_min = p->t_min;
  P.background = v3(p->background[0], p->background[1], p->background[2]);
  P.seed = p->seed;
  PathState ps;
  init_path_state(ps);
  start_sample(P, ps, px, py, sample);
  Counts cn{0u, 0u, 0u, 0u, 0u, 0u};
  uint32_t n = 0;
  float scratch[9];
  for (;;) {
    bool done;
    float* d = n < cap ? out + 9 * n : scratch;
    if (cull == G::CULL_EXACT) done = segment<G::CULL_EXACT, true, false, false>(P, P.nodes, P.prims, ps, cn, d);
    else done = segment<G::CULL_REFERENCE, true, false, false>(P, P.nodes, P.prims, ps, cn, d);
    if (ps.traced) n++;
    if (done) break;
  }
  return (int)n;
}

/* The reference node stream's box decisions for one ray (o, d, time) over [0, main_end): for each node the
 * reference test (aabb.rs) and the EXACT test (box_hit<CULL_EXACT>) at the closest the REFERENCE walk has
 * when it reaches the node; dec[i] bit 0 = visited by the reference walk, bit 1 = reference pass, bit 2 =
 * exact pass; returns the reference walk's winner (diagnostics). */
int lane_sim_ray_boxes(const void* blob, const hrt_blob_info* bi, const float* od, float time, float tmin,
                       uint8_t* dec, float* closest_out) {
  const uint8_t* base = (const uint8_t*)blob;
  const G::Node* nodes = (const G::Node*)(base + bi->off_nodes);
  const G::Prim* prims = (const G::Prim*)(base + bi->off_prims);
  KParams P;
  memset(&P, 0, sizeof(P));
  P.motion_uniform = bi->motion_uniform;
  P.motion_t0 = bi->motion_t0;
  P.motion_span = bi->motion_span;
  TRay r;
  set_ray(r, v3(od[0], od[1], od[2]), v3(od[3], od[4], od[5]), time, P);
  float closest = u2f(0x7f800000u);
  int winner = -1;
  for (uint32_t i = 0; i < bi->main_end;) {
    const G::Node* np = nodes + i;
    const float4 a = ld4(np->mn), b = ld4(np->mx);
    const uint32_t kp = f2u(b.w), kind = (kp >> 24) & G::KIND_MASK, payload = kp & 0xFFFFFFu;
    dec[i] |= 1;
    if (kind == G::K_BOX || kind == G::K_BOX_PRIM) {
      const bool ref = box_hit<G::CULL_REFERENCE>(a, b, r, tmin, closest);
      const bool ex = box_hit<G::CULL_EXACT>(a, b, r, tmin, closest, (kp & G::NODE_REF_ONLY) != 0);
      dec[i] |= (ref ? 2 : 0) | (ex ? 4 : 0);
      if (kind == G::K_BOX) { i = ref ? i + 1 : f2u(a.w); continue; }
      i++;
      if (!ref) continue;
    } else if (kind == G::K_PRIM) {
      i++;
    } else {
      return -2; /* instances / media: not handled here */
    }
    const G::Prim* pp = prims + payload;
    float t;
    bool h;
    if ((pp->km & 3u) == G::P_RECT) h = rect_t(pp, (pp->km >> 2) & 3u, r, tmin, closest, t);
    else h = sphere_root(pp, pp->km & 3u, r, tmin, closest, t, P.motion_uniform != 0);
    if (h) { closest = t; winner = (int)(i - 1); }
  }
  *closest_out = closest;
  return winner;
}
}  // extern "C"

/* lane.h's Perlin noise (op 0) and the noise texture's scalar turbulence term (op 1: noise_value_t, i.e.
 * 1 + sin(scale p.z + 10 |turbulence(scale p, 7)|)) on explicit tables (ranvec 256 x 3, perm 3 x 256, the
 * oracle's layout), for the bit-for-bit check against oracle_perlin (tests/test_lane_sim.py) */
extern "C" float lane_sim_perlin(const float* ranvec, const uint32_t* perm, int op, const float* p, float scale) {
  static G::Perlin pn;
  for (int i = 0; i < 256; i++) {
    pn.ranvec[i][0] = ranvec[3 * i];
    pn.ranvec[i][1] = ranvec[3 * i + 1];
    pn.ranvec[i][2] = ranvec[3 * i + 2];
    pn.ranvec[i][3] = 0.0f;
    for (int c = 0; c < 3; c++) pn.perm[c][i] = pn.perm[c][256 + i] = perm[256 * c + i];
  }
  const Vec3 q = v3(p[0], p[1], p[2]);
  return op == 0 ? perlin_noise(&pn, q) : noise_value_t(&pn, scale, q);
}

/* rotation.rs:104-117 in both of lane.h's forms on the same rays: the run-time-axis form (rotate_any on the host)
 * and the per-axis instantiation the device runs for a wave turning about one axis (rotate_axis<AX>);
 * out[12 i ...] = generic o, d, then specialised o, d */
extern "C" void lane_sim_rotate(uint32_t n, const uint32_t* axis, const float* sc, const float* od, float* out) {
  for (uint32_t i = 0; i < n; i++) {
    const float s = sc[2 * i], c = sc[2 * i + 1];
    Vec3 o = v3(od[6 * i], od[6 * i + 1], od[6 * i + 2]), d = v3(od[6 * i + 3], od[6 * i + 4], od[6 * i + 5]);
    Vec3 go = o, gd = d;
    rotate_any(axis[i], s, c, go, gd);
    if (axis[i] == 0u) rotate_axis<0>(s, c, o, d);
    else if (axis[i] == 1u) rotate_axis<1>(s, c, o, d);
    else rotate_axis<2>(s, c, o, d);
    const float v[12] = {go.x, go.y, go.z, gd.x, gd.y, gd.z, o.x, o.y, o.z, d.x, d.y, d.z};
    for (int k = 0; k < 12; k++) out[12 * i + k] = v[k];
  }
}
