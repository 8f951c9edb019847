/*
 * scene.cpp — the host half of libhrt: scene-graph constructors of the C ABI, BvhNode::new,
 * bounding boxes / counts with the reference's semantics, Camera::new/resize, the tile grid and the
 * lowering of the graph into the pre-order device layout (layout.h).
 *
 * Reference semantics kept here (paths in SkillerRaptor/hyper-ray-tracer):
 *   bounding boxes   sphere.rs:78-83, moving_sphere.rs:98-110, rect.rs:88-103 (incl. the ZX box whose
 *                    x/z ranges are swapped relative to the hit test at rect.rs:57), cuboid.rs:104-106,
 *                    translation.rs:40-48, rotation.rs:41-99 (computed once over t in [0, 1]),
 *                    constant_medium.rs:78-80, list.rs:33-44, bvh_node.rs:129-131
 *   BVH build        bvh_node.rs:27-101 (longest axis, min+max key, upper half right, 1 prim/leaf)
 *   counts           hittable/.rs count() (Rotation::count == 1, rotation.rs:140-142)
 */
#include <algorithm>
#include <functional>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

#include "scene_internal.h"
#include "walk_box.h"

using namespace hrt;
using namespace hrt::host;
namespace G = hrt::gpu;

namespace hrt {
static thread_local std::string g_error;
void set_error(const std::string& msg) { g_error = msg; }
}  // namespace hrt

namespace {

struct Error : std::runtime_error {
  hrt_status code;
  Error(hrt_status c, const std::string& m) : std::runtime_error(m), code(c) {}
};

template <class F>
hrt_status guard(F&& f) {
  try {
    f();
    return HRT_OK;
  } catch (const Error& e) {
    set_error(e.what());
    return e.code;
  } catch (const std::bad_alloc&) {
    set_error("out of host memory");
    return HRT_ERR_OOM;
  } catch (const std::exception& e) {
    set_error(e.what());
    return HRT_ERR_INVALID_ARG;
  }
}

void need(bool c, hrt_status code, const char* msg) {
  if (!c) throw Error(code, msg);
}
void mutable_scene(hrt_scene* s) {
  need(s != nullptr, HRT_ERR_INVALID_ARG, "null scene");
  need(!s->committed, HRT_ERR_STATE, "scene is immutable after hrt_scene_commit");
}
void check_tex(const hrt_scene* s, uint32_t t) {
  need(t < s->texs.size(), HRT_ERR_INVALID_ARG, "bad texture id");
}
void check_mat(const hrt_scene* s, uint32_t m) {
  need(m < s->mats.size(), HRT_ERR_INVALID_ARG, "bad material id");
}
uint32_t take_child(hrt_scene* s, uint32_t c) {
  need(c < s->nodes.size(), HRT_ERR_INVALID_ARG, "bad node id");
  need(!s->nodes[c].owned, HRT_ERR_INVALID_ARG, "node already owned by another node");
  s->nodes[c].owned = true;
  return c;
}
uint32_t push_node(hrt_scene* s, HNode&& n) {
  s->nodes.push_back(std::move(n));
  return (uint32_t)(s->nodes.size() - 1);
}
Vec3 vin(const float* p) {
  need(p != nullptr, HRT_ERR_INVALID_ARG, "null vector");
  return v3(p[0], p[1], p[2]);
}

/* aabb.rs:49-63 */
Aabb surrounding(const Aabb& a, const Aabb& b) {
  return Aabb{v3(fminf(a.mn.x, b.mn.x), fminf(a.mn.y, b.mn.y), fminf(a.mn.z, b.mn.z)),
              v3(fmaxf(a.mx.x, b.mx.x), fmaxf(a.mx.y, b.mx.y), fmaxf(a.mx.z, b.mx.z))};
}

/* moving_sphere.rs:53-59 */
Vec3 moving_center(const HNode& n, float time) {
  return n.c0 + ((time - n.t0) / (n.t1 - n.t0)) * (n.c1 - n.c0);
}

bool bbox(const hrt_scene* s, uint32_t id, float t0, float t1, Aabb& out) {
  const HNode& n = s->nodes[id];
  switch (n.kind) {
    case N_SPHERE: {
      Vec3 rv = v3(n.r, n.r, n.r);
      out = Aabb{n.c0 - rv, n.c0 + rv};
      return true;
    }
    case N_MOVING: {
      Vec3 rv = v3(n.r, n.r, n.r);
      Aabb b0{moving_center(n, t0) - rv, moving_center(n, t0) + rv};
      Aabb b1{moving_center(n, t1) - rv, moving_center(n, t1) + rv};
      out = surrounding(b0, b1);
      return true;
    }
    case N_RECT:
      if (n.plane == HRT_PLANE_XY) out = Aabb{v3(n.a0, n.b0, n.k - 0.0001f), v3(n.a1, n.b1, n.k + 0.0001f)};
      else if (n.plane == HRT_PLANE_YZ) out = Aabb{v3(n.k - 0.0001f, n.a0, n.b0), v3(n.k + 0.0001f, n.a1, n.b1)};
      else out = Aabb{v3(n.a0, n.k - 0.0001f, n.b0), v3(n.a1, n.k + 0.0001f, n.b1)};
      return true;
    case N_CUBOID:
      out = n.box;
      return true;
    case N_TRANSLATE: {
      Aabb b;
      if (!bbox(s, n.children[0], t0, t1, b)) return false;
      out = Aabb{b.mn + n.disp, b.mx + n.disp};
      return true;
    }
    case N_ROTATE:
      if (!n.has_box) return false;
      out = n.box;
      return true;
    case N_MEDIUM:
      return bbox(s, n.children[0], t0, t1, out);
    case N_LIST: {
      if (n.children.empty()) return false;
      Aabb acc;
      if (!bbox(s, n.children[0], t0, t1, acc)) return false;
      for (size_t i = 1; i < n.children.size(); i++) {
        Aabb b;
        if (!bbox(s, n.children[i], t0, t1, b)) return false;
        acc = surrounding(acc, b);
      }
      out = acc;
      return true;
    }
    case N_BVH:
      out = n.box;
      return true;
  }
  return false;
}

uint32_t count(const hrt_scene* s, uint32_t id) {
  const HNode& n = s->nodes[id];
  switch (n.kind) {
    case N_SPHERE: case N_MOVING: case N_RECT: case N_ROTATE:
      return 1;
    case N_TRANSLATE: case N_MEDIUM:
      return count(s, n.children[0]);
    case N_CUBOID: case N_LIST: case N_BVH: {
      uint32_t c = 0;
      for (uint32_t ch : n.children) c += count(s, ch);
      return c;
    }
  }
  return 0;
}

/* bvh_node.rs:27-63.  Rust's sort_unstable_by is an insertion sort (stable) below 21 elements and
 * pdqsort above; a stable sort reproduces the former exactly and fixes an order for key ties in the
 * latter (closest hits do not depend on it). */
uint32_t build_bvh(hrt_scene* s, std::vector<uint32_t> objects, float t0, float t1) {
  need(!objects.empty(), HRT_ERR_EMPTY, "no elements in scene (BvhNode::new with no objects)");
  /* moving-sphere boxes cover [t0, t1] only: remember the shutter every BVH box is valid for */
  s->box_t0 = std::max(s->box_t0, t0);
  s->box_t1 = std::min(s->box_t1, t1);
  float ranges[3];
  for (int a = 0; a < 3; a++) {
    float mn = 3.40282347e+38f, mx = -3.40282347e+38f;
    for (uint32_t o : objects) {
      Aabb b;
      if (!bbox(s, o, t0, t1, b)) continue;
      mn = fminf(mn, b.mn[a]);
      mx = fmaxf(mx, b.mx[a]);
    }
    ranges[a] = mx - mn;
    need(ranges[a] == ranges[a], HRT_ERR_NAN, "NaN axis range in BVH build");
  }
  int order[3] = {0, 1, 2};
  std::stable_sort(order, order + 3, [&](int a, int b) { return ranges[a] > ranges[b]; });
  int axis = order[0];
  std::vector<std::pair<float, uint32_t>> keys;
  keys.reserve(objects.size());
  for (uint32_t o : objects) {
    Aabb b;
    need(bbox(s, o, t0, t1, b), HRT_ERR_NO_BBOX, "object without bounding box inside a BVH");
    float key = b.mn[axis] + b.mx[axis];
    need(key == key, HRT_ERR_NAN, "NaN bounding box inside a BVH");
    keys.emplace_back(key, o);
  }
  std::stable_sort(keys.begin(), keys.end(),
                   [](const std::pair<float, uint32_t>& a, const std::pair<float, uint32_t>& b) {
                     return a.first < b.first;
                   });
  /* hrt_scene_options.bvh_ties = 1 (diagnostics): sorts of more than 20 objects put equal keys in the reverse
   * order, another order Rust's pdqsort could produce; tests/test_gpu_configs.py renders both trees to
   * show what the unpinned tie order changes (hrt_scene_info.bvh_tied_sorts) */
  if (s->opts.bvh_ties == 1 && keys.size() > 20)
    for (size_t i = 0; i < keys.size();) {
      size_t j = i + 1;
      while (j < keys.size() && keys[j].first == keys[i].first) j++;
      std::reverse(keys.begin() + i, keys.begin() + j);
      i = j;
    }
  if (keys.size() > 20)
    for (size_t i = 1; i < keys.size(); i++)
      if (keys[i].first == keys[i - 1].first) {
        s->bvh_tied_sorts++;
        break;
      }
  HNode n;
  n.kind = N_BVH;
  n.has_box = true;
  size_t len = keys.size();
  if (len == 1) {
    n.children.push_back(keys[0].second);
    need(bbox(s, keys[0].second, t0, t1, n.box), HRT_ERR_NO_BBOX, "object without bounding box");
    return push_node(s, std::move(n));
  }
  std::vector<uint32_t> lower, upper;
  for (size_t i = 0; i < len; i++) (i < len / 2 ? lower : upper).push_back(keys[i].second);
  uint32_t right = build_bvh(s, std::move(upper), t0, t1);
  uint32_t left = build_bvh(s, std::move(lower), t0, t1);
  n.box = surrounding(s->nodes[left].box, s->nodes[right].box);
  n.children = {left, right};
  for (uint32_t c : n.children) s->nodes[c].owned = true;
  return push_node(s, std::move(n));
}

/* Does the reference bounding box of `id` contain its geometry?  Only a ZX rect with a0..a1 != b0..b1
 * breaks this (rect.rs:97-102 vs :57), directly or through the boxes that enclose it. */
bool box_ok(const hrt_scene* s, uint32_t id) {
  const HNode& n = s->nodes[id];
  switch (n.kind) {
    case N_RECT:
      return n.plane != HRT_PLANE_ZX || (n.a0 == n.b0 && n.a1 == n.b1);
    case N_CUBOID: case N_SPHERE: case N_MOVING:
      return true;
    default:
      for (uint32_t c : n.children)
        if (!box_ok(s, c)) return false;
      return true;
  }
}

/* ------------------------------------------------------------------ lowering (commit) */
struct Flattener {
  hrt_scene* s;
  struct PendingMedium {
    uint32_t medium;
    uint32_t boundary;
  };
  std::vector<PendingMedium> pending;
  bool in_boundary = false;
  int inst_depth = 0, max_inst_depth = 0;

  uint32_t emit_node(uint32_t kind, uint32_t payload, const Aabb* box) {
    G::Node g;
    memset(&g, 0, sizeof(g));
    if (box) {
      for (int a = 0; a < 3; a++) {
        g.mn[a] = box->mn[a];
        g.mx[a] = box->mx[a];
      }
    }
    g.kp = (kind << 24) | payload;
    g.skip = (uint32_t)s->g_nodes.size() + 1;
    need(payload < (1u << 24), HRT_ERR_UNSUPPORTED, "scene too large (payload > 2^24)");
    s->g_nodes.push_back(g);
    return (uint32_t)(s->g_nodes.size() - 1);
  }

  uint32_t emit_prim(uint32_t id, uint32_t parent) {
    const HNode& n = s->nodes[id];
    G::Prim p;
    memset(&p, 0, sizeof(p));
    p.parent = parent;
    uint32_t kind = 0;
    if (n.kind == N_SPHERE) {
      kind = G::P_SPHERE;
      p.p0[0] = n.c0.x; p.p0[1] = n.c0.y; p.p0[2] = n.c0.z; p.p0[3] = n.r;
    } else if (n.kind == N_MOVING) {
      kind = G::P_MOVING;
      s->feature_mask |= G::F_MOVING;
      Vec3 dc = n.c1 - n.c0;
      p.p0[0] = n.c0.x; p.p0[1] = n.c0.y; p.p0[2] = n.c0.z; p.p0[3] = n.r;
      p.p1[0] = dc.x; p.p1[1] = dc.y; p.p1[2] = dc.z; p.p1[3] = n.t0;
      p.p2[0] = n.t1 - n.t0;
    } else {
      kind = G::P_RECT;
      s->feature_mask |= G::F_RECT;
      p.p0[0] = n.a0; p.p0[1] = n.a1; p.p0[2] = n.b0; p.p0[3] = n.b1;
      p.p1[0] = n.k; p.p1[1] = n.a1 - n.a0; p.p1[2] = n.b1 - n.b0;
    }
    need(n.mat < (1u << 27), HRT_ERR_UNSUPPORTED, "too many materials");
    p.km = kind | ((uint32_t)n.plane << 2) | (n.mat << 4);
    s->g_prims.push_back(p);
    return (uint32_t)(s->g_prims.size() - 1);
  }

  static bool is_prim(NodeKind k) { return k == N_SPHERE || k == N_MOVING || k == N_RECT; }

  void emit(uint32_t id, uint32_t parent) {
    const HNode& n = s->nodes[id];
    switch (n.kind) {
      case N_BVH: {
        const bool ok = box_ok(s, id);
        if (!ok) s->all_boxes_ok = false;
        if (n.children.size() == 1 && is_prim(s->nodes[n.children[0]].kind)) {
          uint32_t me = emit_node(G::K_BOX_PRIM, emit_prim(n.children[0], parent), &n.box);
          if (!ok) s->g_nodes[me].kp |= G::NODE_REF_ONLY;
          return;
        }
        uint32_t me = emit_node(G::K_BOX, 0, &n.box);
        if (!ok) s->g_nodes[me].kp |= G::NODE_REF_ONLY;
        for (uint32_t c : n.children) emit(c, parent);
        s->g_nodes[me].skip = (uint32_t)s->g_nodes.size();
        return;
      }
      case N_SPHERE: case N_MOVING: case N_RECT:
        emit_node(G::K_PRIM, emit_prim(id, parent), nullptr);
        return;
      case N_CUBOID: case N_LIST:
        for (uint32_t c : n.children) emit(c, parent);
        return;
      case N_TRANSLATE: case N_ROTATE: {
        G::Inst in;
        memset(&in, 0, sizeof(in));
        in.kind = n.kind == N_TRANSLATE ? G::I_TRANSLATE : G::I_ROTATE;
        in.d[0] = n.disp.x; in.d[1] = n.disp.y; in.d[2] = n.disp.z;
        in.sin_t = n.sin_t; in.cos_t = n.cos_t;
        in.axis = (uint32_t)n.axis;
        in.parent = parent;
        s->g_insts.push_back(in);
        uint32_t iid = (uint32_t)(s->g_insts.size() - 1);
        s->feature_mask |= G::F_INSTANCE;
        inst_depth++;
        max_inst_depth = std::max(max_inst_depth, inst_depth);
        need(inst_depth <= G::MAX_INST_DEPTH, HRT_ERR_UNSUPPORTED, "instances nested deeper than 8");
        const uint32_t first = emit_node(G::K_INST_BEGIN, iid, nullptr) + 1;
        emit(n.children[0], iid);
        emit_node(G::K_INST_END, iid, nullptr);
        /* what the subtree reads of the ray beyond o, d (layout.h IF_*) */
        for (uint32_t i = first; i + 1 < (uint32_t)s->g_nodes.size(); i++) {
          const uint32_t kp = s->g_nodes[i].kp, k = (kp >> 24) & G::KIND_MASK;
          if (k == G::K_BOX || k == G::K_BOX_PRIM || k == G::K_MEDIUM) s->g_insts[iid].kind |= G::IF_INV;
          if (k == G::K_MEDIUM) s->g_insts[iid].kind |= G::IF_DD;
          if ((k == G::K_BOX_PRIM || k == G::K_PRIM) && (s->g_prims[kp & 0xFFFFFFu].km & 3u) != G::P_RECT)
            s->g_insts[iid].kind |= G::IF_DD;
        }
        inst_depth--;
        return;
      }
      case N_MEDIUM: {
        need(!in_boundary, HRT_ERR_UNSUPPORTED, "ConstantMedium inside a medium boundary");
        G::Medium m;
        memset(&m, 0, sizeof(m));
        m.neg_inv_density = n.neg_inv_density;
        m.medium_id = n.medium_id;
        m.parent = parent;
        /* the Isotropic phase function is a material of its own (constant_medium.rs:28) */
        G::Mat gm;
        memset(&gm, 0, sizeof(gm));
        gm.kind = G::M_ISOTROPIC;
        gm.tex = n.tex;
        gm.needs_uv = 0;
        m.mat = (uint32_t)s->g_mats.size();
        s->g_mats.push_back(gm);
        s->g_media.push_back(m);
        uint32_t mid = (uint32_t)(s->g_media.size() - 1);
        s->feature_mask |= G::F_MEDIUM | G::F_ISOTROPIC;
        emit_node(G::K_MEDIUM, mid, nullptr);
        pending.push_back({mid, n.children[0]});
        return;
      }
    }
  }
};

bool tex_needs_uv(const hrt_scene* s, uint32_t t, int depth = 0) {
  if (depth > 64) return true;
  const HTex& x = s->texs[t];
  if (x.kind == G::T_IMAGE) return true;
  if (x.kind == G::T_CHECKER) return tex_needs_uv(s, x.odd, depth + 1) || tex_needs_uv(s, x.even, depth + 1);
  return false;
}

uint32_t tex_features(const hrt_scene* s, uint32_t t, int depth = 0) {
  if (depth > 64) throw Error(HRT_ERR_INVALID_ARG, "texture cycle");
  const HTex& x = s->texs[t];
  if (x.kind == G::T_NOISE) return G::F_NOISE;
  if (x.kind == G::T_IMAGE) return G::F_IMAGE;
  if (x.kind == G::T_CHECKER)
    return G::F_CHECKER | tex_features(s, x.odd, depth + 1) | tex_features(s, x.even, depth + 1);
  return 0;
}

/* ------------------------------------------------------------------ SAH fast path (f4) */
/* For sphere-only scenes the closest hit does not depend on the BVH (only exact
 * equal-t ties could), so the device may traverse a better tree than BvhNode::new's median split:
 * binned SAH, <= LEAF_MAX primitives per leaf, emitted as 8 stackless pre-order streams, one per ray
 * direction octant, each visiting the near child (by the node's split axis) first. */
struct SahNode {
  Aabb box;
  int axis = 0;
  int left = -1, right = -1;
  uint32_t start = 0, count = 0; /* leaf */
};

struct SahBuilder {
  std::vector<Aabb> boxes;
  std::vector<Vec3> cent;
  std::vector<uint32_t> order;
  std::vector<SahNode> nodes;

  static float area(const Aabb& b) {
    Vec3 d = b.mx - b.mn;
    return 2.0f * (d.x * d.y + d.y * d.z + d.z * d.x);
  }
  int build(uint32_t begin, uint32_t end) {
    SahNode n;
    Aabb bb = boxes[order[begin]];
    Vec3 cmn = cent[order[begin]], cmx = cmn;
    for (uint32_t i = begin; i < end; i++) {
      bb = surrounding(bb, boxes[order[i]]);
      Vec3 c = cent[order[i]];
      for (int a = 0; a < 3; a++) { cmn[a] = std::min(cmn[a], c[a]); cmx[a] = std::max(cmx[a], c[a]); }
    }
    n.box = bb;
    const uint32_t cnt = end - begin;
    const float C_TRAV = 1.0f, C_ISECT = 2.0f;
    float best = cnt * C_ISECT;
    int best_axis = -1, best_bin = -1;
    const int NB = 16;
    if (cnt > 1) {
      for (int a = 0; a < 3; a++) {
        float ext = cmx[a] - cmn[a];
        if (!(ext > 0.0f)) continue;
        Aabb bbox[NB];
        uint32_t bcnt[NB] = {0};
        for (uint32_t i = begin; i < end; i++) {
          int b = std::min(NB - 1, (int)((cent[order[i]][a] - cmn[a]) / ext * NB));
          bbox[b] = bcnt[b] ? surrounding(bbox[b], boxes[order[i]]) : boxes[order[i]];
          bcnt[b]++;
        }
        Aabb racc[NB];
        uint32_t rn[NB];
        Aabb acc;
        uint32_t accn = 0;
        for (int b = NB - 1; b >= 1; b--) {
          if (bcnt[b]) { acc = accn ? surrounding(acc, bbox[b]) : bbox[b]; accn += bcnt[b]; }
          racc[b] = acc;
          rn[b] = accn;
        }
        Aabb lacc;
        uint32_t ln = 0;
        for (int b = 0; b < NB - 1; b++) {
          if (bcnt[b]) { lacc = ln ? surrounding(lacc, bbox[b]) : bbox[b]; ln += bcnt[b]; }
          if (ln == 0 || rn[b + 1] == 0) continue;
          float cost = C_TRAV + C_ISECT * (area(lacc) * ln + area(racc[b + 1]) * rn[b + 1]) / std::max(area(bb), 1e-30f);
          if (cost < best) { best = cost; best_axis = a; best_bin = b; }
        }
      }
    }
    if (best_axis < 0 && cnt <= gpu::LEAF_MAX) {
      n.start = begin;
      n.count = cnt;
      nodes.push_back(n);
      return (int)nodes.size() - 1;
    }
    uint32_t mid;
    if (best_axis >= 0) {
      float ext = cmx[best_axis] - cmn[best_axis];
      auto it = std::stable_partition(order.begin() + begin, order.begin() + end, [&](uint32_t p) {
        int b = std::min(NB - 1, (int)((cent[p][best_axis] - cmn[best_axis]) / ext * NB));
        return b <= best_bin;
      });
      mid = (uint32_t)(it - order.begin());
      n.axis = best_axis;
    } else { /* identical centroids: split by count along the widest box axis */
      Vec3 d = bb.mx - bb.mn;
      n.axis = (d.x >= d.y && d.x >= d.z) ? 0 : (d.y >= d.z ? 1 : 2);
      mid = begin + cnt / 2;
    }
    if (mid == begin || mid == end) mid = begin + cnt / 2;
    nodes.push_back(n);
    int me = (int)nodes.size() - 1;
    int l = build(begin, mid);
    int r = build(mid, end);
    nodes[me].left = l;
    nodes[me].right = r;
    return me;
  }
};

void emit_stream(hrt_scene* s, const SahBuilder& B, int ni, int octant, uint32_t base) {
  const SahNode& n = B.nodes[ni];
  G::Node g;
  memset(&g, 0, sizeof(g));
  for (int a = 0; a < 3; a++) { g.mn[a] = n.box.mn[a]; g.mx[a] = n.box.mx[a]; }
  uint32_t me = (uint32_t)s->f_nodes.size();
  if (n.left < 0) {
    g.kp = (G::K_BOX_LEAF << 24) | n.start | ((n.count - 1) << 21);
    g.skip = me + 1;
    s->f_nodes.push_back(g);
    return;
  }
  g.kp = G::K_BOX << 24;
  s->f_nodes.push_back(g);
  bool neg = (octant >> n.axis) & 1;
  emit_stream(s, B, neg ? n.right : n.left, octant, base);
  emit_stream(s, B, neg ? n.left : n.right, octant, base);
  s->f_nodes[me].skip = (uint32_t)s->f_nodes.size();
}

void build_fast(hrt_scene* s) {
  s->f_nodes.clear();
  s->f_prims.clear();
  s->f_stream_len = 0;
  const size_t np = s->g_prims.size();
  if (np == 0 || np >= (1u << 21)) return;
  SahBuilder B;
  for (size_t i = 0; i < np; i++) {
    const G::Prim& p = s->g_prims[i];
    Vec3 c0 = v3(p.p0[0], p.p0[1], p.p0[2]);
    Vec3 rv = v3(p.p0[3], p.p0[3], p.p0[3]);
    Aabb b{c0 - rv, c0 + rv};
    if ((p.km & 3u) == G::P_MOVING) { /* box over the BVH build interval [0, 1] (application.rs builders) */
      Vec3 dc = v3(p.p1[0], p.p1[1], p.p1[2]);
      Vec3 ca = c0 + ((0.0f - p.p1[3]) / p.p2[0]) * dc, cb = c0 + ((1.0f - p.p1[3]) / p.p2[0]) * dc;
      b = surrounding(Aabb{ca - rv, ca + rv}, Aabb{cb - rv, cb + rv});
    }
    for (int a = 0; a < 3; a++)
      if (!(b.mn[a] <= b.mx[a])) return; /* NaN / inverted: keep the reference traversal */
    B.boxes.push_back(b);
    B.cent.push_back((b.mn + b.mx) * 0.5f);
    B.order.push_back((uint32_t)i);
  }
  int root = B.build(0, (uint32_t)np);
  for (uint32_t i = 0; i < np; i++) s->f_prims.push_back(s->g_prims[B.order[i]]);
  for (int o = 0; o < 8; o++) {
    uint32_t base = (uint32_t)s->f_nodes.size();
    emit_stream(s, B, root, o, base);
    if (o == 0) s->f_stream_len = (uint32_t)s->f_nodes.size();
  }
}

/* ------------------------------------------------------------------ sphere-scene walk stream */
/* layout.h "sphere-scene walk stream": the records render_basic_kernel walks under CULL_EXACT.
 *
 * The leaves are the reference stream's leaves (K_BOX_PRIM: a BvhNode leaf, K_PRIM: a List member) in
 * the reference's pre-order, so the walk tests the same primitives in the same order as BvhNode::hit
 * (bvh_node.rs:104-127).  Above them, by default (hrt_scene_options.walk_tree = 0), the inner boxes are
 * RE-GROUPED: a top-down surface-area split of the fixed leaf sequence (each range cut where
 * SA(left) n_left + SA(right) n_right is least).  The reference's own hierarchy splits on the longest
 * axis of its node's box, which the r = 1000 ground sphere makes the y axis at every level that holds
 * it, so its upper levels group spheres by height and every ray passes a chain of ground-sized boxes;
 * the re-grouped tree puts the ground sphere alone under the root (64.4 -> ~53 node visits per ray on
 * Random in a host simulation).  Any hierarchy over the same leaf sequence whose boxes hold their
 * leaves' boxes gives the reference's result.  The reference hierarchy itself is
 * kept (walk_tree = 1) for A/B, and whenever a leaf has no box or a box that is not a finite
 * well-formed interval. */
/* walk_box.h ce_floored on an Aabb */
bool box_ce_floored(const Aabb& bx, float* C, float* E, Aabb* fb) {
  const float mn[3] = {bx.mn.x, bx.mn.y, bx.mn.z}, mx[3] = {bx.mx.x, bx.mx.y, bx.mx.z};
  float fmn[3], fmx[3];
  const bool raised = walkbox::ce_floored(mn, mx, C, E, fmn, fmx);
  fb->mn = v3(fmn[0], fmn[1], fmn[2]);
  fb->mx = v3(fmx[0], fmx[1], fmx[2]);
  return raised;
}

double half_area(const Aabb& b) {
  const double x = (double)b.mx.x - b.mn.x, y = (double)b.mx.y - b.mn.y, z = (double)b.mx.z - b.mn.z;
  return x * y + y * z + z * x;
}

Aabb box_union(const Aabb& a, const Aabb& b) {
  Aabb u;
  u.mn = v3(fminf(a.mn.x, b.mn.x), fminf(a.mn.y, b.mn.y), fminf(a.mn.z, b.mn.z));
  u.mx = v3(fmaxf(a.mx.x, b.mx.x), fmaxf(a.mx.y, b.mx.y), fmaxf(a.mx.z, b.mx.z));
  return u;
}

/* ---- hrt_scene_set_view: what the hierarchy builders use of the view (performance only: any hierarchy over
 * the reference leaf order, placed anywhere, renders the same image, DESIGN.md sections 4-5) */
/* f64 slab test of b on [lo, hi]; an axis whose product is NaN (0 x inf: the origin on a slab plane) is skipped.
 * On a hit, *entry = the t where the ray enters the box, or -inf when its origin lies inside (a leaf box around
 * the camera, such as Final's fog, stops no ray).  For nested boxes the outcome is monotone (a superset passes
 * whenever a subset does: rounding is monotone). */
static bool view_slab(const Aabb& b, const double* o, const double* inv, double lo, double hi, double* entry = nullptr) {
  double in = -HUGE_VAL;
  for (int k = 0; k < 3; k++) {
    const double t0 = (b.mn[k] - o[k]) * inv[k], t1 = (b.mx[k] - o[k]) * inv[k];
    const double a = std::min(t0, t1), c = std::max(t0, t1);
    if (a == a) in = std::max(in, a);
    if (c == c) hi = std::min(hi, c);
  }
  lo = std::max(lo, in);
  if (entry) *entry = in > 0.0 ? in : -HUGE_VAL;
  return lo <= hi;
}
/* a pinhole camera ray through (u, v) of the view's image plane (lens and shutter ignored) */
static void view_ray(const hrt_camera& c, double u, double v, double* o, double* inv) {
  for (int k = 0; k < 3; k++) {
    o[k] = c.origin[k];
    inv[k] = 1.0 / ((double)c.lower_left_corner[k] + u * c.horizontal[k] + v * c.vertical[k] - o[k]);
  }
}
constexpr double VIEW_TMIN = 0.001;
/* camera rays through a VIEW_DP_GRID x VIEW_DP_GRID grid, each stopped at the nearest leaf box it enters (a
 * stand-in for its closest hit that needs no primitive code) */
constexpr uint32_t VIEW_DP_GRID = 64;
struct ViewRays {
  std::vector<double> o, inv, cl;
  uint32_t n = 0;
};
static ViewRays view_rays(const hrt_camera& c, const std::vector<WalkLeaf>& leaves) {
  ViewRays R;
  R.n = VIEW_DP_GRID * VIEW_DP_GRID;
  R.o.resize(3 * (size_t)R.n);
  R.inv.resize(3 * (size_t)R.n);
  R.cl.assign(R.n, HUGE_VAL);
  for (uint32_t q = 0; q < R.n; q++) {
    view_ray(c, (q % VIEW_DP_GRID + 0.5) / VIEW_DP_GRID, (q / VIEW_DP_GRID + 0.5) / VIEW_DP_GRID, &R.o[3 * q], &R.inv[3 * q]);
    for (const WalkLeaf& L : leaves) {
      double t;
      if (view_slab(L.box, &R.o[3 * q], &R.inv[3 * q], VIEW_TMIN, R.cl[q], &t) && t > VIEW_TMIN) R.cl[q] = t;
    }
  }
  return R;
}
/* the share of the re-grouping DP's node cost given to the view's rays (the rest: surface area, for the
 * scattered rays; priced flat between 0.35 and 0.6 on C2, scripts/price_hierarchy.py) */
constexpr double VIEW_DP_MIX = 0.5;

/* Optimal re-grouping of a fixed leaf sequence by dynamic programming (HRT_WALK_DP = 1 | 2, n <= 2048):
 * cost(i, j) = w(i, j) + min_k cost(i, k) + cost(k, j) over the ranges of the sequence, with w = 2 x the half
 * area (mode 1: the two child tests an inner node makes whenever a ray passes it) or half area x leaves
 * (mode 2: walk_regroup's greedy objective, minimised exactly).  Splits tie to the cut nearest the middle. */
/* With view rays (hrt_scene_set_view, mode 1): w(i, j) = 2 x (VIEW_DP_MIX x the share of the view's rays whose
 * slab test of the range's box passes before their closest + (1 - VIEW_DP_MIX) x half area / area_root). */
bool walk_regroup_dp(std::vector<WNode>& T, const std::vector<WalkLeaf>& all, int mode, uint32_t lo0 = 0,
                     uint32_t hi0 = 0xFFFFFFFFu, uint32_t depth0 = 0, const ViewRays* vr = nullptr,
                     double area_root = 0.0) {
  /* over the leaves [lo0, hi0) (default: all), the subtree's nodes appended to T at depth depth0 */
  if (hi0 > all.size()) hi0 = (uint32_t)all.size();
  const WalkLeaf* leaves = all.data() + lo0;
  const uint32_t n = hi0 - lo0;
  if (n < 2 || n > 2048) return false;
  std::vector<double> A((size_t)n * (n + 1), 0.0), C((size_t)n * (n + 1), 0.0);
  std::vector<uint32_t> K((size_t)n * (n + 1), 0u);
  std::vector<Aabb> box((size_t)n * (n + 1));
  auto at = [n](uint32_t i, uint32_t j) { return (size_t)i * (n + 1) + j; };
  for (uint32_t i = 0; i < n; i++) {
    Aabb u = leaves[i].box;
    box[at(i, i + 1)] = u;
    A[at(i, i + 1)] = half_area(u);
    for (uint32_t j = i + 2; j <= n; j++) {
      u = box_union(u, leaves[j - 1].box);
      box[at(i, j)] = u;
      A[at(i, j)] = half_area(u);
    }
  }
  std::vector<double> P;
  const bool view = vr != nullptr && mode == 1 && area_root > 0.0;
  if (view) {
    /* per start i, each ray's first end j whose box it passes (monotone in j: nested boxes), by bisection */
    P.assign((size_t)n * (n + 1), 0.0);
    std::vector<uint32_t> rs;
    for (uint32_t q = 0; q < vr->n; q++)
      if (view_slab(box[at(0, n)], &vr->o[3 * q], &vr->inv[3 * q], VIEW_TMIN, vr->cl[q])) rs.push_back(q);
    std::vector<uint32_t> first(n + 2);
    for (uint32_t i = 0; i < n; i++) {
      std::fill(first.begin(), first.end(), 0u);
      for (uint32_t q : rs) {
        const double* o = &vr->o[3 * q];
        const double* iv = &vr->inv[3 * q];
        if (!view_slab(box[at(i, n)], o, iv, VIEW_TMIN, vr->cl[q])) continue;
        uint32_t a = i + 1, b = n; /* the smallest j in [a, b] that passes: b does */
        while (a < b) {
          const uint32_t m = a + (b - a) / 2;
          if (view_slab(box[at(i, m)], o, iv, VIEW_TMIN, vr->cl[q])) b = m;
          else a = m + 1;
        }
        first[a]++;
      }
      uint32_t c = 0;
      for (uint32_t j = i + 1; j <= n; j++) {
        c += first[j];
        P[at(i, j)] = (double)c / vr->n;
      }
    }
  }
  for (uint32_t len = 2; len <= n; len++)
    for (uint32_t i = 0; i + len <= n; i++) {
      const uint32_t j = i + len, mid = i + len / 2;
      double best = HUGE_VAL;
      uint32_t bk = mid;
      for (uint32_t k = i + 1; k < j; k++) {
        const double c = C[at(i, k)] + C[at(k, j)];
        const uint32_t dk = k > mid ? k - mid : mid - k, db = bk > mid ? bk - mid : mid - bk;
        if (c < best || (c == best && dk < db)) {
          best = c;
          bk = k;
        }
      }
      C[at(i, j)] = best + (mode == 2 ? A[at(i, j)] * len
                                      : view ? 2.0 * (VIEW_DP_MIX * P[at(i, j)] + (1.0 - VIEW_DP_MIX) * A[at(i, j)] / area_root)
                                             : 2.0 * A[at(i, j)]);
      K[at(i, j)] = bk;
    }
  struct Range { uint32_t lo, hi, depth; };
  std::vector<Range> todo{{0u, n, depth0}};
  while (!todo.empty()) {
    const Range r = todo.back();
    todo.pop_back();
    const uint32_t m = r.hi - r.lo, self = (uint32_t)T.size();
    if (m == 1) {
      T.push_back(WNode{leaves[r.lo].box, (int32_t)(lo0 + r.lo), self + 1, r.depth});
      continue;
    }
    const uint32_t k = K[at(r.lo, r.hi)];
    T.push_back(WNode{box[at(r.lo, r.hi)], -1, self + 2 * m - 1, r.depth});
    todo.push_back({k, r.hi, r.depth + 1});
    todo.push_back({r.lo, k, r.depth + 1});
  }
  return true;
}

/* re-grouped hierarchy over leaves[0, n), iterative, pre-order (a range of n leaves is 2n - 1 nodes) */
void walk_regroup(std::vector<WNode>& T, const std::vector<WalkLeaf>& leaves, const hrt_camera* view = nullptr) {
  /* default: the DP (mode 1) for sequences of at most 700 leaves (O(n^3 / 6) work: ~30 ms at Random's 485),
   * the greedy split above that (and on the device, build_walk.hip).  With a view (hrt_scene_set_view) the
   * DP's node cost mixes in the view's camera rays (walk_regroup_dp); leaves without a box keep it off. */
  const char* dp = knob_env("HRT_WALK_DP");
  const int mode = dp ? dp[0] - '0' : (leaves.size() <= 700 ? 1 : 3);
  ViewRays vr;
  double area_root = 0.0;
  bool boxes = !leaves.empty();
  for (const WalkLeaf& L : leaves) boxes = boxes && !L.nobox;
  if (view && boxes) {
    vr = view_rays(*view, leaves);
    Aabb u = leaves[0].box;
    for (const WalkLeaf& L : leaves) u = box_union(u, L.box);
    area_root = half_area(u);
  }
  const ViewRays* vp = area_root > 0.0 ? &vr : nullptr;
  if ((mode == 1 || mode == 2) && walk_regroup_dp(T, leaves, mode, 0, 0xFFFFFFFFu, 0, vp, area_root)) return;
  /* mode 3 (default above 700 leaves): the greedy split below, and each range of at most DP_SUB leaves it
   * reaches re-grouped by the DP (mode 1) */
  const char* ds = knob_env("HRT_WALK_DP_SUB");
  const uint32_t dp_sub = mode == 3 ? (ds ? (uint32_t)atoi(ds) : 256u) : 0u;
  struct Range { uint32_t lo, hi, depth; };
  std::vector<Range> todo{{0u, (uint32_t)leaves.size(), 0u}};
  std::vector<Aabb> pre, suf;
  while (!todo.empty()) {
    const Range r = todo.back();
    todo.pop_back();
    const uint32_t n = r.hi - r.lo, self = (uint32_t)T.size();
    if (n == 1) {
      T.push_back(WNode{leaves[r.lo].box, (int32_t)r.lo, self + 1, r.depth});
      continue;
    }
    if (n <= dp_sub && walk_regroup_dp(T, leaves, 1, r.lo, r.hi, r.depth, vp, area_root)) continue;
    pre.resize(n);
    suf.resize(n);
    pre[0] = leaves[r.lo].box;
    for (uint32_t k = 1; k < n; k++) pre[k] = box_union(pre[k - 1], leaves[r.lo + k].box);
    suf[n - 1] = leaves[r.hi - 1].box;
    for (uint32_t k = n - 1; k-- > 0;) suf[k] = box_union(suf[k + 1], leaves[r.lo + k].box);
    /* cut after leaf k (left = [lo, lo+k], right = the rest); ties go to the cut nearest the middle */
    uint32_t best = (n - 1) / 2;
    double best_cost = half_area(pre[best]) * (best + 1) + half_area(suf[best + 1]) * (n - 1 - best);
    for (uint32_t k = 0; k + 1 < n; k++) {
      const double c = half_area(pre[k]) * (k + 1) + half_area(suf[k + 1]) * (n - 1 - k);
      const uint32_t dk = k > (n - 1) / 2 ? k - (n - 1) / 2 : (n - 1) / 2 - k;
      const uint32_t db = best > (n - 1) / 2 ? best - (n - 1) / 2 : (n - 1) / 2 - best;
      if (c < best_cost || (c == best_cost && dk < db)) {
        best_cost = c;
        best = k;
      }
    }
    T.push_back(WNode{pre[n - 1], -1, self + 2 * n - 1, r.depth});
    todo.push_back({r.lo + best + 1, r.hi, r.depth + 1}); /* right after left */
    todo.push_back({r.lo, r.lo + best + 1, r.depth + 1});
  }
}

void put4(std::vector<float>& o, size_t at, float a, float b, float c, float d) {
  o[at / 4] = a; o[at / 4 + 1] = b; o[at / 4 + 2] = c; o[at / 4 + 3] = d;
}

}  // namespace
namespace hrt {
void build_walk(hrt_scene* s);
}
namespace {
using hrt::build_walk;

/* The reference node stream, primitives, instances, media, materials, textures and the facts derived from them
 * (feature mask, culling mode, motion): everything but the walk streams (flatten). */
void flatten_reference(hrt_scene* s) {
  s->g_nodes.clear(); s->g_prims.clear(); s->g_insts.clear(); s->g_media.clear();
  s->g_mats.clear(); s->g_texs.clear();
  s->feature_mask = 0;
  s->all_boxes_ok = true;
  /* materials and textures first (media append their isotropic materials after these) */
  for (const HMat& m : s->mats) {
    G::Mat g;
    memset(&g, 0, sizeof(g));
    g.kind = m.kind;
    g.tex = m.tex == G::NONE ? 0 : m.tex;
    if (m.kind == G::M_METAL) {
      g.a[0] = m.albedo.x; g.a[1] = m.albedo.y; g.a[2] = m.albedo.z; g.a[3] = m.fuzz;
      s->feature_mask |= G::F_METAL;
    } else if (m.kind == G::M_DIELECTRIC) {
      g.a[0] = m.ior;
      s->feature_mask |= G::F_DIELECTRIC;
    } else {
      g.needs_uv = tex_needs_uv(s, m.tex) ? 1u : 0u;
      s->feature_mask |= tex_features(s, m.tex);
      if (m.kind == G::M_DIFFUSE_LIGHT) s->feature_mask |= G::F_LIGHT;
      if (m.kind == G::M_ISOTROPIC) s->feature_mask |= G::F_ISOTROPIC;
    }
    s->g_mats.push_back(g);
  }
  for (const HTex& t : s->texs) {
    G::Tex g;
    memset(&g, 0, sizeof(g));
    g.kind = t.kind;
    if (t.kind == G::T_SOLID) { g.a[0] = t.color.x; g.a[1] = t.color.y; g.a[2] = t.color.z; }
    else if (t.kind == G::T_CHECKER) { g.i0 = t.odd; g.i1 = t.even; }
    else if (t.kind == G::T_NOISE) { g.a[0] = t.scale; g.i0 = t.perlin; }
    else { g.i0 = (uint32_t)t.img_off; g.i1 = t.w; g.i2 = t.h; g.i3 = t.c; }
    s->g_texs.push_back(g);
  }
  Flattener f{s, {}, false, 0, 0};
  f.emit(s->root, G::NONE);
  s->main_end = (uint32_t)s->g_nodes.size();
  f.in_boundary = true;
  for (size_t i = 0; i < f.pending.size(); i++) {
    uint32_t bstart = (uint32_t)s->g_nodes.size();
    f.emit(f.pending[i].boundary, G::NONE);
    s->g_media[f.pending[i].medium].bstart = bstart;
    s->g_media[f.pending[i].medium].bend = (uint32_t)s->g_nodes.size();
    G::Medium& gm = s->g_media[f.pending[i].medium];
    gm.sphere = G::NONE;
    if (gm.bend == gm.bstart + 1) {
      const uint32_t kp = s->g_nodes[gm.bstart].kp;
      if (((kp >> 24) & G::KIND_MASK) == G::K_PRIM && (s->g_prims[kp & 0xFFFFFFu].km & 3u) != G::P_RECT)
        gm.sphere = kp & 0xFFFFFFu;
    }
  }
  for (const G::Medium& m : s->g_media) s->feature_mask |= tex_features(s, s->g_mats[m.mat].tex);
  /* every instance's chain, outermost first (layout.h CHAIN_F4) */
  s->g_chains.assign(s->g_insts.size() * G::CHAIN_F4 * 4, 0.0f);
  for (uint32_t q = 0; q < (uint32_t)s->g_insts.size(); q++) {
    std::vector<uint32_t> ids;
    for (uint32_t x = q; x != G::NONE; x = s->g_insts[x].parent) ids.push_back(x);
    need(ids.size() <= G::MAX_INST_DEPTH, HRT_ERR_UNSUPPORTED, "instances nested deeper than 8");
    float* c = &s->g_chains[(size_t)q * G::CHAIN_F4 * 4];
    c[0] = u2f((uint32_t)ids.size());
    for (size_t l = 0; l < ids.size(); l++) {
      const G::Inst& in = s->g_insts[ids[ids.size() - 1 - l]];
      float* v = c + 4 * (1 + l);
      if ((in.kind & G::I_KIND_MASK) == G::I_TRANSLATE) {
        v[0] = in.d[0]; v[1] = in.d[1]; v[2] = in.d[2]; v[3] = u2f(G::I_TRANSLATE);
      } else {
        v[0] = in.sin_t; v[1] = in.cos_t; v[2] = u2f(in.axis); v[3] = u2f(G::I_ROTATE);
      }
    }
  }
  /* Default culling: the reference's per-axis test AND the provably safe inflated slab test
   * (layout.h CULL_EXACT; boxes that may not hold their geometry are flagged NODE_REF_ONLY). */
  s->cull_mode = G::CULL_EXACT;
  s->ln_e = ln_f(E_F);
  /* moving_sphere.rs:55-58 divides by (time1 - time0) per call; when every moving sphere has the
   * same time0 and time1 (all reference scenes) the quotient depends on the ray only */
  s->motion_uniform = true;
  bool first = true;
  for (const G::Prim& p : s->g_prims) {
    if ((p.km & 3u) != G::P_MOVING) continue;
    if (first) {
      s->motion_t0 = p.p1[3];
      s->motion_span = p.p2[0];
      first = false;
    } else if (memcmp(&s->motion_t0, &p.p1[3], 4) != 0 || memcmp(&s->motion_span, &p.p2[0], 4) != 0) {
      s->motion_uniform = false;
    }
  }
  if (first) s->motion_uniform = false; /* no moving sphere */
  s->media_nested = false;
  for (const G::Medium& m : s->g_media) s->media_nested |= m.parent != G::NONE;
}

void flatten(hrt_scene* s) {
  flatten_reference(s);
  const bool sphere_only = (s->feature_mask & (G::F_RECT | G::F_INSTANCE | G::F_MEDIUM)) == 0;
  s->f_nodes.clear();
  s->f_prims.clear();
  s->f_stream_len = 0;
  if (sphere_only && (s->feature_mask & ~G::F_BASIC) == 0) build_fast(s); /* opt-in approximate path */
  build_walk(s);
}

}  // namespace


namespace hrt {
/* ---- 16-B node parts (layout.h WALK_C16) ----
 * IEEE binary16 of a finite double: round to nearest even (up = false) or towards +inf (up = true, x >= 0).
 * Returns false when the value does not fit (|x| > 65504 after rounding). */
static bool half_round(double x, bool up, uint16_t& bits, double& value) {
  const double ax = fabs(x);
  if (!(ax <= 65504.0)) return false;
  if (ax == 0.0) {
    bits = std::signbit(x) ? 0x8000u : 0u;
    value = 0.0;
    return true;
  }
  int e = (int)floor(log2(ax));
  if (ldexp(1.0, e) > ax) e--; /* log2 rounding */
  if (ldexp(1.0, e + 1) <= ax) e++;
  if (e < -14) e = -14; /* subnormals share the smallest exponent's ulp */
  const double ulp = ldexp(1.0, e - 10);
  double q = ax / ulp; /* exact: a power-of-two scaling */
  q = up ? (x >= 0 ? ceil(q) : floor(q)) : nearbyint(q);
  double v = q * ulp;
  if (!(v <= 65504.0)) return false;
  /* bits of the exactly representable v */
  uint32_t b;
  if (v < ldexp(1.0, -14)) b = (uint32_t)(v / ldexp(1.0, -24)); /* subnormal */
  else {
    int ve = (int)floor(log2(v));
    if (ldexp(1.0, ve) > v) ve--;
    if (ldexp(1.0, ve + 1) <= v) ve++;
    const uint32_t mant = (uint32_t)(v / ldexp(1.0, ve - 10)) - 1024u;
    b = (uint32_t)(ve + 15) << 10 | mant;
  }
  bits = (uint16_t)(b | (x < 0 ? 0x8000u : 0u));
  value = x < 0 ? -v : v;
  return true;
}

/* Transcode a finished hybrid sphere stream (32-B node parts densely in [0, 32 N), the payloads behind them)
 * into 16-B node parts (layout.h WALK_C16): per node (C, E) as binary16 -- C rounded to nearest, E rounded UP,
 * so [C' - E', C' + E'] holds the 32-B part's box [C - E, C + E] and therefore the node's geometry, which is
 * all the inflated test needs (any boxes holding their leaves), with CE_FLOOR kept on the
 * rounded values.  Children first: an inner node's encoded box also holds its children's ENCODED boxes, so
 * inclusion stays monotone as in the 32-B stream (every hierarchy over the same leaves then culls the same
 * leaves).  The links become 16-bit node indices (pass of a leaf: WALK_C16_LEAF | its payload index); the
 * payloads move down by 16 N bytes and their successor fields become node indices.  Left as it is when a scene
 * does not fit the format (more than WALK_C16_MAX nodes or leaves, coordinates beyond binary16's range). */
void walk_transcode_c16(hrt_scene* s, uint32_t N) {
  const uint32_t END = s->w_end, NB = 32u * N, PB = G::WALK_PAYLOAD_BYTES;
  if (N == 0 || N > G::WALK_C16_MAX || END < NB || (END - NB) % PB != 0 || (END - NB) / PB > G::WALK_C16_MAX) return;
  const std::vector<float>& o = s->w_stream;
  auto unit = [&](uint32_t off) -> uint32_t { return off == END ? N : off / 32u; };
  std::vector<uint32_t> packed((size_t)N * 4);
  std::vector<double> lo((size_t)N * 3), hi((size_t)N * 3); /* each node's encoded box */
  std::vector<char> done(N, 0), inf_box(N, 0);
  bool ok = true;
  /* post-order from the root (node 0): children = pass, and the first child's skip */
  std::function<void(uint32_t, int)> enc = [&](uint32_t j, int depth) {
    if (!ok) return;
    if (j >= N || done[j] || depth > 200) {
      ok = false;
      return;
    }
    const float* a = &o[(size_t)j * 8];
    const float* b = a + 4;
    const uint32_t skip = f2u(a[3]), pass = f2u(b[3]);
    double L[3], H[3];
    bool inf = false;
    for (int k = 0; k < 3; k++) {
      if (b[k] == HUGE_VALF) inf = true;
      L[k] = (double)a[k] - (double)b[k];
      H[k] = (double)a[k] + (double)b[k];
    }
    uint32_t pu;
    if (pass & G::WALK_PEND) {
      const uint32_t q = pass & ~G::WALK_PEND;
      if (q < NB || (q - NB) % PB != 0) {
        ok = false;
        return;
      }
      pu = G::WALK_C16_LEAF | (q - NB) / PB;
    } else {
      if (pass >= NB || pass % 32u != 0) {
        ok = false;
        return;
      }
      const uint32_t c0 = pass / 32u;
      enc(c0, depth + 1);
      if (!ok) return;
      const uint32_t s0 = f2u(o[(size_t)c0 * 8 + 3]);
      if (s0 >= NB || s0 % 32u != 0) {
        ok = false;
        return;
      }
      const uint32_t c1 = s0 / 32u;
      enc(c1, depth + 1);
      if (!ok) return;
      for (uint32_t c : {c0, c1}) {
        inf = inf || inf_box[c];
        for (int k = 0; k < 3; k++) {
          L[k] = std::min(L[k], lo[(size_t)c * 3 + k]);
          H[k] = std::max(H[k], hi[(size_t)c * 3 + k]);
        }
      }
      pu = c0;
    }
    if (skip != END && (skip >= NB || skip % 32u != 0)) {
      ok = false;
      return;
    }
    uint16_t hc[3] = {0, 0, 0}, he[3] = {0x7C00u, 0x7C00u, 0x7C00u}; /* a box-less leaf: C = 0, E = +inf */
    double cv[3] = {0, 0, 0}, ev[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL};
    if (!inf) {
      double cmax = 0.0, emax = 0.0;
      for (int k = 0; k < 3; k++) {
        if (!half_round(0.5 * (L[k] + H[k]), false, hc[k], cv[k]) ||
            !half_round(std::max(cv[k] - L[k], H[k] - cv[k]), true, he[k], ev[k])) {
          ok = false;
          return;
        }
        cmax = std::max(cmax, fabs(cv[k]));
        emax = std::max(emax, ev[k]);
      }
      if (emax < ldexp(cmax, -12)) /* CE_FLOOR on the encoded box (walk_box.h) */
        for (int k = 0; k < 3; k++)
          if (ev[k] < ldexp(cmax, -12) && !half_round(ldexp(cmax, -12), true, he[k], ev[k])) {
            ok = false;
            return;
          }
    }
    for (int k = 0; k < 3; k++) {
      lo[(size_t)j * 3 + k] = cv[k] - ev[k];
      hi[(size_t)j * 3 + k] = cv[k] + ev[k];
    }
    inf_box[j] = inf;
    done[j] = 1;
    packed[(size_t)j * 4 + 0] = (uint32_t)hc[0] | (uint32_t)hc[1] << 16;
    packed[(size_t)j * 4 + 1] = (uint32_t)hc[2] | (uint32_t)he[0] << 16;
    packed[(size_t)j * 4 + 2] = (uint32_t)he[1] | (uint32_t)he[2] << 16;
    packed[(size_t)j * 4 + 3] = unit(skip) | pu << 16;
  };
  enc(0u, 0);
  for (uint32_t j = 0; ok && j < N; j++) ok = done[j] != 0; /* every node part reached from the root */
  if (!ok) return;
  const uint32_t n_leaf = (END - NB) / PB, pbase = 16u * N;
  std::vector<float> t((size_t)(pbase + n_leaf * PB) / 4, 0.0f);
  for (size_t k = 0; k < packed.size(); k++) t[k] = u2f(packed[k]);
  for (uint32_t l = 0; l < n_leaf; l++) {
    const float* src = &o[(size_t)(NB + l * PB) / 4];
    float* dst = &t[(size_t)(pbase + l * PB) / 4];
    std::copy(src, src + PB / 4, dst);
    const uint32_t w = f2u(dst[3]); /* flags | successor << 2 */
    const uint32_t succ = w >> 2;
    if (succ != END && (succ >= NB || succ % 32u != 0)) return;
    dst[3] = u2f((w & 3u) | unit(succ) << 2);
  }
  s->w_stream.swap(t);
  s->w_end = pbase + n_leaf * PB;
  s->w_hot /= 2; /* the staged node parts at half the bytes */
  s->w_c16 = true;
  s->w_pbase = pbase;
}

/* How often camera rays through a VIEW_GRID x VIEW_GRID grid of the view's image plane (pinhole: lens and
 * shutter ignored) visit each node of the walk hierarchy T (pre-order, T[i].end one past i's subtree), walked
 * with T's boxes in f64 and stopped at the nearest LEAF BOX entered so far (a stand-in for the closest hit
 * that needs no primitive code).  The placement's ranking only: any ranking gives the same image. */
constexpr uint32_t VIEW_GRID = 128;
static std::vector<uint32_t> view_heat(const hrt_camera& c, const std::vector<WNode>& T) {
  const uint32_t N = (uint32_t)T.size();
  std::vector<uint32_t> heat(N, 0);
  for (uint32_t gy = 0; gy < VIEW_GRID; gy++)
    for (uint32_t gx = 0; gx < VIEW_GRID; gx++) {
      double o[3], inv[3];
      view_ray(c, (gx + 0.5) / VIEW_GRID, (gy + 0.5) / VIEW_GRID, o, inv);
      double closest = HUGE_VAL;
      for (uint32_t i = 0; i < N;) {
        heat[i]++;
        double t;
        if (view_slab(T[i].box, o, inv, VIEW_TMIN, closest, &t)) {
          if (T[i].leaf >= 0 && t > VIEW_TMIN) closest = std::min(closest, t);
          i++;
        } else {
          i = T[i].end;
        }
      }
    }
  return heat;
}

/* c16: a hybrid sphere stream is laid out for 16-B node parts: twice the node parts selected for the staged
 * set, then transcoded (walk_transcode_c16).  Returns false when that was asked for and could not be done
 * (the caller lays the stream out again without it). */
static bool walk_place_and_write_impl(hrt_scene* s, const std::vector<WNode>& T, const std::vector<WalkLeaf>& leaves,
                                      bool c16) {
  const uint32_t N = (uint32_t)T.size();
  uint64_t total = 0;
  const uint32_t PB = s->w_general ? G::GWALK_PAYLOAD_BYTES : G::WALK_PAYLOAD_BYTES;
  for (const WNode& w : T) total += G::WALK_NODE_BYTES + (w.leaf >= 0 ? PB : 0);
  need(total < (1ull << 30), HRT_ERR_UNSUPPORTED, "scene too large for the walk stream");
  std::vector<uint32_t> addr(N), paddr(N, 0);
  const char* hot_env = knob_env("HRT_WALK_HOT"); /* "0": no LDS-staged top levels (A/B) */
  /* the staged budget: general streams twice the sphere kernel's (layout.h GWALK_LDS_BIG_BYTES; HRT_GWALK_BIG=0
   * keeps LDS_SCENE_MAX_BYTES, A/B) */
  const char* big_env = knob_env("HRT_GWALK_BIG");
  const uint32_t budget = s->w_general && !(big_env && strcmp(big_env, "0") == 0) ? G::GWALK_LDS_BIG_BYTES
                                                                                   : G::LDS_SCENE_MAX_BYTES;
  const bool hybrid = total > G::LDS_SCENE_MAX_BYTES && !(hot_env && strcmp(hot_env, "0") == 0);
  const char* pl = knob_env("HRT_WALK_PAYLOADS");
  const bool apart = !(pl && strcmp(pl, "inline") == 0);
  /* 16-B parts: the F_BASIC sphere kernel only (textured sphere scenes keep the 32-B parts of its HEAVY walk) */
  c16 = c16 && hybrid && apart && !s->w_general && !s->w_regroup_pending && N <= G::WALK_C16_MAX &&
        (s->feature_mask & ~G::F_BASIC) == 0;
  const uint32_t stage_budget = c16 ? 2u * budget : budget; /* in 32-B parts: halved by the transcode */
  uint32_t off = 0;
  std::vector<char> hot(N, 0);
  /* Hybrid placement (C4 1/8 share, r03u: +1.5% for both together, bit-identical): the node parts staged
   * are those a ray is likeliest to reach (largest parent box surface first; HRT_WALK_HOTSEL=depth: the
   * top levels breadth first), and the global node parts stay dense in pre-order with every payload
   * after them (HRT_WALK_PAYLOADS=inline: each payload behind its leaf) */
  const char* hotsel = knob_env("HRT_WALK_HOTSEL");
  const bool by_area = !(hotsel && strcmp(hotsel, "depth") == 0);
  std::vector<uint32_t> order; /* hybrid: the node parts in staging priority */
  if (hybrid) {
    order.resize(N);
    for (uint32_t i = 0; i < N; i++) order[i] = i;
    if (s->has_view && by_area) {
      /* hrt_scene_set_view: the node parts the view's camera rays visit most (lane-simulated C4 segments, held-out
       * rows: 14.2 -> 1.6 of 73.7 node visits per segment outside LDS, scripts/price_hotset.py), then the
       * largest parent box first among the rest */
      const std::vector<uint32_t> heat = view_heat(s->view, T);
      std::vector<double> key(N, 0.0);
      key[0] = HUGE_VAL;
      for (uint32_t i = 0; i < N; i++)
        if (T[i].leaf < 0 && i + 1 < N) {
          const double a = half_area(T[i].box);
          key[i + 1] = a;
          if (T[i + 1].end < N) key[T[i + 1].end] = a;
        }
      std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
        if (heat[a] != heat[b]) return heat[a] > heat[b];
        return key[a] != key[b] ? key[a] > key[b] : T[a].depth < T[b].depth;
      });
    } else if (by_area) {
      std::vector<double> key(N, 0.0);
      key[0] = HUGE_VAL;
      for (uint32_t i = 0; i < N; i++)
        if (T[i].leaf < 0 && i + 1 < N) {
          const double a = half_area(T[i].box);
          key[i + 1] = a;
          if (T[i + 1].end < N) key[T[i + 1].end] = a;
        }
      std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
        return key[a] != key[b] ? key[a] > key[b] : T[a].depth < T[b].depth;
      });
    } else {
      std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return T[a].depth < T[b].depth; });
    }
    for (uint32_t i : order) {
      if (off + G::WALK_NODE_BYTES > stage_budget) break;
      addr[i] = off;
      off += G::WALK_NODE_BYTES;
      hot[i] = 1;
    }
  }
  s->w_hot = hybrid ? off : 0;
  /* (the payloads of a hybrid stream all lie behind the staged node parts: lane.h payload_mem reads them
   * from global memory without a per-lane choice; checked below) */
  for (uint32_t i = 0; i < N; i++) {
    if (!hot[i]) {
      addr[i] = off;
      off += G::WALK_NODE_BYTES;
    }
    if (T[i].leaf >= 0 && !hot[i] && !(hybrid && apart)) {
      paddr[i] = off;
      off += PB;
    }
  }
  if (hybrid && apart)
    for (uint32_t i = 0; i < N; i++)
      if (T[i].leaf >= 0 && !hot[i]) {
        paddr[i] = off;
        off += PB;
      }
  for (uint32_t i = 0; i < N; i++)
    if (T[i].leaf >= 0 && hot[i]) {
      paddr[i] = off;
      off += PB;
    }
  need(off == total, HRT_ERR_STATE, "walk stream placement");
  uint32_t END = off;
  /* split node parts (layout.h WALK_SPLIT_HALF), opt-in (HRT_WALK_SPLIT=1): sphere streams staged whole in
   * LDS that fill the space between the two halves with payloads */
  const char* sp_env = knob_env("HRT_WALK_SPLIT");
  const uint32_t H2 = G::WALK_SPLIT_HALF;
  s->w_half = 16;
  s->w_generic = false; /* set below by the first leaf that needs trace_ray */
  if (!hybrid && !s->w_general && (s->feature_mask & ~G::F_BASIC) == 0 && sp_env && strcmp(sp_env, "1") == 0 &&
      (uint64_t)N * 16u <= H2 &&
      total >= (uint64_t)H2 + 16u * N) {
    uint32_t a = 0, q = 16u * N; /* node parts in pre-order, payloads in the gap, then behind the second half */
    for (uint32_t i = 0; i < N; i++) {
      addr[i] = a;
      a += 16;
    }
    for (uint32_t i = 0; i < N; i++) {
      if (T[i].leaf < 0) continue;
      if (q + PB > H2 && q < H2 + 16u * N) q = H2 + 16u * N;
      paddr[i] = q;
      q += PB;
    }
    END = std::max(q, H2 + 16u * N);
    s->w_half = H2;
  }
  /* split node parts of a HYBRID sphere stream (opt-in HRT_WALK_SPLIT=1): pages of 2 x
   * WALK_SPLIT_HALF_HYB bytes, each holding the first halves of WALK_SPLIT_HALF_HYB / 16 node parts back to back
   * and their second halves WALK_SPLIT_HALF_HYB further, so the LDS and the buffer reads both find a part's second
   * half at a fixed immediate offset.  The staged set keeps the hot order, as many parts as fit the budget (a
   * partial last page staged up to its last second half); the other parts start on the next page, in pre-order;
   * every payload after the last page. */
  if (hybrid && !c16 && !s->w_general && (s->feature_mask & ~G::F_BASIC) == 0 && sp_env && strcmp(sp_env, "1") == 0 &&
      apart) {
    const uint32_t HH = G::WALK_SPLIT_HALF_HYB, PPP = HH / 16u;
    auto extent = [&](uint32_t n) { return (n / PPP) * 2u * HH + (n % PPP ? HH + 16u * (n % PPP) : 0u); };
    auto slot = [&](uint32_t k) { return (k / PPP) * 2u * HH + (k % PPP) * 16u; };
    uint32_t n_hot = 0;
    while (n_hot < N && extent(n_hot + 1) <= budget) n_hot++;
    std::fill(hot.begin(), hot.end(), 0);
    uint32_t k = 0;
    for (; k < n_hot; k++) {
      hot[order[k]] = 1;
      addr[order[k]] = slot(k);
    }
    if (k % PPP) k += PPP - k % PPP; /* the global parts start on a page of their own */
    for (uint32_t i = 0; i < N; i++)
      if (!hot[i]) addr[i] = slot(k++);
    uint32_t q = k % PPP ? (k / PPP) * 2u * HH + HH + 16u * (k % PPP) : (k / PPP) * 2u * HH;
    for (uint32_t i = 0; i < N; i++) /* payloads: the global leaves' in pre-order, then the staged leaves' */
      if (T[i].leaf >= 0 && !hot[i]) {
        paddr[i] = q;
        q += PB;
      }
    for (uint32_t i = 0; i < N; i++)
      if (T[i].leaf >= 0 && hot[i]) {
        paddr[i] = q;
        q += PB;
      }
    END = q;
    s->w_hot = extent(n_hot);
    s->w_half = HH;
  }
  if (s->w_hot)
    for (uint32_t i = 0; i < N; i++)
      need(T[i].leaf < 0 || paddr[i] >= s->w_hot, HRT_ERR_STATE, "walk stream: a hybrid stream's payload in its staged part");
  if (!hybrid) s->w_hot = 0;
  std::vector<float>& o = s->w_stream;
  o.assign(END / 4, 0.0f);
  const float inf = u2f(0x7f800000u);
  /* every node's C, E (layout.h CE_FLOOR), children first: a node raised by the floor widens the boxes
   * above it (pre-order: an inner node's children are i + 1 and T[i + 1].end) */
  std::vector<float> CE((size_t)N * 6);
  std::vector<Aabb> fb(N);
  std::vector<char> fbox_ok(N, 1);
  for (uint32_t i = N; i-- > 0;) {
    const WNode& w = T[i];
    float* C = &CE[(size_t)i * 6];
    float* E = C + 3;
    if (w.leaf >= 0 && leaves[w.leaf].nobox) {
      C[0] = C[1] = C[2] = 0.0f;
      E[0] = E[1] = E[2] = inf;
      fbox_ok[i] = 0;
      continue;
    }
    Aabb bx = w.box;
    if (w.leaf < 0) { /* the union of the children's (possibly widened) boxes, when both have one */
      const uint32_t c1 = i + 1, c2 = T[i + 1].end;
      if (c2 < N && fbox_ok[c1] && fbox_ok[c2]) bx = box_union(bx, box_union(fb[c1], fb[c2]));
    }
    box_ce_floored(bx, C, E, &fb[i]);
  }
  for (uint32_t i = 0; i < N; i++) {
    const WNode& w = T[i];
    const uint32_t skip = w.end < N ? addr[w.end] : END;
    const float* C = &CE[(size_t)i * 6];
    const float* E = C + 3;
    if (w.leaf < 0) {
      need(i + 1 < N, HRT_ERR_STATE, "walk stream: inner node without children");
      put4(o, addr[i], C[0], C[1], C[2], u2f(skip));
      put4(o, addr[i] + s->w_half, E[0], E[1], E[2], u2f(addr[i + 1])); /* pass: the first child */
      continue;
    }
    const WalkLeaf& L = leaves[w.leaf];
    put4(o, addr[i], C[0], C[1], C[2], u2f(skip));
    put4(o, addr[i] + s->w_half, E[0], E[1], E[2], u2f(paddr[i] | G::WALK_PEND));
    if (s->w_general) { /* layout.h general-scene walk stream: the leaf's program range */
      const uint32_t q = paddr[i];
      /* GL_ONE: the node's kind word instead of the range's end; GL_MED: the medium, and the boundary
       * sphere instead of the (world-level) instance */
      uint32_t one = 0, second = L.end, fourth = L.inst;
      if (L.end == L.begin + 1) {
        const uint32_t k = (s->g_nodes[L.begin].kp >> 24) & G::KIND_MASK;
        if (k == G::K_BOX_PRIM || k == G::K_PRIM) {
          one = G::GL_ONE;
          second = s->g_nodes[L.begin].kp;
        }
      } else if (L.end == L.begin + 2 && !(L.gflags & G::GL_INST) && L.inst == G::NONE) {
        const uint32_t k0 = (s->g_nodes[L.begin].kp >> 24) & G::KIND_MASK;
        const uint32_t k1 = (s->g_nodes[L.begin + 1].kp >> 24) & G::KIND_MASK;
        const uint32_t mi = s->g_nodes[L.begin + 1].kp & 0xFFFFFFu;
        const char* me = knob_env("HRT_GWALK_MED"); /* "0": media leaves run trace_ray (A/B) */
        if (HRT_MEDIUM_PAIR && k0 == G::K_BOX && k1 == G::K_MEDIUM && s->g_media[mi].sphere != G::NONE &&
            !(me && strcmp(me, "0") == 0)) {
          one = G::GL_MED;
          second = mi;
          fourth = s->g_media[mi].sphere;
        }
      }
      if (!one) s->w_generic = true;
      put4(o, q, u2f(L.begin), u2f(second), u2f((L.has_rbox ? G::GL_BOX : 0u) | L.gflags | one), u2f(skip << 2));
      put4(o, q + 16, L.rbox.mn.x, L.rbox.mn.y, L.rbox.mn.z, u2f(fourth));
      put4(o, q + 32, L.rbox.mx.x, L.rbox.mx.y, L.rbox.mx.z, u2f(L.rgroup));
      continue;
    }
    const G::Prim& p = s->g_prims[L.prim];
    const bool moving = (p.km & 3u) == G::P_MOVING;
    /* the reference test at the leaf: its own box, or for a box-less List member the nearest enclosing
     * BvhNode box (monotone: it implies every enclosing box's test), or none at world level */
    const bool ref_test = !L.nobox;
    need(!L.has_rbox, HRT_ERR_STATE, "sphere walk stream: a leaf needs its group's box test (general stream)");
    const Aabb& rb = L.box;
    const uint32_t wflags = (moving ? G::WL_MOVING : 0u) | (ref_test ? 0u : G::WL_NOBOX) | (skip << 2);
    const uint32_t q = paddr[i];
    put4(o, q, rb.mn.x, rb.mn.y, rb.mn.z, u2f(wflags));
    put4(o, q + 16, rb.mx.x, rb.mx.y, rb.mx.z, p.p0[3]);
    put4(o, q + 32, p.p0[0], p.p0[1], p.p0[2], moving ? p.p1[3] : 0.0f);
    put4(o, q + 48, moving ? p.p1[0] : 0.0f, moving ? p.p1[1] : 0.0f, moving ? p.p1[2] : 0.0f, moving ? p.p2[0] : 1.0f);
    /* the material, inline (layout.h) */
    const uint32_t mi = p.km >> 4;
    need(mi < (1u << 24), HRT_ERR_UNSUPPORTED, "too many materials for the walk stream");
    const G::Mat& m = s->g_mats[mi];
    float A[4] = {0.0f, 0.0f, 0.0f, 0.0f}, Bc[3] = {0.0f, 0.0f, 0.0f};
    uint32_t wt = G::WT_GLOBAL;
    if (m.kind == G::M_METAL) {
      A[0] = m.a[0]; A[1] = m.a[1]; A[2] = m.a[2]; A[3] = m.a[3];
      wt = G::WT_SOLID;
    } else if (m.kind == G::M_DIELECTRIC) {
      A[3] = m.a[0];
      wt = G::WT_SOLID;
    } else {
      const G::Tex& t = s->g_texs[m.tex];
      if (t.kind == G::T_SOLID) {
        A[0] = t.a[0]; A[1] = t.a[1]; A[2] = t.a[2];
        wt = G::WT_SOLID;
      } else if (t.kind == G::T_CHECKER && s->g_texs[t.i0].kind == G::T_SOLID && s->g_texs[t.i1].kind == G::T_SOLID) {
        const G::Tex &odd = s->g_texs[t.i0], &even = s->g_texs[t.i1];
        A[0] = odd.a[0]; A[1] = odd.a[1]; A[2] = odd.a[2];
        Bc[0] = even.a[0]; Bc[1] = even.a[1]; Bc[2] = even.a[2];
        wt = G::WT_CHECKER;
      }
    }
    put4(o, q + 64, A[0], A[1], A[2], A[3]);
    put4(o, q + 80, Bc[0], Bc[1], Bc[2], u2f(m.kind | wt << 4 | mi << 8));
  }
  s->w_end = END;
  s->w_nodes = N;
  s->w_c16 = false;
  s->w_pbase = 0;
  if (c16) walk_transcode_c16(s, N);
  return !c16 || s->w_c16;
}

void walk_place_and_write(hrt_scene* s, const std::vector<WNode>& T, const std::vector<WalkLeaf>& leaves) {
  /* "1": 16-B node parts for hybrid sphere streams (opt-in: r05 measured them 8% slower on C4's 1/8 share,
   * 6 357 -> 5 833 Mrays/s: the binary16 widening and the link decode add ~8 VALU to a node step, more than the
   * doubled staged set saves; profiles/r05_c16_ab.txt) */
  const char* c16_env = knob_env("HRT_WALK_C16");
  const bool c16 = c16_env && strcmp(c16_env, "1") == 0;
  if (!walk_place_and_write_impl(s, T, leaves, c16)) walk_place_and_write_impl(s, T, leaves, false);
}

/* The leaf sequence of the reference stream (its pre-order) and the reference hierarchy over it. */
std::vector<WalkLeaf> walk_leaves(const hrt_scene* s, std::vector<WNode>* ref_tree, bool* regroup_ok) {
  const uint32_t n = s->main_end;
  std::vector<WalkLeaf> leaves;
  std::vector<uint32_t> open; /* enclosing box nodes (index into the reference tree) */
  std::vector<WNode> T;
  bool ok = true;
  for (uint32_t i = 0; i < n; i++) {
    const G::Node& g = s->g_nodes[i];
    const uint32_t kind = (g.kp >> 24) & G::KIND_MASK;
    while (!open.empty() && T[open.back()].end <= i) open.pop_back();
    Aabb b;
    b.mn = v3(g.mn[0], g.mn[1], g.mn[2]);
    b.mx = v3(g.mx[0], g.mx[1], g.mx[2]);
    if (kind == G::K_BOX) {
      need(g.skip > i && g.skip <= n, HRT_ERR_STATE, "walk stream: bad skip link");
      T.push_back(WNode{b, -1, g.skip, (uint32_t)open.size()});
      open.push_back(i);
      continue;
    }
    need(kind == G::K_BOX_PRIM || kind == G::K_PRIM, HRT_ERR_STATE, "walk stream: unexpected node kind");
    WalkLeaf L;
    L.nobox = kind == G::K_PRIM;
    L.prim = g.kp & 0xFFFFFFu;
    L.box = b;
    if (L.nobox) ok = false;
    if (L.nobox && !open.empty()) { /* a List member inside a BvhNode leaf: that box's reference test */
      L.has_rbox = true;
      L.rbox = T[open.back()].box;
      L.rgroup = open.back();
    }
    for (int k = 0; k < 3 && !L.nobox; k++)
      if (!(g.mn[k] <= g.mx[k]) || !std::isfinite(g.mn[k]) || !std::isfinite(g.mx[k])) ok = false;
    T.push_back(WNode{b, (int32_t)leaves.size(), i + 1, (uint32_t)open.size()});
    leaves.push_back(L);
  }
  if (ref_tree) *ref_tree = std::move(T);
  if (regroup_ok) *regroup_ok = ok;
  return leaves;
}

/* The general stream's leaf objects (layout.h) in the reference's pre-order, and the reference
 * hierarchy above them (WNode ends as reference-stream indices: the caller renumbers).  A K_BOX is a
 * hierarchy node when its subtree holds a box node outside every instance bracket (its children are
 * BvhNodes); otherwise it is a leaf, its program the whole subtree (boxes inside instances included:
 * trace_ray walks them in the instance's frame). */
std::vector<WalkLeaf> gwalk_leaves(const hrt_scene* s, std::vector<WNode>* ref_tree, bool* regroup_ok,
                                   const std::vector<char>* whole) {
  const uint32_t n = s->main_end;
  const float inf = u2f(0x7f800000u);
  std::vector<WalkLeaf> leaves;
  std::vector<WNode> T;
  std::vector<uint32_t> start; /* reference-stream index at which each hierarchy node starts */
  struct Open { uint32_t end; Aabb box; uint32_t node; };
  std::vector<Open> open;
  bool ok = true;
  auto node_box = [&](uint32_t i) {
    const G::Node& g = s->g_nodes[i];
    Aabb b;
    b.mn = v3(g.mn[0], g.mn[1], g.mn[2]);
    b.mx = v3(g.mx[0], g.mx[1], g.mx[2]);
    return b;
  };
  auto finite_box = [](const Aabb& b) {
    for (int k = 0; k < 3; k++)
      if (!(b.mn[k] <= b.mx[k]) || !std::isfinite(b.mn[k]) || !std::isfinite(b.mx[k])) return false;
    return true;
  };
  /* the true extent of a world-level sphere or rect (rect.rs:55-59 axes: a ZX rect spans z over
   * [a0, a1] and x over [b0, b1], the transpose of its bounding box, G17) */
  auto prim_extent = [&](uint32_t prim, Aabb& b) { /* in the primitive's own frame */
    const G::Prim& p = s->g_prims[prim];
    const uint32_t kind = p.km & 3u;
    if (kind == G::P_SPHERE) {
      b.mn = v3(p.p0[0] - p.p0[3], p.p0[1] - p.p0[3], p.p0[2] - p.p0[3]);
      b.mx = v3(p.p0[0] + p.p0[3], p.p0[1] + p.p0[3], p.p0[2] + p.p0[3]);
      return finite_box(b);
    }
    if (kind != G::P_RECT) return false;
    const uint32_t plane = (p.km >> 2) & 3u;
    const int ka = plane == HRT_PLANE_XY ? 2 : (plane == HRT_PLANE_YZ ? 0 : 1);
    const int aa = plane == HRT_PLANE_XY ? 0 : (plane == HRT_PLANE_YZ ? 1 : 2);
    const int ba = plane == HRT_PLANE_XY ? 1 : (plane == HRT_PLANE_YZ ? 2 : 0);
    float mn[3], mx[3];
    mn[ka] = mx[ka] = p.p1[0];
    mn[aa] = p.p0[0]; mx[aa] = p.p0[1];
    mn[ba] = p.p0[2]; mx[ba] = p.p0[3];
    b.mn = v3(mn[0], mn[1], mn[2]);
    b.mx = v3(mx[0], mx[1], mx[2]);
    return finite_box(b);
  };
  /* the world image of a box in instance `inst`'s frame: its corners through the chain back to the world
   * (innermost first, the inverse of lane.h inst_ray, in double), padded for the f32 rounding of the
   * reference's ray transforms */
  auto to_world = [&](const Aabb& b, uint32_t inst, Aabb& out) {
    double mn[3] = {1e300, 1e300, 1e300}, mx[3] = {-1e300, -1e300, -1e300}, scale = 0.0;
    for (int c = 0; c < 8; c++) {
      double p[3] = {(c & 1) ? b.mx.x : b.mn.x, (c & 2) ? b.mx.y : b.mn.y, (c & 4) ? b.mx.z : b.mn.z};
      for (int k = 0; k < 3; k++) scale = std::max(scale, std::fabs(p[k]));
      for (uint32_t q = inst; q != G::NONE; q = s->g_insts[q].parent) {
        const G::Inst& in = s->g_insts[q];
        if ((in.kind & G::I_KIND_MASK) == G::I_TRANSLATE) {
          for (int k = 0; k < 3; k++) p[k] += (double)in.d[k];
        } else {
          const int a = (int)(in.axis + 1) % 3, bb = (int)(in.axis + 2) % 3;
          const double sn = in.sin_t, cs = in.cos_t, pa = p[a], pb = p[bb];
          p[a] = cs * pa - sn * pb;
          p[bb] = sn * pa + cs * pb;
        }
        for (int k = 0; k < 3; k++) scale = std::max(scale, std::fabs(p[k]));
      }
      for (int k = 0; k < 3; k++) {
        mn[k] = std::min(mn[k], p[k]);
        mx[k] = std::max(mx[k], p[k]);
      }
    }
    const double pad = 1e-5 * scale + 1e-30;
    float fmn[3], fmx[3];
    for (int k = 0; k < 3; k++) {
      fmn[k] = (float)(mn[k] - pad);
      fmx[k] = (float)(mx[k] + pad);
      if ((double)fmn[k] > mn[k] - pad) fmn[k] = nextafterf(fmn[k], -3.40282347e+38f);
      if ((double)fmx[k] < mx[k] + pad) fmx[k] = nextafterf(fmx[k], 3.40282347e+38f);
    }
    out.mn = v3(fmn[0], fmn[1], fmn[2]);
    out.mx = v3(fmx[0], fmx[1], fmx[2]);
    return finite_box(out);
  };
  /* Flatten the instance chains of a leaf object's content [a, b) (layout.h): every leaf object inside
   * (a primitive, a box-less Cuboid / List member, a BvhNode leaf or box-only subtree of the instance's
   * own hierarchy) becomes a leaf with its chain.  Not possible (false) when a box sits in an outer frame
   * of a nested instance, a box-less primitive sits under a box of its frame, or a medium is inside. */
  struct Flat { uint32_t begin, end, inst; bool has_box; Aabb box; bool ref_only; int prim; };
  auto flatten_chains = [&](uint32_t a, uint32_t b, std::vector<Flat>& out) {
    std::vector<uint32_t> insts, local_end;
    for (uint32_t j = a; j < b;) {
      while (!local_end.empty() && local_end.back() <= j) local_end.pop_back();
      const G::Node& g = s->g_nodes[j];
      const uint32_t k = (g.kp >> 24) & G::KIND_MASK, pl = g.kp & 0xFFFFFFu;
      const bool ro = (g.kp & G::NODE_REF_ONLY) != 0;
      const uint32_t inst = insts.empty() ? G::NONE : insts.back();
      if (k == G::K_INST_BEGIN) {
        if (!local_end.empty()) return false;
        insts.push_back(pl);
        j++;
      } else if (k == G::K_INST_END) {
        if (!local_end.empty() || insts.empty()) return false;
        insts.pop_back();
        j++;
      } else if (k == G::K_BOX) {
        if (insts.empty()) return false;
        bool has_inst = false, has_box = false;
        for (uint32_t m = j + 1; m < g.skip; m++) {
          const uint32_t km = (s->g_nodes[m].kp >> 24) & G::KIND_MASK;
          has_inst |= km == G::K_INST_BEGIN || km == G::K_MEDIUM;
          has_box |= km == G::K_BOX || km == G::K_BOX_PRIM;
        }
        if (has_inst) return false;
        if (has_box) { /* a hierarchy node of the instance's BvhNode: implied by its leaves' own tests */
          local_end.push_back(g.skip);
          j++;
          continue;
        }
        const int prim = (g.skip == j + 2 && ((s->g_nodes[j + 1].kp >> 24) & G::KIND_MASK) == G::K_PRIM)
                             ? (int)(s->g_nodes[j + 1].kp & 0xFFFFFFu) : -1;
        Aabb bx;
        bx.mn = v3(g.mn[0], g.mn[1], g.mn[2]);
        bx.mx = v3(g.mx[0], g.mx[1], g.mx[2]);
        out.push_back(Flat{j, g.skip, inst, true, bx, ro, prim});
        j = g.skip;
      } else if (k == G::K_BOX_PRIM) {
        if (insts.empty()) return false;
        Aabb bx;
        bx.mn = v3(g.mn[0], g.mn[1], g.mn[2]);
        bx.mx = v3(g.mx[0], g.mx[1], g.mx[2]);
        out.push_back(Flat{j, j + 1, inst, true, bx, ro, (int)pl});
        j++;
      } else if (k == G::K_PRIM) {
        if (!local_end.empty()) return false;
        out.push_back(Flat{j, j + 1, inst, false, Aabb{}, false, (int)pl});
        j++;
      } else {
        return false; /* a medium */
      }
    }
    return insts.empty();
  };
  auto add_leaf = [&](uint32_t begin, uint32_t end, bool has_box, const Aabb& box, bool ref_only, int prim) {
    WalkLeaf L;
    L.begin = begin;
    L.end = end;
    L.prim = prim >= 0 ? (uint32_t)prim : G::NONE;
    L.nobox = true;
    Aabb ext;
    const bool has_ext = prim >= 0 && prim_extent((uint32_t)prim, ext);
    if (has_box && !ref_only) { /* a BvhNode box that holds its geometry (box_ok) */
      L.box = box;
      L.nobox = false;
    } else if (has_ext) { /* a world-level primitive: its extent (joined with its transposed box) */
      L.box = has_box ? box_union(box, ext) : ext;
      L.nobox = false;
    }
    if (!L.nobox && !finite_box(L.box)) L.nobox = true;
    if (L.nobox) {
      ok = false;
      L.box.mn = v3(-inf, -inf, -inf);
      L.box.mx = v3(inf, inf, inf);
    }
    if (!has_box && !open.empty()) { /* box-less: the nearest enclosing BvhNode's reference test first */
      L.has_rbox = true;
      L.rbox = open.back().box;
      L.rgroup = open.back().node;
    }
    T.push_back(WNode{L.box, (int32_t)leaves.size(), end, (uint32_t)open.size()});
    start.push_back(begin);
    leaves.push_back(L);
  };
  /* a leaf of a flattened chain: its program in the frame of `f.inst`, after the reference test of the
   * world-frame box `wbox` around the chain (if any) */
  auto add_flat = [&](const Flat& f, bool has_wbox, const Aabb& wbox, uint32_t wgroup, uint32_t ref_end) {
    WalkLeaf L;
    L.begin = f.begin;
    L.end = f.end;
    L.prim = f.prim >= 0 ? (uint32_t)f.prim : G::NONE;
    L.inst = f.inst;
    L.nobox = true;
    Aabb local, ext;
    bool has_local = false;
    const bool has_ext = f.prim >= 0 && prim_extent((uint32_t)f.prim, ext);
    if (f.has_box && !f.ref_only) { local = f.box; has_local = true; }
    else if (has_ext) { local = f.has_box ? box_union(f.box, ext) : ext; has_local = true; }
    if (has_local) L.nobox = !(f.inst == G::NONE ? (L.box = local, finite_box(local)) : to_world(local, f.inst, L.box));
    if (L.nobox) {
      ok = false;
      L.box.mn = v3(-inf, -inf, -inf);
      L.box.mx = v3(inf, inf, inf);
    }
    L.has_rbox = has_wbox;
    L.rbox = wbox;
    L.rgroup = wgroup;
    if (f.inst != G::NONE) {
      L.gflags |= G::GL_INST;
      bool dir = false;
      for (uint32_t q = f.inst; q != G::NONE; q = s->g_insts[q].parent)
        dir |= (s->g_insts[q].kind & G::I_KIND_MASK) != G::I_TRANSLATE;
      if (dir) {
        L.gflags |= G::GL_DIR;
        for (uint32_t m = f.begin; m < f.end; m++) {
          const uint32_t km = (s->g_nodes[m].kp >> 24) & G::KIND_MASK;
          if (km == G::K_BOX || km == G::K_BOX_PRIM) L.gflags |= G::GL_INV;
          if ((km == G::K_BOX_PRIM || km == G::K_PRIM) && (s->g_prims[s->g_nodes[m].kp & 0xFFFFFFu].km & 3u) != G::P_RECT)
            L.gflags |= G::GL_DD;
        }
      }
    }
    T.push_back(WNode{L.box, (int32_t)leaves.size(), ref_end, (uint32_t)open.size()});
    start.push_back(f.begin);
    leaves.push_back(L);
  };
  const char* flat_env = knob_env("HRT_GWALK_FLAT"); /* "0": instance chains stay whole leaf programs (A/B) */
  const bool flat_ok = !(flat_env && strcmp(flat_env, "0") == 0);
  const char* fl_env = knob_env("HRT_GWALK_FLATLIST"); /* "0": a BvhNode leaf's Cuboid / List stays one program (A/B) */
  const bool flat_lists = !(fl_env && strcmp(fl_env, "0") == 0);
  uint32_t i = 0;
  while (i < n) {
    while (!open.empty() && open.back().end <= i) open.pop_back();
    const G::Node& g = s->g_nodes[i];
    const uint32_t kind = (g.kp >> 24) & G::KIND_MASK, payload = g.kp & 0xFFFFFFu;
    const bool ref_only = (g.kp & G::NODE_REF_ONLY) != 0;
    if (kind == G::K_BOX) {
      const uint32_t skip = g.skip;
      need(skip > i && skip <= n, HRT_ERR_STATE, "general walk stream: bad skip link");
      bool hierarchy = false;
      int depth = 0;
      for (uint32_t j = i + 1; j < skip && !hierarchy; j++) {
        const uint32_t k = (s->g_nodes[j].kp >> 24) & G::KIND_MASK;
        if (k == G::K_INST_BEGIN) depth++;
        else if (k == G::K_INST_END) depth--;
        else if (depth == 0 && (k == G::K_BOX || k == G::K_BOX_PRIM)) hierarchy = true;
      }
      if (hierarchy && whole && (*whole)[i]) hierarchy = false; /* kept whole (gwalk_leaves_grouped) */
      if (hierarchy) {
        T.push_back(WNode{node_box(i), -1, skip, (uint32_t)open.size()});
        start.push_back(i);
        open.push_back(Open{skip, node_box(i), i});
        i++;
        continue;
      }
      /* the leaf's single primitive, if the subtree is one world-level prim (for its true extent) */
      std::vector<Flat> fl;
      bool chains = false, prims_only = skip > i + 2;
      for (uint32_t j = i + 1; j < skip; j++) {
        const uint32_t kj = (s->g_nodes[j].kp >> 24) & G::KIND_MASK;
        chains |= kj == G::K_INST_BEGIN;
        prims_only &= kj == G::K_PRIM;
      }
      /* a Cuboid's or a List's box-less primitives under a BvhNode leaf: each its own leaf (its true extent
       * for the inflated test, the leaf's box tested once per group), as a flattened chain's members */
      if ((chains || (prims_only && flat_lists)) && flat_ok && flatten_chains(i + 1, skip, fl) && !fl.empty()) {
        /* the BvhNode leaf's box is tested (world frame) before each flattened leaf's program */
        for (size_t q = 0; q < fl.size(); q++) add_flat(fl[q], true, node_box(i), i, q + 1 < fl.size() ? fl[q + 1].begin : skip);
        i = skip;
        continue;
      }
      const int prim = (skip == i + 2 && ((s->g_nodes[i + 1].kp >> 24) & G::KIND_MASK) == G::K_PRIM)
                           ? (int)(s->g_nodes[i + 1].kp & 0xFFFFFFu) : -1;
      add_leaf(i, skip, true, node_box(i), ref_only, prim);
      i = skip;
    } else if (kind == G::K_BOX_PRIM) {
      add_leaf(i, i + 1, true, node_box(i), ref_only, (int)payload);
      i++;
    } else if (kind == G::K_PRIM) {
      add_leaf(i, i + 1, false, Aabb{}, false, (int)payload);
      i++;
    } else if (kind == G::K_INST_BEGIN) { /* a box-less instance chain: up to its matching end */
      int depth = 0;
      uint32_t j = i;
      for (; j < n; j++) {
        const uint32_t k = (s->g_nodes[j].kp >> 24) & G::KIND_MASK;
        if (k == G::K_INST_BEGIN) depth++;
        else if (k == G::K_INST_END && --depth == 0) break;
      }
      need(j < n, HRT_ERR_STATE, "general walk stream: unbalanced instance brackets");
      std::vector<Flat> fl;
      if (flat_ok && flatten_chains(i, j + 1, fl) && !fl.empty()) {
        const bool wb = !open.empty();
        const Aabb wbox = wb ? open.back().box : Aabb{};
        const uint32_t wg = wb ? open.back().node : G::NONE;
        for (size_t q = 0; q < fl.size(); q++) add_flat(fl[q], wb, wbox, wg, q + 1 < fl.size() ? fl[q + 1].begin : j + 1);
        i = j + 1;
        continue;
      }
      add_leaf(i, j + 1, false, Aabb{}, false, -1);
      i = j + 1;
    } else if (kind == G::K_MEDIUM) {
      add_leaf(i, i + 1, false, Aabb{}, false, -1);
      i++;
    } else {
      need(false, HRT_ERR_STATE, "general walk stream: unbalanced instance brackets");
    }
  }
  /* ends: reference-stream indices -> hierarchy indices (the first node starting at or after the end) */
  for (size_t k = 0; k < T.size(); k++) {
    size_t m = k + 1;
    while (m < T.size() && start[m] < T[k].end) m++;
    T[k].end = (uint32_t)m;
  }
  /* an inner node's box for the inflated test: the union of its children's (a BvhNode box is the union
   * of its children's REFERENCE boxes, which for a transposed ZX rect (G17) need not hold the rect) */
  for (size_t k = T.size(); k-- > 0;) {
    if (T[k].leaf >= 0) continue;
    Aabb u = T[k + 1].box;
    for (uint32_t c = T[k + 1].end; c < T[k].end; c = T[c].end) u = box_union(u, T[c].box);
    T[k].box = u;
  }
  if (ref_tree) *ref_tree = std::move(T);
  if (regroup_ok) *regroup_ok = ok;
  return leaves;
}

/* The group-box state of a lane (lane.h gwalk_leaf_test gstate) remembers the outcome of the LAST group
 * whose box it tested.  A group's box-less leaves must therefore be contiguous in the leaf sequence: a
 * List inside a BvhNode leaf whose members come before AND after a nested BvhNode holding box-less members
 * of its own would re-test the outer box with a smaller closest after the inner group (the reference tests
 * it once, G19).  Such a box is kept as one leaf whose program is its whole subtree (trace_ray walks it
 * in the reference's order), which the leaf sequence is rebuilt with. */
std::vector<WalkLeaf> gwalk_leaves_grouped(const hrt_scene* s, std::vector<WNode>* ref_tree, bool* regroup_ok) {
  const char* ge = knob_env("HRT_GWALK_GROUPED"); /* "0": no fallback (tests show the case it covers) */
  if (ge && strcmp(ge, "0") == 0) return gwalk_leaves(s, ref_tree, regroup_ok);
  std::vector<char> whole(s->g_nodes.size(), 0);
  for (;;) {
    std::vector<WalkLeaf> leaves = gwalk_leaves(s, ref_tree, regroup_ok, &whole);
    std::vector<char> closed(s->g_nodes.size(), 0);
    uint32_t cur = G::NONE;
    bool again = false;
    for (const WalkLeaf& L : leaves) {
      if (!L.has_rbox || L.rgroup == cur) continue;
      if (cur != G::NONE) closed[cur] = 1;
      cur = L.rgroup;
      if (closed[cur]) { /* the group comes back after another one: keep its box whole */
        need(!whole[cur], HRT_ERR_STATE, "general walk stream: group kept whole twice");
        whole[cur] = 1;
        again = true;
      }
    }
    if (!again) return leaves;
  }
}

void build_walk(hrt_scene* s) {
  s->w_stream.clear();
  s->w_end = 0;
  s->w_hot = 0;
  s->w_regrouped = false;
  s->w_device_built = false;
  s->w_regroup_pending = false;
  s->w_general = false;
  if ((s->feature_mask & ~(G::F_BASIC | G::F_HEAVY_TEX)) != 0) { /* general scenes: the leaf-object stream */
    const char* gw = knob_env("HRT_GWALK"); /* "0": no general walk stream (segment kernels only) */
    if ((gw && strcmp(gw, "0") == 0) || s->media_nested) return;
    std::vector<WNode> T;
    bool regroup_ok = false;
    const std::vector<WalkLeaf> leaves = gwalk_leaves_grouped(s, &T, &regroup_ok);
    if (leaves.empty()) return;
    s->w_general = true;
    if (regroup_ok && s->opts.walk_tree == 0) {
      const auto t0 = std::chrono::steady_clock::now();
      T.clear();
      /* general streams keep the surface-area DP: with the view's rays Final walks 64.4 -> 65.4 node visits per
       * segment (lane simulator); the view still places their staged part */
      walk_regroup(T, leaves, nullptr);
      s->w_build_us = (uint32_t)std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count();
      s->w_regrouped = true;
    }
    walk_place_and_write(s, T, leaves);
    return;
  }
  std::vector<WNode> T;
  bool regroup_ok = false;
  const std::vector<WalkLeaf> leaves = walk_leaves(s, &T, &regroup_ok);
  if (leaves.empty()) return;
  for (const WalkLeaf& L : leaves)
    if (L.has_rbox) { /* a List member inside a BvhNode leaf: the box is tested once for the whole List,
                       * which the general stream's group test does (render_gwalk_kernel) */
      std::vector<WNode> TG;
      bool gok = false;
      const std::vector<WalkLeaf> gl = gwalk_leaves_grouped(s, &TG, &gok);
      s->w_general = true;
      if (gok && s->opts.walk_tree == 0) {
        TG.clear();
        walk_regroup(TG, gl, nullptr); /* general stream: the surface-area DP (above) */
        s->w_regrouped = true;
      }
      walk_place_and_write(s, TG, gl);
      return;
    }
  const char* wb = knob_env("HRT_WALK_BUILD"); /* host | device | auto (default) */
  const bool regroup = regroup_ok && s->opts.walk_tree == 0;
  /* large scenes are re-grouped on the device at upload (build_walk.hip): until then the
   * stream keeps the reference hierarchy (valid for the host-side tools that read it) */
  if (regroup && (wb ? strcmp(wb, "device") == 0 : leaves.size() >= 32768)) s->w_regroup_pending = true;
  else if (regroup) {
    const auto t0 = std::chrono::steady_clock::now();
    T.clear();
    walk_regroup(T, leaves, s->has_view ? &s->view : nullptr);
    s->w_build_us = (uint32_t)std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count();
    s->w_regrouped = true;
  }
  walk_place_and_write(s, T, leaves);
}

}  // namespace hrt
namespace hrt {
void flatten_scene(hrt_scene* s) { flatten(s); }
void flatten_scene_reference(hrt_scene* s) { flatten_reference(s); }

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

/* one blob per device: every layout.h section 256-B aligned */
std::vector<uint8_t> build_blob(hrt_scene* s) {
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
  s->off_chains = section(s->g_chains.size() * sizeof(float));
  s->off_fnodes = section(s->f_nodes.size() * sizeof(G::Node));
  s->off_fprims = section(s->f_prims.size() * sizeof(G::Prim));
  s->off_walk = section(s->w_stream.size() * sizeof(float));
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
  put(s->off_chains, s->g_chains.data(), s->g_chains.size() * sizeof(float));
  put(s->off_fnodes, s->f_nodes.data(), s->f_nodes.size() * sizeof(G::Node));
  put(s->off_fprims, s->f_prims.data(), s->f_prims.size() * sizeof(G::Prim));
  put(s->off_walk, s->w_stream.data(), s->w_stream.size() * sizeof(float));
  return blob;
}
}  // namespace hrt

/* ============================================================================ C ABI */
extern "C" {

const char* hrt_last_error(void) { return g_error.c_str(); }
const char* hrt_version(void) { return "hrt 0.6.0 (gfx950)"; }
uint32_t hrt_abi_version(void) { return HRT_ABI_VERSION; }

hrt_status hrt_scene_create(hrt_scene** out) {
  return guard([&] {
    need(out != nullptr, HRT_ERR_INVALID_ARG, "null out");
    *out = new hrt_scene();
  });
}

void hrt_scene_destroy(hrt_scene* s) {
  if (!s) return;
  device_release(s);
  delete s;
}

hrt_status hrt_tex_solid(hrt_scene* s, float r, float g, float b, uint32_t* id) {
  return guard([&] {
    mutable_scene(s);
    need(id != nullptr, HRT_ERR_INVALID_ARG, "null id");
    HTex t;
    t.kind = G::T_SOLID;
    t.color = v3(r, g, b);
    s->texs.push_back(t);
    *id = (uint32_t)(s->texs.size() - 1);
  });
}

hrt_status hrt_tex_checker(hrt_scene* s, uint32_t odd, uint32_t even, uint32_t* id) {
  return guard([&] {
    mutable_scene(s);
    need(id != nullptr, HRT_ERR_INVALID_ARG, "null id");
    check_tex(s, odd);
    check_tex(s, even);
    HTex t;
    t.kind = G::T_CHECKER;
    t.odd = odd;
    t.even = even;
    s->texs.push_back(t);
    *id = (uint32_t)(s->texs.size() - 1);
  });
}

hrt_status hrt_tex_noise(hrt_scene* s, float scale, const float* ranvec, const uint32_t* perm,
                         uint32_t* id) {
  return guard([&] {
    mutable_scene(s);
    need(id && ranvec && perm, HRT_ERR_INVALID_ARG, "null argument");
    G::Perlin p;
    memset(&p, 0, sizeof(p));
    for (int i = 0; i < 256; i++) {
      for (int c = 0; c < 3; c++) p.ranvec[i][c] = ranvec[3 * i + c];
      for (int c = 0; c < 3; c++) {
        need(perm[256 * c + i] < 256, HRT_ERR_INVALID_ARG, "permutation entry >= 256");
        p.perm[c][i] = p.perm[c][256 + i] = perm[256 * c + i]; /* twice over (layout.h Perlin) */
      }
    }
    s->perlin.push_back(p);
    HTex t;
    t.kind = G::T_NOISE;
    t.scale = scale;
    t.perlin = (uint32_t)(s->perlin.size() - 1);
    s->texs.push_back(t);
    *id = (uint32_t)(s->texs.size() - 1);
  });
}

hrt_status hrt_tex_image(hrt_scene* s, const uint8_t* data, uint32_t width, uint32_t height,
                         uint32_t components, uint32_t* id) {
  return guard([&] {
    mutable_scene(s);
    need(id != nullptr, HRT_ERR_INVALID_ARG, "null id");
    HTex t;
    t.kind = G::T_IMAGE;
    size_t bytes = (size_t)width * height * components;
    if (data && bytes) {
      need(components >= 3, HRT_ERR_INVALID_ARG, "image needs >= 3 components");
      need(s->images.size() + bytes < (1ull << 32), HRT_ERR_UNSUPPORTED, "image data > 4 GiB");
      t.img_off = s->images.size();
      s->images.insert(s->images.end(), data, data + bytes);
      t.w = width; t.h = height; t.c = components;
    } /* else: empty image -> magenta (image_texture.rs:37-39) */
    s->texs.push_back(t);
    *id = (uint32_t)(s->texs.size() - 1);
  });
}

static hrt_status add_mat(hrt_scene* s, HMat m, uint32_t* id) {
  return guard([&] {
    mutable_scene(s);
    need(id != nullptr, HRT_ERR_INVALID_ARG, "null id");
    if (m.tex != G::NONE) check_tex(s, m.tex);
    s->mats.push_back(m);
    *id = (uint32_t)(s->mats.size() - 1);
  });
}

hrt_status hrt_mat_lambertian(hrt_scene* s, uint32_t tex, uint32_t* id) {
  HMat m; m.kind = G::M_LAMBERTIAN; m.tex = tex;
  if (s && tex >= s->texs.size()) { set_error("bad texture id"); return HRT_ERR_INVALID_ARG; }
  return add_mat(s, m, id);
}
hrt_status hrt_mat_metal(hrt_scene* s, float r, float g, float b, float fuzz, uint32_t* id) {
  HMat m; m.kind = G::M_METAL; m.albedo = v3(r, g, b); m.fuzz = fuzz;
  return add_mat(s, m, id);
}
hrt_status hrt_mat_dielectric(hrt_scene* s, float ior, uint32_t* id) {
  HMat m; m.kind = G::M_DIELECTRIC; m.ior = ior;
  return add_mat(s, m, id);
}
hrt_status hrt_mat_diffuse_light(hrt_scene* s, uint32_t tex, uint32_t* id) {
  HMat m; m.kind = G::M_DIFFUSE_LIGHT; m.tex = tex;
  if (s && tex >= s->texs.size()) { set_error("bad texture id"); return HRT_ERR_INVALID_ARG; }
  return add_mat(s, m, id);
}
hrt_status hrt_mat_isotropic(hrt_scene* s, uint32_t tex, uint32_t* id) {
  HMat m; m.kind = G::M_ISOTROPIC; m.tex = tex;
  if (s && tex >= s->texs.size()) { set_error("bad texture id"); return HRT_ERR_INVALID_ARG; }
  return add_mat(s, m, id);
}

hrt_status hrt_node_sphere(hrt_scene* s, const float c[3], float r, uint32_t mat, uint32_t* id) {
  return guard([&] {
    mutable_scene(s);
    need(id != nullptr, HRT_ERR_INVALID_ARG, "null id");
    check_mat(s, mat);
    HNode n;
    n.kind = N_SPHERE;
    n.c0 = vin(c);
    n.r = r;
    n.mat = mat;
    *id = push_node(s, std::move(n));
  });
}

hrt_status hrt_node_moving_sphere(hrt_scene* s, const float c0[3], const float c1[3], float t0,
                                  float t1, float r, uint32_t mat, uint32_t* id) {
  return guard([&] {
    mutable_scene(s);
    need(id != nullptr, HRT_ERR_INVALID_ARG, "null id");
    check_mat(s, mat);
    HNode n;
    n.kind = N_MOVING;
    n.c0 = vin(c0);
    n.c1 = vin(c1);
    n.t0 = t0;
    n.t1 = t1;
    n.r = r;
    n.mat = mat;
    *id = push_node(s, std::move(n));
  });
}

hrt_status hrt_node_rect(hrt_scene* s, int32_t plane, float a0, float a1, float b0, float b1,
                         float k, uint32_t mat, uint32_t* id) {
  return guard([&] {
    mutable_scene(s);
    need(id != nullptr, HRT_ERR_INVALID_ARG, "null id");
    need(plane >= 0 && plane <= 2, HRT_ERR_INVALID_ARG, "bad plane");
    check_mat(s, mat);
    HNode n;
    n.kind = N_RECT;
    n.plane = plane;
    n.a0 = a0; n.a1 = a1; n.b0 = b0; n.b1 = b1; n.k = k;
    n.mat = mat;
    *id = push_node(s, std::move(n));
  });
}

/* cuboid.rs:29-97: six rects in this exact order (List order decides equal-t ties) */
hrt_status hrt_node_cuboid(hrt_scene* s, const float bmin[3], const float bmax[3], uint32_t mat,
                           uint32_t* id) {
  return guard([&] {
    mutable_scene(s);
    need(id != nullptr, HRT_ERR_INVALID_ARG, "null id");
    check_mat(s, mat);
    Vec3 p0 = vin(bmin), p1 = vin(bmax);
    struct R { int plane; float a0, a1, b0, b1, k; };
    const R sides[6] = {{HRT_PLANE_XY, p0.x, p1.x, p0.y, p1.y, p1.z}, {HRT_PLANE_XY, p0.x, p1.x, p0.y, p1.y, p0.z},
                        {HRT_PLANE_ZX, p0.z, p1.z, p0.x, p1.x, p1.y}, {HRT_PLANE_ZX, p0.z, p1.z, p0.x, p1.x, p0.y},
                        {HRT_PLANE_YZ, p0.y, p1.y, p0.z, p1.z, p1.x}, {HRT_PLANE_YZ, p0.y, p1.y, p0.z, p1.z, p0.x}};
    HNode c;
    c.kind = N_CUBOID;
    c.box = Aabb{p0, p1};
    c.has_box = true;
    for (const R& r : sides) {
      HNode n;
      n.kind = N_RECT;
      n.plane = r.plane;
      n.a0 = r.a0; n.a1 = r.a1; n.b0 = r.b0; n.b1 = r.b1; n.k = r.k;
      n.mat = mat;
      n.owned = true;
      c.children.push_back(push_node(s, std::move(n)));
    }
    *id = push_node(s, std::move(c));
  });
}

hrt_status hrt_node_translate(hrt_scene* s, uint32_t child, const float d[3], uint32_t* id) {
  return guard([&] {
    mutable_scene(s);
    need(id != nullptr, HRT_ERR_INVALID_ARG, "null id");
    Vec3 disp = vin(d);
    HNode n;
    n.kind = N_TRANSLATE;
    n.disp = disp;
    n.children.push_back(take_child(s, child));
    *id = push_node(s, std::move(n));
  });
}

/* rotation.rs:38-99 */
hrt_status hrt_node_rotate(hrt_scene* s, int32_t axis, uint32_t child, float angle, uint32_t* id) {
  return guard([&] {
    mutable_scene(s);
    need(id != nullptr, HRT_ERR_INVALID_ARG, "null id");
    need(axis >= 0 && axis <= 2, HRT_ERR_INVALID_ARG, "bad axis");
    need(child < s->nodes.size(), HRT_ERR_INVALID_ARG, "bad node id");
    need(!s->nodes[child].owned, HRT_ERR_INVALID_ARG, "node already owned by another node");
    int r_axis = axis, a_axis = (axis + 1) % 3, b_axis = (axis + 2) % 3;
    HNode n;
    n.kind = N_ROTATE;
    n.axis = axis;
    float radians = (PI_F / 180.0f) * angle;
    n.sin_t = sin_f(radians);
    n.cos_t = cos_f(radians);
    Aabb b;
    n.has_box = bbox(s, child, 0.0f, 1.0f, b);
    if (n.has_box) {
      const float FMAX = 3.40282347e+38f;
      Vec3 mn = v3(FMAX, FMAX, FMAX), mx = v3(-FMAX, -FMAX, -FMAX);
      for (int i = 0; i < 2; i++)
        for (int j = 0; j < 2; j++)
          for (int k = 0; k < 2; k++) {
            float r = (float)k * b.mx[r_axis] + (float)(1 - k) * b.mn[r_axis];
            float a = (float)i * b.mx[a_axis] + (float)(1 - i) * b.mn[a_axis];
            float bb = (float)j * b.mx[b_axis] + (float)(1 - j) * b.mn[b_axis];
            float new_a = n.cos_t * a - n.sin_t * bb;
            float new_b = n.sin_t * a + n.cos_t * bb;
            if (new_a < mn[a_axis]) mn[a_axis] = new_a;
            if (new_b < mn[b_axis]) mn[b_axis] = new_b;
            if (r < mn[r_axis]) mn[r_axis] = r;
            if (new_a > mx[a_axis]) mx[a_axis] = new_a;
            if (new_b > mx[b_axis]) mx[b_axis] = new_b;
            if (r > mx[r_axis]) mx[r_axis] = r;
          }
      n.box = Aabb{mn, mx};
    }
    n.children.push_back(take_child(s, child));
    *id = push_node(s, std::move(n));
  });
}

hrt_status hrt_node_constant_medium(hrt_scene* s, uint32_t boundary, float density, uint32_t tex,
                                    uint32_t* id) {
  return guard([&] {
    mutable_scene(s);
    need(id != nullptr, HRT_ERR_INVALID_ARG, "null id");
    check_tex(s, tex);
    HNode n;
    n.kind = N_MEDIUM;
    n.neg_inv_density = -1.0f / density;
    n.tex = tex;
    n.medium_id = s->n_media++;
    n.children.push_back(take_child(s, boundary));
    *id = push_node(s, std::move(n));
  });
}

hrt_status hrt_node_list(hrt_scene* s, const uint32_t* children, uint32_t n_children, uint32_t* id) {
  return guard([&] {
    mutable_scene(s);
    need(id != nullptr && (children != nullptr || n_children == 0), HRT_ERR_INVALID_ARG, "null argument");
    for (uint32_t i = 0; i < n_children; i++) {
      need(children[i] < s->nodes.size(), HRT_ERR_INVALID_ARG, "bad node id");
      need(!s->nodes[children[i]].owned, HRT_ERR_INVALID_ARG, "node already owned by another node");
      for (uint32_t j = 0; j < i; j++) need(children[j] != children[i], HRT_ERR_INVALID_ARG, "duplicate child");
    }
    HNode n;
    n.kind = N_LIST;
    for (uint32_t i = 0; i < n_children; i++) n.children.push_back(take_child(s, children[i]));
    *id = push_node(s, std::move(n));
  });
}

hrt_status hrt_node_bvh(hrt_scene* s, const uint32_t* children, uint32_t n_children, float t0,
                        float t1, uint32_t* id) {
  return guard([&] {
    mutable_scene(s);
    need(id != nullptr && (children != nullptr || n_children == 0), HRT_ERR_INVALID_ARG, "null argument");
    std::vector<uint32_t> objs;
    for (uint32_t i = 0; i < n_children; i++) {
      need(children[i] < s->nodes.size(), HRT_ERR_INVALID_ARG, "bad node id");
      need(!s->nodes[children[i]].owned, HRT_ERR_INVALID_ARG, "node already owned by another node");
      for (uint32_t j = 0; j < i; j++) need(children[j] != children[i], HRT_ERR_INVALID_ARG, "duplicate child");
      objs.push_back(children[i]);
    }
    size_t before = s->nodes.size();
    try {
      uint32_t root = build_bvh(s, objs, t0, t1);
      for (uint32_t c : objs) s->nodes[c].owned = true;
      *id = root;
    } catch (...) {
      s->nodes.resize(before); /* leave the scene as it was */
      throw;
    }
  });
}

hrt_status hrt_node_count(const hrt_scene* s, uint32_t node, uint32_t* out) {
  return guard([&] {
    need(s && out && node < s->nodes.size(), HRT_ERR_INVALID_ARG, "bad argument");
    *out = count(s, node);
  });
}

hrt_status hrt_node_bounding_box(const hrt_scene* s, uint32_t node, float t0, float t1,
                                 int32_t* has_box, float bmin[3], float bmax[3]) {
  return guard([&] {
    need(s && has_box && bmin && bmax && node < s->nodes.size(), HRT_ERR_INVALID_ARG, "bad argument");
    Aabb b;
    *has_box = bbox(s, node, t0, t1, b) ? 1 : 0;
    if (*has_box)
      for (int a = 0; a < 3; a++) { bmin[a] = b.mn[a]; bmax[a] = b.mx[a]; }
  });
}

hrt_status hrt_scene_set_options(hrt_scene* s, const hrt_scene_options* o) {
  return guard([&] {
    mutable_scene(s);
    need(o != nullptr, HRT_ERR_INVALID_ARG, "hrt_scene_set_options: null options");
    need(o->bvh_ties <= 1 && o->walk_tree <= 1 && o->chunk_uniform <= 1, HRT_ERR_INVALID_ARG,
         "hrt_scene_set_options: bvh_ties, walk_tree and chunk_uniform are 0 or 1");
    s->opts = *o;
  });
}

hrt_status hrt_scene_set_view(hrt_scene* s, const hrt_camera* view) {
  return guard([&] {
    mutable_scene(s);
    s->has_view = view != nullptr;
    s->view = view ? *view : hrt_camera{};
  });
}

hrt_status hrt_scene_get_options(const hrt_scene* s, hrt_scene_options* o) {
  return guard([&] {
    need(s && o, HRT_ERR_INVALID_ARG, "hrt_scene_get_options: null argument");
    *o = s->opts;
  });
}

hrt_status hrt_scene_set_root(hrt_scene* s, uint32_t node) {
  return guard([&] {
    mutable_scene(s);
    need(node < s->nodes.size(), HRT_ERR_INVALID_ARG, "bad node id");
    need(!s->nodes[node].owned, HRT_ERR_INVALID_ARG, "root is owned by another node");
    s->root = node;
  });
}

hrt_status hrt_scene_commit(hrt_scene* s, int32_t device) {
  hrt_status st = guard([&] {
    mutable_scene(s);
    need(s->root != G::NONE, HRT_ERR_STATE, "no root set");
    s->commit_knobs = knobs_in_effect(); /* what the walk builders and the upload read */
    flatten(s);
  });
  if (st != HRT_OK) return st;
  st = device_upload(s, device);
  if (st == HRT_OK) s->committed = true;
  return st;
}

hrt_status hrt_scene_get_info(const hrt_scene* s, hrt_scene_info* info) {
  return guard([&] {
    need(s && info, HRT_ERR_INVALID_ARG, "null argument");
    need(s->committed, HRT_ERR_STATE, "scene not committed");
    info->nodes = (uint32_t)s->g_nodes.size();
    info->prims = (uint32_t)s->g_prims.size();
    info->materials = (uint32_t)s->g_mats.size();
    info->textures = (uint32_t)s->g_texs.size();
    info->instances = (uint32_t)s->g_insts.size();
    info->media = (uint32_t)s->g_media.size();
    info->feature_mask = s->feature_mask;
    info->blob_bytes = (uint32_t)s->blob_bytes;
    /* the default plan (render.hip plan()): sphere scenes stage their walk stream in LDS when it fits */
    info->in_lds = ((s->feature_mask & ~G::F_BASIC) == 0 && s->w_end > 0 && s->w_end <= G::LDS_SCENE_MAX_BYTES) ? 1u
                   : s->w_hot > 0 ? 2u : 0u;
    info->cull_mode = (uint32_t)s->cull_mode;
    info->sah_stream_len = s->f_stream_len;
    info->bvh_tied_sorts = s->bvh_tied_sorts;
    info->walk_regrouped = s->w_regrouped ? 1u : 0u;
    info->walk_device_built = s->w_device_built ? 1u : 0u;
    info->walk_build_us = s->w_build_us;
  });
}

/* Flatten without a device (tests/native/lane_sim.hip runs the kernels' per-lane code on it). */
hrt_status hrt_debug_scene_blob(hrt_scene* s, void* out, uint64_t cap, uint64_t* size, hrt_blob_info* info) {
  return guard([&] {
    need(s && size, HRT_ERR_INVALID_ARG, "bad argument");
    need(s->root != G::NONE, HRT_ERR_STATE, "no root set");
    if (!s->committed) flatten(s);
    std::vector<uint8_t> blob = build_blob(s);
    *size = blob.size();
    if (out) {
      need(cap >= blob.size(), HRT_ERR_INVALID_ARG, "buffer too small");
      memcpy(out, blob.data(), blob.size());
    }
    if (info) {
      memset(info, 0, sizeof(*info));
      info->off_nodes = s->off_nodes; info->off_prims = s->off_prims; info->off_insts = s->off_insts;
      info->off_media = s->off_media; info->off_mats = s->off_mats; info->off_texs = s->off_texs;
      info->off_perlin = s->off_perlin; info->off_images = s->off_images;
      info->n_nodes = (uint32_t)s->g_nodes.size();
      info->main_end = s->main_end;
      info->n_prims = (uint32_t)s->g_prims.size();
      info->feature_mask = s->feature_mask;
      info->cull_mode = (uint32_t)s->cull_mode;
      info->motion_uniform = s->motion_uniform ? 1u : 0u;
      info->motion_t0 = s->motion_t0;
      info->motion_span = s->motion_span;
      info->ln_e = s->ln_e;
      info->media_nested = s->media_nested ? 1u : 0u;
      info->box_t0 = s->box_t0;
      info->box_t1 = s->box_t1;
      info->off_walk = s->off_walk;
      info->walk_bytes = s->w_end;
      info->walk_c16 = s->w_c16 ? 1u : 0u;
      info->walk_nodes = s->w_nodes;
      info->walk_pbase = s->w_pbase;
      info->walk_regrouped = s->w_regrouped ? 1u : 0u;
      info->bvh_tied_sorts = s->bvh_tied_sorts;
      info->walk_hot = s->w_hot;
      info->walk_general = s->w_general ? 1u : 0u;
      info->off_chains = s->off_chains;
      info->walk_half = s->w_half;
    }
  });
}

/* Diagnostics: the flattened record of primitive `index` (order 0: reference pre-order, 1: SAH). */
hrt_status hrt_debug_prim_record(const hrt_scene* s, int32_t order, uint32_t index, float* out12) {
  return guard([&] {
    need(s && out12, HRT_ERR_INVALID_ARG, "bad argument");
    const std::vector<G::Prim>& v = order == 1 ? s->f_prims : s->g_prims;
    need(index < v.size(), HRT_ERR_INVALID_ARG, "prim index out of range (commit first)");
    memcpy(out12, &v[index], sizeof(G::Prim));
  });
}

/* camera.rs:34-83 */
hrt_status hrt_camera_init(hrt_camera* cam, const float from_[3], const float at_[3], float fov,
                           float aperture, float focus_dist, float time0, float time1,
                           int32_t width, int32_t height) {
  return guard([&] {
    need(cam != nullptr, HRT_ERR_INVALID_ARG, "null camera");
    need(width > 0 && height > 0, HRT_ERR_INVALID_ARG, "bad size");
    /* rand's gen_range(time0..time1) panics unless time0 < time1 (camera.rs:93) */
    need(time0 < time1, HRT_ERR_INVALID_ARG, "time0 must be < time1");
    Vec3 from = vin(from_), at = vin(at_);
    float aspect_ratio = (float)width / (float)height;
    float theta = fov * (PI_F / 180.0f); /* f32::to_radians */
    float h = tan_f(theta / 2.0f);
    float viewport_height = 2.0f * h;
    float viewport_width = aspect_ratio * viewport_height;
    Vec3 w = normalize(from - at);
    Vec3 u = normalize(cross(v3(0.0f, 1.0f, 0.0f), w));
    Vec3 v = cross(w, u);
    Vec3 origin = from;
    Vec3 horizontal = (focus_dist * viewport_width) * u;
    Vec3 vertical = (focus_dist * viewport_height) * v;
    Vec3 llc = ((origin - horizontal / 2.0f) - vertical / 2.0f) - focus_dist * w;
    const Vec3* src[7] = {&origin, &llc, &horizontal, &vertical, &u, &v, &w};
    float* dst[7] = {cam->origin, cam->lower_left_corner, cam->horizontal, cam->vertical, cam->u, cam->v, cam->w};
    for (int i = 0; i < 7; i++) { dst[i][0] = src[i]->x; dst[i][1] = src[i]->y; dst[i][2] = src[i]->z; }
    cam->lens_radius = aperture / 2.0f;
    cam->time0 = time0;
    cam->time1 = time1;
  });
}

/* application.rs:363-364 (tile counts) and :404-430 (tile rectangles).  The reference derives the
 * ragged width with a float formula; integer min() gives the same for every BASELINE size and never
 * drops a column.  Tile i of the grid goes to rank i % world. */
hrt_status hrt_tile_grid(uint32_t width, uint32_t height, uint32_t tile_size, uint32_t rank,
                         uint32_t world, hrt_tile* tiles, uint32_t cap, uint32_t* n) {
  return guard([&] {
    need(n != nullptr && tile_size > 0 && world > 0 && rank < world, HRT_ERR_INVALID_ARG, "bad argument");
    uint32_t tx = (width + tile_size - 1) / tile_size, ty = (height + tile_size - 1) / tile_size;
    uint32_t k = 0;
    for (uint32_t i = 0; i < tx * ty; i++) {
      if (i % world != rank) continue;
      if (tiles && k < cap) {
        uint32_t x = (i % tx) * tile_size, y = (i / tx) * tile_size;
        tiles[k] = hrt_tile{x, y, std::min(tile_size, width - x), std::min(tile_size, height - y)};
      }
      k++;
    }
    *n = k;
  });
}

}  // extern "C"
