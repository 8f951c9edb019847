/*
 * scene_internal.h — host-side scene graph (what the hrt_* constructors record) and the flattened,
 * device-ready form produced by hrt_scene_commit.  Shared by scene.cpp (host) and render.hip.
 */
#pragma once
#include <hrt/hd_math.h>
#include <hrt/hrt.h>

#include <string>
#include <vector>

#include "layout.h"

namespace hrt {
namespace host {

struct Aabb {
  Vec3 mn, mx;
};

enum NodeKind { N_SPHERE, N_MOVING, N_RECT, N_CUBOID, N_TRANSLATE, N_ROTATE, N_MEDIUM, N_LIST, N_BVH };

struct HNode {
  NodeKind kind;
  /* spheres */
  Vec3 c0{}, c1{};
  float t0 = 0, t1 = 0, r = 0;
  uint32_t mat = gpu::NONE;
  /* rect */
  int plane = 0;
  float a0 = 0, a1 = 0, b0 = 0, b1 = 0, k = 0;
  /* cuboid / bvh box */
  Aabb box{};
  bool has_box = false; /* rotation: bbox computed at construction; bvh: always */
  /* translate / rotate */
  Vec3 disp{};
  int axis = 0;
  float sin_t = 0, cos_t = 1;
  /* medium */
  float neg_inv_density = 0;
  uint32_t tex = gpu::NONE;
  uint32_t medium_id = 0;
  /* children: list / cuboid sides / bvh (1 = leaf, 2 = left,right) / translate, rotate, medium (1) */
  std::vector<uint32_t> children;
  bool owned = false; /* already a child of another node (Box<dyn Hittable> ownership) */
};

struct HTex {
  uint32_t kind;
  Vec3 color{};
  uint32_t odd = 0, even = 0;
  float scale = 0;
  uint32_t perlin = 0;
  uint64_t img_off = 0;
  uint32_t w = 0, h = 0, c = 0;
};

struct HMat {
  uint32_t kind;
  uint32_t tex = gpu::NONE;
  Vec3 albedo{};
  float fuzz = 0, ior = 0;
};

/* the sphere kernel's walk stream (layout.h): a leaf of the reference stream, and the hierarchy the
 * stream encodes, in pre-order (a node's subtree is [i, end)) */
struct WalkLeaf {
  Aabb box;   /* holds the leaf's geometry (sphere stream: the reference box) */
  bool nobox; /* no such box: the inflated test always passes */
  uint32_t prim;
  /* general stream (layout.h): the leaf's program [begin, end) of the reference stream, and the
   * enclosing BvhNode box a box-less leaf is tested against first */
  uint32_t begin = 0, end = 0;
  bool has_rbox = false;
  Aabb rbox{};
  uint32_t rgroup = 0xFFFFFFFFu; /* the BvhNode (reference-stream index) rbox belongs to: the reference
                                    tests it ONCE before all the leaves it holds (layout.h GL_BOX) */
  uint32_t inst = 0xFFFFFFFFu; /* innermost enclosing instance of a flattened leaf (layout.h GL_INST) */
  uint32_t gflags = 0;         /* layout.h GL_INST | GL_DIR | GL_INV | GL_DD */
};
struct WNode {
  Aabb box;     /* inner: the union of its leaves' boxes */
  int32_t leaf; /* index into the leaf sequence, or -1 for an inner node */
  uint32_t end;
  uint32_t depth;
};

}  // namespace host

/* knobs.cpp: the library's A/B environment knobs (none changes an image's bits).  Every read goes through
 * knob_env; knobs_in_effect lists the set ones as "NAME=value;..." (hrt_last_launch). */
const char* knob_env(const char* name);
std::string knobs_in_effect();
}  // namespace hrt

struct hrt_scene {
  /* ---- host graph ---- */
  std::vector<hrt::host::HNode> nodes;
  std::vector<hrt::host::HTex> texs;
  std::vector<hrt::host::HMat> mats;
  std::vector<hrt::gpu::Perlin> perlin;
  std::vector<uint8_t> images;
  uint32_t root = hrt::gpu::NONE;
  uint32_t bvh_tied_sorts = 0; /* BvhNode::new sorts of > 20 objects with equal keys (hrt_scene_info) */
  uint32_t n_media = 0;
  bool committed = false;
  std::string commit_knobs; /* knobs_in_effect() when hrt_scene_commit ran (placement knobs act there) */
  hrt_scene_options opts{}; /* explicit configuration (hrt_scene_set_options); all-zero = default */
  bool has_view = false;    /* placement hint (hrt_scene_set_view): the camera most renders will use */
  hrt_camera view{};

  /* ---- flattened (valid after commit) ---- */
  std::vector<hrt::gpu::Node> g_nodes;
  std::vector<hrt::gpu::Prim> g_prims;
  std::vector<hrt::gpu::Inst> g_insts;
  std::vector<hrt::gpu::Medium> g_media;
  std::vector<hrt::gpu::Mat> g_mats;
  std::vector<hrt::gpu::Tex> g_texs;
  std::vector<float> g_chains; /* layout.h CHAIN_F4 float4 per instance */
  uint32_t main_end = 0;
  /* SAH fast path (sphere-only scenes, slab culling): 8 pre-order streams of equal length, one per
   * ray-direction octant (near child first), over a reordered copy of the primitives. */
  std::vector<hrt::gpu::Node> f_nodes;
  std::vector<hrt::gpu::Prim> f_prims;
  uint32_t f_stream_len = 0;
  size_t off_fnodes = 0, off_fprims = 0;
  /* sphere-scene walk stream (layout.h; render_basic_kernel under CULL_EXACT): byte records */
  std::vector<float> w_stream;
  uint32_t w_end = 0;        /* bytes */
  uint32_t w_hot = 0;        /* > 0: the stream exceeds the LDS budget; its first w_hot bytes (the top
                              * levels' node parts) are staged in LDS, the rest is read from global memory */
  bool w_regrouped = false;  /* inner boxes re-grouped over the reference leaf order (build_walk) */
  bool w_device_built = false; /* ... by the device-side build (build_walk.hip) */
  bool w_regroup_pending = false; /* re-grouping left to the device build at upload */
  bool w_general = false;    /* the stream is the general-scene walk stream (layout.h; build_gwalk) */
  uint32_t w_half = 16;      /* bytes from a node part's first 16 B to its second (16, or layout.h WALK_SPLIT_HALF) */
  uint32_t w_nodes = 0;      /* node parts of the stream */
  bool w_c16 = false;        /* 16-B node parts (layout.h WALK_C16; hybrid sphere streams) */
  uint32_t w_pbase = 0;      /* w_c16: byte offset of the payloads (payload j at w_pbase + j * WALK_PAYLOAD_BYTES) */
  bool w_generic = true;     /* general stream: a leaf's program is neither GL_ONE nor GL_MED (needs trace_ray) */
  uint32_t w_build_us = 0;   /* time of the re-grouping (host or device) */
  size_t off_walk = 0;
  uint32_t feature_mask = 0;
  int cull_mode = hrt::gpu::CULL_REFERENCE;
  bool all_boxes_ok = true;         /* no NODE_REF_ONLY node (slab culling is geometrically safe) */
  float box_t0 = -3.40282347e+38f;  /* every BVH box is valid for ray times in [box_t0, box_t1] */
  float box_t1 = 3.40282347e+38f;
  float ln_e = 0; /* ln(E) as computed by hd_math (constant_medium.rs:59) */
  bool motion_uniform = false; /* every moving sphere shares (time0, time1 - time0) */
  bool media_nested = false;   /* a ConstantMedium inside a Translation/Rotation */
  float motion_t0 = 0, motion_span = 1;

  /* ---- device ---- */
  int device = -1;
  void* d_blob = nullptr;
  size_t blob_bytes = 0;
  size_t off_nodes = 0, off_prims = 0, off_insts = 0, off_media = 0, off_mats = 0, off_texs = 0,
         off_perlin = 0, off_images = 0, off_chains = 0;
  /* Render scratch slots (allocated at commit, reused round-robin): device [counter | stats |
   * tiles], a pinned host staging copy of the tile list, and the event that marks the end of the
   * slot's last use.  A call waits for its slot's previous use, so calls on any streams are safe. */
  struct Slot {
    void* d_mem = nullptr;
    void* h_tiles = nullptr;
    size_t tiles_cap = 0;
    void* event = nullptr; /* hipEvent_t */
    void* d_partial = nullptr; /* sample-chunk sums [pixels][n_chunks] */
    size_t partial_cap = 0;
    bool used = false;
  };
  static constexpr int N_SLOTS = 4;
  Slot slots[N_SLOTS];
  unsigned next_slot = 0;
  void* slot_mutex = nullptr; /* std::mutex*, owned by render.hip */
  void* out_pool = nullptr;   /* hrt_render's reusable device output buffers (render.hip OutPool) */
};

namespace hrt {
void set_error(const std::string& msg);
/* implemented in render.hip */
hrt_status device_upload(hrt_scene* s, int device);
void flatten_scene(hrt_scene* s);          /* scene.cpp: graph -> layout.h arrays */
void flatten_scene_reference(hrt_scene* s); /* ... without the walk streams (the reference stream and the facts
                                               derived from it: feature mask, main_end) */
std::vector<uint8_t> build_blob(hrt_scene* s); /* scene.cpp: the arrays in one blob; sets s->off_* */
/* scene.cpp: the walk stream's leaves (with the reference hierarchy and whether it may be re-grouped),
 * and the placement + records of a hierarchy over them */
std::vector<host::WalkLeaf> walk_leaves(const hrt_scene* s, std::vector<host::WNode>* ref_tree, bool* regroup_ok);
void walk_place_and_write(hrt_scene* s, const std::vector<host::WNode>& T, const std::vector<host::WalkLeaf>& leaves);
void walk_transcode_c16(hrt_scene* s, uint32_t N);
/* scene.cpp: the general-scene walk stream's leaf objects (layout.h) in the reference's pre-order; a
 * BvhNode box whose reference-stream index is marked in `whole` stays ONE leaf (its subtree the program),
 * and gwalk_leaves_grouped marks every box whose group's box-less leaves would not be contiguous */
std::vector<host::WalkLeaf> gwalk_leaves(const hrt_scene* s, std::vector<host::WNode>* ref_tree, bool* regroup_ok,
                                         const std::vector<char>* whole = nullptr);
std::vector<host::WalkLeaf> gwalk_leaves_grouped(const hrt_scene* s, std::vector<host::WNode>* ref_tree, bool* regroup_ok);
/* build_walk.hip: the re-grouped hierarchy (scene.cpp walk_regroup's splits) built on the device */
void device_walk_regroup(const std::vector<host::WalkLeaf>& leaves, std::vector<host::WNode>& T, int device);
void device_release(hrt_scene* s);
}  // namespace hrt
