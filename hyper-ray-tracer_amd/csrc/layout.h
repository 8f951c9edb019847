/*
 * layout.h — the flattened scene as it lives in HBM (one blob per device, uploaded once at commit).
 *
 * The reference scene is an object graph of Box<dyn Hittable> (src/hittable/).  It is lowered into
 *   nodes  : the world tree in DFS PRE-ORDER, 32 B per node (two 16-B loads).  A box node stores its
 *            `skip` = index one past its subtree, so the reference's recursive BvhNode::hit
 *            (bvh_node.rs:104-127: left subtree, then right subtree with the shrunken t_max) is a
 *            stackless loop: box passes -> i+1, box fails -> skip.  Lists/Cuboids are consecutive
 *            PRIM nodes (list.rs:20-31 order), Translation/Rotation are BEGIN/END brackets that
 *            transform / restore the ray, a ConstantMedium is one MEDIUM node whose boundary subtree
 *            is emitted after the main stream ([bstart, bend)).
 *   prims  : sphere / moving sphere / rect records, 48 B.
 *   insts, media, mats, texs, perlin tables, image bytes.
 * Every section is 256-B aligned inside the blob.
 */
#pragma once
#include <stdint.h>

namespace hrt {
/* 0 (A/B build): a one-sphere medium boundary takes the two boundary walks of constant_medium.rs:37-48 in
 * every kernel; the general stream then emits no GL_MED leaves either (scene.cpp), so the build is a clean
 * comparison.  1: both queries from one evaluation of the quadratic (lane.h sphere_pair_at). */
#ifndef HRT_MEDIUM_PAIR
#define HRT_MEDIUM_PAIR 1
#endif

namespace gpu {

constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr int MAX_INST_DEPTH = 8;

/* node kinds (Node.kp >> 24) */
enum : uint32_t {
  K_BOX = 0,        /* BvhNode box: pass -> i+1, fail -> skip */
  K_BOX_PRIM = 1,   /* BvhNode leaf holding one primitive: box, then prim[payload] */
  K_PRIM = 2,       /* primitive without box (List / Cuboid side / root) */
  K_INST_BEGIN = 3, /* Translation / Rotation: transform ray (payload = inst) */
  K_INST_END = 4,   /* restore ray */
  K_MEDIUM = 5,     /* ConstantMedium (payload = medium) */
  K_BOX_LEAF = 6    /* SAH stream leaf: box, then prims [start, start+count) (payload = start | (count-1) << 21) */
};
constexpr uint32_t LEAF_MAX = 4; /* primitives per SAH leaf */
struct alignas(16) Node {
  float mn[3];
  uint32_t skip;
  float mx[3];
  uint32_t kp; /* kind << 24 | payload */
};
static_assert(sizeof(Node) == 32, "node is two dwordx4");

enum : uint32_t { P_SPHERE = 0, P_MOVING = 1, P_RECT = 2 };
/* sphere : p0 = (cx, cy, cz, r)
 * moving : p0 = (c0, r), p1 = (c1 - c0, time_start), p2[0] = time_end - time_start
 *          (both differences are exactly what moving_sphere.rs:55-58 computes per call)
 * rect   : p0 = (a0, a1, b0, b1), p1 = (k, a1 - a0, b1 - b0, 0)
 * km     = kind | plane << 2 | material << 4 */
struct alignas(16) Prim {
  float p0[4];
  float p1[4];
  float p2[2];
  uint32_t parent; /* enclosing instance (NONE at world level) */
  uint32_t km;
};
static_assert(sizeof(Prim) == 48, "prim is three dwordx4");

enum : uint32_t { I_TRANSLATE = 0, I_ROTATE = 1 };
/* Inst.kind = I_* | IF_* flags: what a Rotation's subtree reads of the ray beyond o and d, so that
 * entering and leaving it recompute only that (a Translation leaves the direction, and so 1/d and
 * d.d, unchanged): IF_INV 1/d and the inflated test's widening (box or medium nodes below),
 * IF_DD d.d and RN(1/d.d) (spheres or media below) */
constexpr uint32_t I_KIND_MASK = 0xFFu, IF_INV = 1u << 8, IF_DD = 1u << 9;
struct alignas(16) Inst {
  float d[3];     /* translation displacement */
  float sin_t;    /* rotation */
  float cos_t;
  uint32_t axis;  /* HRT_AXIS_* */
  uint32_t parent;
  uint32_t kind;
};

/* The chain of instance q (what apply_chain applies to reach q's children's frame), outermost first,
 * CHAIN_F4 float4 per instance: [0].x = the number of levels n (bits), [1..n] = each level's
 * transform: Translation (dx, dy, dz, I_TRANSLATE), Rotation (sin, cos, axis, I_ROTATE) (bits in z, w).
 * One record per instance instead of a walk up the parent links: the loads are independent. */
constexpr uint32_t CHAIN_F4 = MAX_INST_DEPTH + 1;

struct alignas(16) Medium {
  float neg_inv_density;
  uint32_t bstart, bend;
  uint32_t mat; /* Isotropic phase function */
  uint32_t medium_id;
  uint32_t parent;
  uint32_t sphere; /* the boundary is ONE sphere / moving sphere primitive (its prim index), else NONE:
                      both boundary queries then come from one evaluation of its quadratic (lane.h) */
  uint32_t pad1;
};

enum : uint32_t { M_LAMBERTIAN = 0, M_METAL = 1, M_DIELECTRIC = 2, M_DIFFUSE_LIGHT = 3, M_ISOTROPIC = 4 };
/* lambertian/diffuse_light/isotropic: tex; metal: a = (albedo, fuzz); dielectric: a[0] = ior */
struct alignas(16) Mat {
  float a[4];
  uint32_t kind, tex;
  uint32_t needs_uv; /* texture tree reads (u, v) (only ImageTexture does) */
  uint32_t pad;
};

enum : uint32_t { T_SOLID = 0, T_CHECKER = 1, T_NOISE = 2, T_IMAGE = 3 };
/* solid: a = color; checker: i0 odd, i1 even; noise: a[0] scale, i0 perlin table;
 * image: i0 byte offset, i1 width, i2 height, i3 components (width == 0 -> magenta) */
struct alignas(16) Tex {
  float a[4];
  uint32_t kind, i0, i1, i2;
  uint32_t i3, pad0, pad1, pad2;
};

/* perm: each axis's permutation twice over (perm[c][256 + i] = perm[c][i]), so perlin_noise.rs:92-94's
 * `(i + di) & 255` for di in {0, 1} is the index (i & 255) + di: the second lattice corner's entry is the next word,
 * one LDS / global read with an immediate offset and no add / mask of its own */
constexpr uint32_t PERM_N = 512;
/* 12 KB, three 4-KB pages: the kernels stage the tables in LDS at 4096-aligned addresses (kernel_common.h
 * stage_perlin), where each permutation word becomes its ranvec entry's address (lane.h perlin_noise_t XADDR) */
constexpr uint32_t PERLIN_LDS_ALIGN = 4096;
struct alignas(16) Perlin {
  float ranvec[256][4];
  uint32_t perm[3][PERM_N];
  uint32_t pad[512];
};
static_assert(sizeof(Perlin) == 3 * PERLIN_LDS_ALIGN, "Perlin tables stage at 4-KB-aligned LDS addresses");

/* tile list entry (device) */
struct alignas(16) TileDev {
  uint32_t x, y, w, h;
  uint32_t bw;        /* ceil(w / 8) */
  uint32_t pad_start; /* first padded work index of this tile */
  uint32_t out_off;   /* first output pixel of this tile */
  uint32_t pad;
};

/* feature bits (scene-wide) */
enum : uint32_t {
  F_MOVING = 1u << 0,
  F_RECT = 1u << 1,
  F_INSTANCE = 1u << 2,
  F_MEDIUM = 1u << 3,
  F_NOISE = 1u << 4,
  F_IMAGE = 1u << 5,
  F_CHECKER = 1u << 6,
  F_LIGHT = 1u << 7,
  F_ISOTROPIC = 1u << 8,
  F_METAL = 1u << 9,
  F_DIELECTRIC = 1u << 10
};
/* what the lean kernel instantiation handles (the BASELINE headline scene needs only these) */
constexpr uint32_t F_BASIC = F_MOVING | F_CHECKER | F_METAL | F_DIELECTRIC;
/* what the sphere kernel's HEAVY instantiation adds under exact culling: noise and image textures on
 * sphere scenes (BASELINE config 3, Earth + Perlin) */
constexpr uint32_t F_HEAVY_TEX = F_NOISE | F_IMAGE;

/* box-culling modes */
enum : int {
  CULL_REFERENCE = 0, /* aabb.rs:20-47 verbatim: each axis tested alone against [t_min, t_max] */
  CULL_SLAB = 1,      /* intervals narrowed across axes: fast, NOT bit-faithful (f32 grazing hits) */
  CULL_EXACT = 2      /* the reference test, plus culling of boxes that no accepted hit can come
                         from: the box inflated by EXACT_MARGIN x its distance misses the ray */
};
/* Bound on how far outside a primitive an f32 hit test of the reference can place an ACCEPTED hit,
 * relative to the distance |oc| from the ray origin: the sphere discriminant's rounding error lets a
 * grazing ray "hit" up to sqrt(32 eps) |oc| (~1.4e-3 |oc|) away from the sphere (sphere.rs:42-46);
 * rect and box arithmetic err by ~1e-7 relative.  The box's L-inf distance D bounds |oc| / sqrt(3).
 * 4e-3 * D covers sqrt(3) * 1.4e-3 * D with a 1.65x margin. */
constexpr float EXACT_MARGIN = 4.0e-3f;
/* Node.kp bit 31: the node's reference box may not contain its geometry (a ZX rect, rect.rs:97-102,
 * below it): only the reference test may cull it. */
constexpr uint32_t NODE_REF_ONLY = 1u << 31;
constexpr uint32_t KIND_MASK = 0x7Fu;

/* ---------------------------------------------------------------- sphere-scene walk stream
 * What render_basic_kernel walks under CULL_EXACT: byte-addressed records built at commit from the
 * reference stream (scene.cpp build_walk).  Same leaves in the same order as the reference's BvhNode
 * tree, so the walk tests the same primitives in the same order with the same closest (DESIGN.md
 * section 4); the inner boxes above them may be re-grouped (any hierarchy whose boxes contain their
 * leaves' boxes gives the same result: the inflated test is conservative for any box that holds the
 * geometry, and the reference test is applied at leaves).
 *   node part (32 B), inner or leaf: float4(C.xyz, skip)  float4(E.xyz, pass)
 *   leaf payload (96 B):  float4(mn.xyz, w)    float4(mx.xyz, radius)      the reference box (aabb.rs)
 *                         float4(c0.xyz, t0)   float4(c1 - c0, t1 - t0)    the sphere (moving_sphere.rs:55-58)
 *                         float4(A.xyz, f)     float4(B.xyz, mw)           its material, inline (shading reads
 *                                                                          no global memory): mw = M_* kind |
 *                                                                          WT_* << 4 | material index << 8;
 *                                                                          A = albedo (WT_SOLID, Metal) or the
 *                                                                          checker's odd colour, B its even
 *                                                                          colour (WT_CHECKER), f = fuzz (Metal)
 *                                                                          or ior (Dielectric); WT_GLOBAL: the
 *                                                                          texture is read from texs (any tree)
 * C, E: centre and half-extent of a box holding the node's box ([C - E, C + E] contains [mn, mx] in
 * real arithmetic: E rounded up), for the inflated test (lane.h box_ce).  CE_FLOOR: max_k E_k >=
 * 2^-12 max_k |C_k| for every box (walk_box.h ce_floored raises E where needed), which bounds the
 * error box_ce's per-ray o inv product adds.  Every link is explicit, so
 * records may be placed anywhere: skip = the node that follows the subtree in pre-order (or the end
 * offset); pass = the first child for an inner node, and (payload | WALK_PEND) for a leaf: the lane
 * parks on the leaf until the wave runs its primitive test (walk_prim), which continues at the
 * successor kept in w = WL_* flags | successor << 2.  A leaf's skip equals that successor (the next node in
 * pre-order after a one-node subtree; tests/test_lane_sim.py checks every stream), so the walk kernels continue
 * a parked lane at the skip they kept from the leaf's step (lane.h walk_box, HRT_KEEP_SKIP).  The walk's winner is the payload's offset.  A leaf
 * without a reference box (a List member: K_PRIM) has C = 0, E = +inf (the inflated test always
 * passes) and WL_NOBOX (no reference test).
 * Placement (scene.cpp walk_place_and_write): a stream within LDS_SCENE_MAX_BYTES is laid out in
 * pre-order with each payload after its node part and staged in LDS whole; a larger one puts the node
 * parts a ray is likeliest to reach first (largest parent box surface first, up to LDS_SCENE_MAX_BYTES:
 * the bytes the kernel stages in LDS, w_hot), then the other node parts in pre-order, then the payloads,
 * in global memory. */
constexpr uint32_t WALK_PEND = 1u << 31;
/* the largest scene a sphere-kernel workgroup stages in LDS: two workgroups per CU share its 160 KiB,
 * each also holding a u32 result slot for each of its (at most 768) threads */
constexpr uint32_t LDS_SCENE_MAX_BYTES = 77u * 1024u;
static_assert(2u * (LDS_SCENE_MAX_BYTES + 768u * 4u) <= 160u * 1024u, "two sphere workgroups per CU");
/* a GENERAL walk stream beyond LDS_SCENE_MAX_BYTES stages this much of its node parts: the general kernel then
 * runs one 1024-thread workgroup per CU (16 waves, the 4 waves/SIMD of two 512-thread ones; render_general.hip
 * BIG) with the node parts a ray is likeliest to reach in LDS, twice the two-workgroup budget */
constexpr uint32_t GWALK_LDS_BIG_BYTES = 152u * 1024u;
static_assert(GWALK_LDS_BIG_BYTES + 1024u * 4u <= 160u * 1024u, "one 1024-thread general workgroup per CU");
/* general streams of at most this many node parts (staged whole in LDS with their reference arrays) are walked
 * by each wave as one packet (render_general.hip PACKET): Cornell 35, Cornell-smoke, simple-light */
constexpr uint32_t GWALK_PACKET_NODES = 128u;
/* sphere streams of at most this many node parts (staged whole in LDS) are walked by each wave as one packet
 * (render_sphere.hip PACKET): Earth + Perlin (C3), Earth, the two-sphere scenes: 3 node parts each */
constexpr uint32_t SPHERE_PACKET_NODES = 15u;
constexpr uint32_t WALK_NODE_BYTES = 32, WALK_PAYLOAD_BYTES = 96;
/* Split node parts (r04, sphere streams staged whole in LDS): a node part's first 16 B (C, skip) at its
 * offset, its second 16 B (E, pass) WALK_SPLIT_HALF bytes further (an immediate offset of the LDS read),
 * so consecutive node parts lie 16 B apart in each half and a 16-lane group of ds_read_b128 spreads over
 * all 16 bank slots (interleaved 32-B parts use 8).  Node parts then occupy [0, 16 N) and
 * [WALK_SPLIT_HALF, WALK_SPLIT_HALF + 16 N); payloads fill the rest (N <= 1024).  Opt-in (HRT_WALK_SPLIT=1):
 * no faster on C2 (14 024 vs 14 038 Mrays/s, profiles/r04g_ab.txt), so the conflicts are not what
 * bounds the step. */
constexpr uint32_t WALK_SPLIT_HALF = 16384;
/* ... and for hybrid sphere streams (r06, opt-in HRT_WALK_SPLIT=1): pages of 2 x 8 KiB, 512 node parts each,
 * first halves then second halves (scene.cpp walk_place_and_write); the staged part ends on a page's second
 * halves, so at most 15 KiB of the 77 KiB budget is left unused */
constexpr uint32_t WALK_SPLIT_HALF_HYB = 8192;
/* 16-B node parts (r05, WALK_C16; hybrid sphere streams, the C4 class; opt-in HRT_WALK_C16=1: measured 8% slower
 * on C4's 1/8 share, the binary16 widening and link decode cost more than twice the staged node parts save):
 * the staged budget holds twice the node parts.  A part is four u32: (C.x | C.y << 16), (C.z | E.x << 16), (E.y | E.z << 16), (skip | pass << 16), C and
 * E in IEEE binary16 (C rounded to nearest, E rounded up after adding C's rounding error, so the part's box
 * holds the 32-B part's box and with it the node's geometry: all the inflated test needs), the links 16-bit
 * node indices: node k's part at byte 16 k, the end = the node count N; pass of a leaf = WALK_C16_LEAF | j, its
 * payload at walk_pbase + j * WALK_PAYLOAD_BYTES (payload records unchanged, their successor field a node
 * index).  Walk positions are node indices; a lane parked on leaf j holds WALK_C16_LEAF | j.  Scenes with more
 * than WALK_C16_MAX nodes or leaves, or coordinates beyond binary16's range, keep the 32-B parts
 * (scene.cpp walk_transcode_c16). */
constexpr uint32_t WALK_C16_MAX = 0x7FFFu, WALK_C16_LEAF = 0x8000u;
constexpr uint32_t WL_MOVING = 1u, WL_NOBOX = 2u;
enum : uint32_t { WT_SOLID = 0, WT_CHECKER = 1, WT_GLOBAL = 2 }; /* inline texture of a leaf's material */

/* ---------------------------------------------------------------- general-scene walk stream
 * What render_gwalk_kernel walks under CULL_EXACT for scenes with rects, instances, media and every
 * texture (scene.cpp build_gwalk).  The node parts are the sphere stream's; the leaves are the LEAF
 * OBJECTS of the reference stream, in its pre-order: the smallest pieces the reference's BvhNode
 * hierarchy hands to a non-BVH hittable -- a BvhNode leaf (K_BOX_PRIM, or a K_BOX whose subtree holds no
 * box outside an instance: an instance chain, a Cuboid, a List, a ConstantMedium), or a box-less List
 * member.  A leaf's PROGRAM is its range [begin, end) of the reference node stream, run by lane.h
 * trace_ray from the world ray (the leaf's own box node first: the reference test at the leaf).  Leaf
 * payload (GWALK_PAYLOAD_BYTES):
 *   float4(begin, end, flags, w)     w = successor << 2 (walk_successor, as in the sphere stream); a GL_ONE
 *                                         leaf holds the node's kind word in place of end (lane.h gwalk_one),
 *                                         a GL_MED leaf its medium
 *   float4(mn.xyz, inst) float4(mx.xyz, group)   GL_BOX: the nearest enclosing BvhNode box of a box-less
 *                                         leaf (world frame; `group` = that node's reference-stream index).
 *                                         The reference tests it once, before all the leaves it holds
 *                                         (List::hit, Translation::hit below one BvhNode leaf), so a lane
 *                                         tests it at the first of them it reaches and keeps the outcome
 *                                         for the rest (lane.h gwalk_leaf_test `gstate`): the closest then is
 *                                         the reference's, since the walk visits leaves in its order
 * Instance chains are flattened: each leaf object inside a Translation / Rotation (a primitive, a Cuboid,
 * a leaf of the instance's own BvhNode) is a leaf of the stream, its box the chain's image of its geometry.
 * The node part's C, E box holds the leaf's geometry (its reference box, or for a transposed ZX rect
 * (G17) that box joined with the rect's true extent; E = +inf when no finite box is known), so the
 * inflated test culls only what cannot hold an accepted hit. */
constexpr uint32_t GWALK_PAYLOAD_BYTES = 48;
/* leaf flags (payload word 2).  A leaf inside a Translation / Rotation chain (GL_INST: the innermost
 * instance in word 7) runs its program in that instance's frame: the world ray through the chain (lane.h
 * apply_chain, the reference's own operations), with 1/d (GL_INV: boxes below) and d.d (GL_DD: spheres
 * below) recomputed when the chain turns the direction (GL_DIR).  Its GL_BOX box is then the nearest
 * world-frame BvhNode box around the chain; boxes inside the instance are tested by the program itself. */
constexpr uint32_t GL_BOX = 1u, GL_INST = 2u, GL_DIR = 4u, GL_INV = 8u, GL_DD = 16u;
/* GL_ONE: the program is ONE primitive node (K_BOX_PRIM or K_PRIM: a BvhNode leaf, a Cuboid side, a List
 * member), run without trace_ray's node loop and kind dispatch (lane.h gwalk_one) */
constexpr uint32_t GL_ONE = 32u;
/* GL_MED: the program is [a ConstantMedium's box node, its K_MEDIUM node] at world level with a one-sphere
 * boundary (Medium.sphere); the payload holds the medium in place of end and the sphere in place of the
 * instance (lane.h gwalk_medium) */
constexpr uint32_t GL_MED = 64u;

}  // namespace gpu
}  // namespace hrt
