/*
 * hrt.h — the drop-in C ABI of the MI355X path-tracing inner loop (libhrt.so).
 *
 * What it replaces (reference = SkillerRaptor/hyper-ray-tracer, a Rust crate with no FFI of its own):
 *   - the trait surface the scene builders construct (src/hittable/mod.rs:19-25 `Hittable`,
 *     src/materials/mod.rs:15-19 `Material`, src/textures/mod.rs:14-16 `Texture`): a GPU cannot call
 *     back into trait objects per ray, so each concrete type gets a constructor here that records a
 *     lowered description (the additive `lower()` a Rust binding adds to each type);
 *   - `Application::render` (src/application.rs:393-475) + `ray_color` (:477-495): the per-tile,
 *     per-pixel, per-sample loop, which becomes hrt_render / hrt_render_tiles_device (one persistent
 *     HIP megakernel launch for a whole tile set);
 *   - `Camera::new`/`resize` (src/camera.rs:34-83): hrt_camera_init.
 *
 * Conventions
 *   - Every function returns hrt_status (0 = OK) and never unwinds; the reference's panics (empty BVH
 *     bvh_node.rs:38, NaN bbox bvh_node.rs:31/76, missing image image_texture.rs:20, gen_range with
 *     lo >= hi) become status codes.  hrt_last_error() returns a thread-local message.
 *   - Ids returned through uint32_t* are indices into the scene's texture / material / node tables.
 *     Inputs (Perlin tables, image bytes, child lists) are deep-copied during the call.
 *   - A scene is mutable until hrt_scene_commit, immutable afterwards; rendering is re-entrant per
 *     scene (each call uses its own stream-ordered scratch).
 *   - Image layout: pixel (x, y) with y = 0 the BOTTOM row (src/application.rs:444-445); output of a
 *     w*h region is RGBA f32 at index (x-x0) + w*(y-y0), alpha = 1 (src/application.rs:451-456).
 */
#ifndef HRT_HRT_H
#define HRT_HRT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int32_t hrt_status;
enum {
  HRT_OK = 0,
  HRT_ERR_INVALID_ARG = 1, /* bad id, null pointer, bad enum, lo >= hi ... */
  HRT_ERR_EMPTY = 2,       /* BvhNode::new with no objects (bvh_node.rs:38) */
  HRT_ERR_NO_BBOX = 3,     /* object without bounding box inside a BVH (bvh_node.rs:42,79) */
  HRT_ERR_NAN = 4,         /* NaN in a bounding box / sort key (bvh_node.rs:31,76) */
  HRT_ERR_STATE = 5,       /* mutation after commit, render before commit, ... */
  HRT_ERR_HIP = 6,         /* HIP runtime error (message in hrt_last_error) */
  HRT_ERR_OOM = 7,
  HRT_ERR_UNSUPPORTED = 8  /* e.g. a ConstantMedium nested inside another medium's boundary */
};

typedef struct hrt_scene hrt_scene;

/* rect.rs:12-17 */
enum { HRT_PLANE_XY = 0, HRT_PLANE_YZ = 1, HRT_PLANE_ZX = 2 };
/* rotation.rs:10-25 */
enum { HRT_AXIS_X = 0, HRT_AXIS_Y = 1, HRT_AXIS_Z = 2 };

/* Camera after Camera::resize (src/camera.rs:16-31, 67-83). */
typedef struct hrt_camera {
  float origin[3];
  float lower_left_corner[3];
  float horizontal[3];
  float vertical[3];
  float u[3], v[3], w[3];
  float lens_radius;
  float time0, time1;
} hrt_camera;

/* Render knobs: src/arguments.rs:23-47 (width/height/samples/depth/tile) + the values the reference
 * hard-codes (background per scene application.rs:132-197, t_min = 0.001 at :482) + the seed that
 * replaces thread_rng.  Pixels are keyed by their index in the FULL width x height image. */
typedef struct hrt_render_params {
  uint32_t width, height;   /* full image (u = (x+xi)/(width-1), application.rs:444); each must lie in
                               [2, 65535] (HRT_ERR_INVALID_ARG otherwise): the camera divisions are
                               computed with host reciprocals proven exact on that range only */
  uint32_t samples;         /* spp (application.rs:443) */
  uint32_t max_depth;       /* ray_color depth (application.rs:478); reference CLI default 10 */
  uint32_t sample_offset;   /* first sample index (0; >0 splits one pixel's samples across jobs) */
  uint32_t flags;           /* HRT_RENDER_* bits */
  float t_min;              /* 0.001 */
  float background[3];
  uint64_t seed;
} hrt_render_params;

/* hrt_render_params.flags */
enum {
  HRT_RENDER_COUNT_WORK = 1, /* instrumented kernel: stats also count node visits / prim tests / texture
                                evaluations (for the algorithmic-bytes model; slower) */
  HRT_RENDER_NO_LDS = 2,     /* keep the scene in global memory even when it fits in LDS (A/B) */
  HRT_RENDER_REFERENCE_CULL = 8, /* aabb.rs's per-axis box test alone (the verbatim reference traversal) */
  HRT_RENDER_FAST_CULL = 16,     /* APPROXIMATE: plain slab culling; differs from the reference on ~1e-7 of
                                    rays (f32 grazing hits the reference accepts outside a box) */
  HRT_RENDER_SAH = 32            /* APPROXIMATE, with FAST_CULL on sphere-only scenes: SAH octant streams
                                    (traversal order changes which of two near-equal f32 hits wins) */
};

/* hrt_image_write formats (the reference only displays its frame) */
enum {
  HRT_IMAGE_PFM = 0, /* float RGB, little-endian, rows bottom to top: the frame bit for bit */
  HRT_IMAGE_PPM = 1  /* 8-bit binary RGB, rows top to bottom, 256 * clamp(c, 0, 0.999) per channel */
};

typedef struct hrt_tile {
  uint32_t x, y, w, h; /* image coordinates, y up */
} hrt_tile;

/* Work counters of one render call (exact, counted on the device). */
typedef struct hrt_render_stats {
  uint64_t segments;        /* world.hit calls == rays (application.rs:482) */
  uint64_t samples;         /* primary samples = pixels * spp */
  uint64_t pixels;
  uint64_t node_visits;     /* HRT_RENDER_COUNT_WORK only: node-stream entries read */
  uint64_t prim_tests;      /* HRT_RENDER_COUNT_WORK only: primitive intersection tests */
  uint64_t tex_evals;       /* HRT_RENDER_COUNT_WORK only: Texture::value evaluations */
  uint64_t walk_slots;      /* HRT_RENDER_COUNT_WORK only: 64 x wave iterations of the node walk
                               (node_visits / walk_slots = SIMD lane utilisation of the walk) */
  uint64_t shade_slots;     /* HRT_RENDER_COUNT_WORK only: 64 x wave passes through shading */
  uint64_t prim_slots;      /* HRT_RENDER_COUNT_WORK only: 64 x wave runs of the batched leaf-test block
                               (walk kernels; 0 for the segment kernels) */
  uint64_t phase_cycles[3]; /* HRT_RENDER_COUNT_WORK, walk kernels: shader cycles summed over
                               waves spent in [0] work claim + sample start, [1] walk, [2] shading */
  uint64_t park_slots;      /* HRT_RENDER_COUNT_WORK, walk kernels: lane slots of walk steps spent parked on
                               a leaf (waiting for the batched primitive test) */
  uint64_t wait_slots;      /* ... spent with the walk done, waiting for the wave to leave the walk and shade */
  uint64_t leaf_cycles;     /* HRT_RENDER_COUNT_WORK, walk kernels: the part of phase_cycles[1] spent in the batched
                               leaf tests (sphere tests / leaf programs) */
  uint64_t walk_steps;      /* HRT_RENDER_COUNT_WORK, walk kernels: lane slots of the walk loop that stepped a node
                               (walk_steps / walk_slots = the walk's SIMD lane utilisation; node_visits also counts
                               the nodes leaf programs test) */
} hrt_render_stats;

/* Scene description of one reference preset (application.rs:132-211). */
typedef struct hrt_preset_info {
  float look_from[3];
  float look_at[3];
  float fov;
  float aperture;
  float focus_dist;
  float time0, time1;
  float background[3];
  uint32_t root;
} hrt_preset_info;

/* Reference scenes (src/arguments.rs:9-19) + build-defined benchmark scenes. */
enum {
  HRT_PRESET_RANDOM = 0,             /* application.rs:497-565 (BASELINE configs 1, 2) */
  HRT_PRESET_TWO_SPHERES = 1,        /* :567-587 */
  HRT_PRESET_TWO_PERLIN_SPHERES = 2, /* :589-602 */
  HRT_PRESET_EARTH = 3,              /* :604-612 */
  HRT_PRESET_SIMPLE_LIGHT = 4,       /* :614-637 */
  HRT_PRESET_CORNELL = 5,            /* :639-721 (config 5) */
  HRT_PRESET_CORNELL_SMOKE = 6,      /* :723-815 */
  HRT_PRESET_FINAL = 7,              /* :817-935 */
  HRT_PRESET_EARTH_PERLIN = 8,       /* config 3: earth (0,2,0) r2 over the Perlin ground of :589-602 */
  HRT_PRESET_RANDOM_10K = 9,         /* config 4: :511-545 with a, b in [-50, 50) */
  HRT_PRESET_FEATURES = 10,          /* X/Z rotations, lists, nested instances, media in instances */
  HRT_PRESET_RANDOM_40K = 11,        /* :511-545 with a, b in [-100, 100): 39.9k leaves, so the walk stream's
                                        hierarchy is built on the device by default */
  HRT_PRESET_MOTION = 12,            /* moving spheres with their own shutter intervals (moving_sphere.rs:53-58
                                        per sphere: no scene-wide motion factor), a sphere-kernel scene */
  HRT_PRESET_COUNT = 13
};

const char* hrt_last_error(void);
const char* hrt_version(void);
/* ABI version.  Structs the library writes (hrt_render_stats, hrt_launch_info, hrt_blob_info) have
 * grown between releases with no size field, so a caller built against an older header would be written past
 * its buffers: check hrt_abi_version() == HRT_ABI_VERSION once before any other call, and rebuild on a mismatch.
 *   6: hrt_abi_version; hrt_launch_info.knobs is the launch's snapshot, commit-time knobs as "commit:NAME=value"
 *   5: hrt_launch_info.knobs (+256 B), hrt_render_stats.walk_steps, hrt_blob_info walk_c16/walk_nodes/walk_pbase,
 *      hrt_scene_options, hrt_scene_set_view, hrt_debug_sample_chunks */
#define HRT_ABI_VERSION 6u
uint32_t hrt_abi_version(void);

/* ---- scene lifetime ---- */
hrt_status hrt_scene_create(hrt_scene** out);
void hrt_scene_destroy(hrt_scene* scene);

/* ---- textures (src/textures/) ---- */
hrt_status hrt_tex_solid(hrt_scene* s, float r, float g, float b, uint32_t* id);
hrt_status hrt_tex_checker(hrt_scene* s, uint32_t odd, uint32_t even, uint32_t* id);
/* ranvec: 256*3 f32 unit vectors; perm: 3*256 u32 (x, y, z permutations), perlin_noise.rs:14-19 */
hrt_status hrt_tex_noise(hrt_scene* s, float scale, const float* ranvec, const uint32_t* perm,
                         uint32_t* id);
/* Decoded image bytes (image_texture.rs:19-33); data may be NULL/empty -> magenta (:37-39). */
hrt_status hrt_tex_image(hrt_scene* s, const uint8_t* data, uint32_t width, uint32_t height,
                         uint32_t components, uint32_t* id);

/* ---- materials (src/materials/) ---- */
hrt_status hrt_mat_lambertian(hrt_scene* s, uint32_t albedo_tex, uint32_t* id);
hrt_status hrt_mat_metal(hrt_scene* s, float r, float g, float b, float fuzz, uint32_t* id);
hrt_status hrt_mat_dielectric(hrt_scene* s, float index_of_refraction, uint32_t* id);
hrt_status hrt_mat_diffuse_light(hrt_scene* s, uint32_t emit_tex, uint32_t* id);
hrt_status hrt_mat_isotropic(hrt_scene* s, uint32_t albedo_tex, uint32_t* id);

/* ---- hittables (src/hittable/) ---- */
hrt_status hrt_node_sphere(hrt_scene* s, const float center[3], float radius, uint32_t mat,
                           uint32_t* id);
hrt_status hrt_node_moving_sphere(hrt_scene* s, const float center0[3], const float center1[3],
                                  float time0, float time1, float radius, uint32_t mat,
                                  uint32_t* id);
hrt_status hrt_node_rect(hrt_scene* s, int32_t plane, float a0, float a1, float b0, float b1,
                         float k, uint32_t mat, uint32_t* id);
hrt_status hrt_node_cuboid(hrt_scene* s, const float box_min[3], const float box_max[3],
                           uint32_t mat, uint32_t* id);
hrt_status hrt_node_translate(hrt_scene* s, uint32_t child, const float displacement[3],
                              uint32_t* id);
hrt_status hrt_node_rotate(hrt_scene* s, int32_t axis, uint32_t child, float angle_degrees,
                           uint32_t* id);
/* The medium's isotropic phase texture is given as a texture id (constant_medium.rs:22-29). */
hrt_status hrt_node_constant_medium(hrt_scene* s, uint32_t boundary, float density,
                                    uint32_t albedo_tex, uint32_t* id);
hrt_status hrt_node_list(hrt_scene* s, const uint32_t* children, uint32_t n, uint32_t* id);
/* BvhNode::new(objects, t0, t1) (bvh_node.rs:27-63): built immediately, consumes the children. */
hrt_status hrt_node_bvh(hrt_scene* s, const uint32_t* children, uint32_t n, float time0,
                        float time1, uint32_t* id);
/* Hittable::count (hittable/mod.rs:24) and bounding_box (:22). has_box = 0 when None. */
hrt_status hrt_node_count(const hrt_scene* s, uint32_t node, uint32_t* count);
hrt_status hrt_node_bounding_box(const hrt_scene* s, uint32_t node, float time0, float time1,
                                 int32_t* has_box, float box_min[3], float box_max[3]);

/* Scene options: explicit configuration, as the reference takes its configuration as arguments
 * (src/arguments.rs:23-47); the library reads nothing that can change an image from the environment.
 * All-zero is the default.  Set before the nodes they affect (bvh_ties: hrt_node_bvh and the preset
 * builders; everything else: hrt_scene_commit and the renders); after commit, HRT_ERR_STATE. */
typedef struct hrt_scene_options {
  uint32_t bvh_ties;       /* 0: BvhNode::new's equal sort keys in stable order; 1: each run of ties reversed
                              (another order Rust's sort_unstable_by may produce, bvh_node.rs:34) */
  uint32_t walk_tree;      /* 0: the walk's hierarchy re-grouped over the reference leaf order; 1: the reference
                              BvhNode tree itself (same image bit for bit) */
  uint32_t chunk_min;      /* sample chunks (a pixel's samples summed in chunks, then the chunk sums in chunk
                              order): smallest chunk, 0 = the scene class's default */
  uint32_t chunk_max;      /* at most this many head chunks, 0 = default */
  uint32_t chunk_uniform;  /* 1: no halving tail chunks */
} hrt_scene_options;
hrt_status hrt_scene_set_options(hrt_scene* s, const hrt_scene_options* options);
hrt_status hrt_scene_get_options(const hrt_scene* s, hrt_scene_options* options);
/* Placement hint (no reference counterpart; never changes an image's bits): the camera most renders of this
 * scene will use (NULL: none, the default).  A walk stream too large for LDS keeps part of its node parts in
 * LDS and reads the rest from global memory; with a view, hrt_scene_commit stages the node parts that camera
 * rays through a 128 x 128 grid of the view's image plane visit most instead of those
 * under the largest boxes.  Any placement renders the same image bit for bit.  Before commit (HRT_ERR_STATE
 * after). */
hrt_status hrt_scene_set_view(hrt_scene* s, const hrt_camera* view);

hrt_status hrt_scene_set_root(hrt_scene* s, uint32_t node);
/* Flatten + upload to HIP device `device` (-1: the calling thread's current device). */
hrt_status hrt_scene_commit(hrt_scene* s, int32_t device);

/* Reference scene builders (application.rs:497-935) driven by a seeded stream in place of
 * thread_rng.  `image` feeds the Earth texture (earthmap.jpg decoded by the caller, or synthetic). */
hrt_status hrt_preset_build(hrt_scene* s, int32_t preset, uint64_t scene_seed, const uint8_t* image,
                            uint32_t image_w, uint32_t image_h, uint32_t image_c,
                            hrt_preset_info* info);

/* Camera::new + resize (camera.rs:34-83). */
hrt_status hrt_camera_init(hrt_camera* cam, const float look_from[3], const float look_at[3],
                           float fov_degrees, float aperture, float focus_dist, float time0,
                           float time1, int32_t width, int32_t height);

/* ---- rendering ---- */
/* Render `n_tiles` tiles into device memory d_rgba (tiles packed back to back, tile i at
 * 4 * sum_{j<i} w_j*h_j floats; each tile row-major with y up).  Asynchronous on `stream`
 * (a hipStream_t, NULL = default stream).  stats (optional, host pointer) is filled after an
 * internal stream synchronisation when non-NULL.
 * Errors of the launch itself: with stats, HRT_ERR_STATE when the walk watchdog stopped walks that
 * could not end (corrupt scene data; the frame is incomplete).  Without stats the call returns before
 * the kernel ends; such a launch is then reported as HRT_ERR_STATE by the first later call on the
 * scene that finds it finished (the next hrt_render_* call, or hrt_scene_synchronize). */
hrt_status hrt_render_tiles_device(hrt_scene* s, const hrt_camera* cam, const hrt_render_params* p,
                                   const hrt_tile* tiles, uint32_t n_tiles, float* d_rgba,
                                   void* stream, hrt_render_stats* stats);
/* Wait for every render launched on the scene; HRT_ERR_STATE if one of them did not complete its
 * frame (walk watchdog) and no earlier call has reported it. */
hrt_status hrt_scene_synchronize(hrt_scene* s);
/* One delivered tile (application.rs:45-52 Tile): tile-grid indices (pixel origin = index * tile_size),
 * size in pixels, and RGBA f32 pixels row-major in the tile (row 0 = bottom).  `pixels` is valid only
 * during the callback. */
typedef struct hrt_tile_pixels {
  uint32_t x, y;
  uint32_t width, height;
  const float* pixels;
} hrt_tile_pixels;
typedef void (*hrt_tile_fn)(const hrt_tile_pixels* tile, void* user);
/* Application::render with progressive delivery (application.rs:393-475 + the mpsc receive of
 * :284-306): this rank's tiles of the hrt_tile_grid(width, height, tile_size, rank, world) grid are
 * rendered in launches of `batch` tiles; each finished batch is copied back and passed to `fn` tile by
 * tile (grid order) while the next batch renders.  Pixels are those of hrt_render on the same tile. */
hrt_status hrt_render_progressive(hrt_scene* s, const hrt_camera* cam, const hrt_render_params* p,
                                  uint32_t tile_size, uint32_t rank, uint32_t world, uint32_t batch,
                                  hrt_tile_fn fn, void* user, hrt_render_stats* stats);
/* One region into device memory. */
hrt_status hrt_render_device(hrt_scene* s, const hrt_camera* cam, const hrt_render_params* p,
                             uint32_t x0, uint32_t y0, uint32_t w, uint32_t h, float* d_rgba,
                             void* stream, hrt_render_stats* stats);
/* One region into caller-owned host memory (w*h*4 floats); synchronous. */
hrt_status hrt_render(hrt_scene* s, const hrt_camera* cam, const hrt_render_params* p, uint32_t x0,
                      uint32_t y0, uint32_t w, uint32_t h, float* rgba_out, hrt_render_stats* stats);

/* Reference tile grid (application.rs:363-364, 404-430 with integer ragged edges) and its
 * round-robin split across `world` ranks: writes up to `cap` tiles of rank `rank`; *n = count. */
hrt_status hrt_tile_grid(uint32_t width, uint32_t height, uint32_t tile_size, uint32_t rank,
                         uint32_t world, hrt_tile* tiles, uint32_t cap, uint32_t* n);

/* ---- diagnostics ---- */
/* Device occupancy / layout facts of the committed scene (for DESIGN/bench). */
typedef struct hrt_scene_info {
  uint32_t nodes, prims, materials, textures, instances, media;
  uint32_t feature_mask;
  uint32_t blob_bytes;     /* device bytes of the flattened scene */
  uint32_t in_lds;         /* 1 if the megakernel stages the scene in LDS, 2 if only its top levels */
  uint32_t cull_mode;      /* default culling: 2 = exact (reference test + provably safe extra culling) */
  uint32_t sah_stream_len; /* >0: sphere-only scene with the SAH octant streams (8 x this many nodes) */
  /* BvhNode::new sorts of more than 20 objects with equal keys (bvh_node.rs:34): Rust's sort_unstable_by
   * may order such ties differently from this build's stable sort (below 21 objects both are an
   * insertion sort), so 0 means the BVH topology is the reference's for any Rust version */
  uint32_t bvh_tied_sorts;
  uint32_t walk_regrouped; /* sphere scenes: the walk stream's inner boxes are re-grouped (layout.h) */
  uint32_t walk_device_built; /* ... by the device-side build (HRT_WALK_BUILD) */
  uint32_t walk_build_us;  /* the re-grouping's time, host or device (us) */
} hrt_scene_info;
hrt_status hrt_scene_get_info(const hrt_scene* s, hrt_scene_info* info);
/* The last render launch the calling thread made (thread-local, like hrt_last_error): the kernel, its
 * persistent grid and the occupancy answer it was sized by (hipOccupancyMaxActiveBlocksPerMultiprocessor),
 * and the kernel's registers, scratch and LDS (hipFuncGetAttributes), so that a measurement records what
 * ran.  HRT_ERR_STATE before the thread's first launch. */
typedef struct hrt_launch_info {
  char kernel[160];        /* the kernel and its template arguments */
  uint32_t grid, block;    /* workgroups launched, threads per workgroup */
  uint32_t blocks_per_cu;  /* resident workgroups per CU (the occupancy answer) */
  uint32_t cus;            /* compute units of the device */
  uint32_t waves_per_simd; /* blocks_per_cu * block / 64 / 4 */
  uint32_t vgprs;          /* registers per lane */
  uint32_t scratch_bytes;  /* private (scratch) bytes per lane: register spills and stack */
  uint32_t lds_bytes;      /* dynamic LDS per workgroup */
  char knobs[256];         /* the library's A/B environment knobs set in this process ("NAME=value;..."; empty:
                              none).  None of them changes an image's bits (hrt_scene_options does that) */
} hrt_launch_info;
hrt_status hrt_last_launch(hrt_launch_info* out);
/* Write an RGBA f32 frame (w x h, row-major, row 0 = image y 0 = bottom, as the render calls produce;
 * alpha is dropped) to `path` in an HRT_IMAGE_* format. */
hrt_status hrt_image_write(const char* path, const float* rgba, uint32_t w, uint32_t h, int32_t format);
/* Trace ONE path (pixel x,y of the full image; sample index) on the device with the traversal the
 * renderer would use for these params; out[9*i .. 9*i+8] = origin, direction, time, closest t,
 * winner id (bits) of segment i; out[9*max_segments .. +2] = the path's radiance. */
hrt_status hrt_debug_trace_path(hrt_scene* s, const hrt_camera* cam, const hrt_render_params* p, uint32_t x,
                                uint32_t y, uint32_t sample, uint32_t max_segments, float* out,
                                uint32_t* n_segments);
/* The flattened scene as the kernels see it (layout.h sections inside one blob), for host-side
 * inspection and for tests/native/lane_sim.hip, which runs the kernels' per-lane code on the host.
 * Flattens the scene if needed (no device involved; the scene stays mutable unless committed).
 * Call with out == NULL to get the size.  Offsets are byte offsets into the blob. */
typedef struct hrt_blob_info {
  uint64_t off_nodes, off_prims, off_insts, off_media, off_mats, off_texs, off_perlin, off_images;
  uint32_t n_nodes;        /* node-stream entries: main stream + medium boundary subtrees */
  uint32_t main_end;       /* end of the main stream */
  uint32_t n_prims;
  uint32_t feature_mask;
  uint32_t cull_mode;      /* the default culling (layout.h CULL_*) */
  uint32_t motion_uniform; /* every moving sphere shares time0 / time1 */
  float motion_t0, motion_span;
  float ln_e;
  uint32_t media_nested;   /* a ConstantMedium inside a Translation/Rotation */
  float box_t0, box_t1;    /* ray times the BVH boxes are valid for */
  uint64_t off_walk;       /* sphere scenes: the walk stream of the default (exact) sphere kernel */
  uint32_t walk_bytes;     /* its size (0: not a sphere scene) */
  uint32_t walk_regrouped; /* its inner boxes re-grouped over the reference leaf order */
  uint32_t bvh_tied_sorts; /* as hrt_scene_info */
  uint32_t walk_hot;       /* > 0: the walk stream's first walk_hot bytes are staged in LDS, the rest is read
                            * from global memory (streams beyond the LDS budget) */
  uint32_t walk_general;   /* 1: the walk stream is the general-scene stream (leaf programs, render_gwalk_kernel);
                            * 0: the sphere-scene stream (render_basic_kernel) */
  uint64_t off_chains;     /* every instance's transform chain, outermost first (layout.h CHAIN_F4) */
  uint32_t walk_half;      /* bytes from a walk-stream node part's first 16 B to its second: 16, or the split of
                            * sphere streams staged whole in LDS (layout.h WALK_SPLIT_HALF) */
  uint32_t walk_c16;       /* 1: 16-B node parts (layout.h WALK_C16; hybrid sphere streams): positions are node
                            * indices, the walk ends at walk_nodes, payloads from walk_pbase */
  uint32_t walk_nodes;     /* node parts of the walk stream */
  uint32_t walk_pbase;     /* walk_c16: byte offset of the payloads */
} hrt_blob_info;
hrt_status hrt_debug_scene_blob(hrt_scene* s, void* out, uint64_t cap, uint64_t* size, hrt_blob_info* info);
/* The sample chunks a render of these params would use (no device involved; an uncommitted scene is flattened
 * without its walk streams, which the schedule does not depend on):
 * out[0] = chunk size, out[1] = head chunks, out[2] = samples of the first chunk, out[3] = halving tail chunks.
 * A pixel's samples are summed chunk by chunk and the chunk sums added in chunk order, so this schedule is
 * what fixes the image's bits beyond the paths themselves (hrt_scene_options chunk_*). */
hrt_status hrt_debug_sample_chunks(hrt_scene* s, const hrt_render_params* p, uint32_t* out4);
/* Overwrite n bytes of the committed scene's DEVICE blob at byte `offset` (hrt_blob_info offsets), after
 * a device synchronisation.  Fault injection for the watchdog test (e.g. a skip link pointing back). */
hrt_status hrt_debug_poke_blob(hrt_scene* s, uint64_t offset, const void* data, uint64_t n);
/* The flattened 48-byte record of a primitive (order 0: reference pre-order, 1: SAH streams). */
hrt_status hrt_debug_prim_record(const hrt_scene* s, int32_t order, uint32_t index, float* out12);
/* Evaluate the shared deterministic math on the DEVICE (op: 0 sin, 1 cos, 2 acos, 3 atan2, 4 ln,
 * 5 pow5, 6 tan, 7 the walk's division x / y, 8 / 9 the saturating casts `as i32` / `as u32` with the
 * integer's bits in out) for n inputs; used by the GPU KAT test to prove host/device bit identity. */
hrt_status hrt_debug_device_math(int32_t op, const float* x, const float* y, float* out, uint32_t n);
/* The walk's inflated box test (CULL_EXACT's culling half, lane.h box_ce; form 0: sub/mul/add, 1: the fused
 * o*inv form) on every (box, ray) pair, on the DEVICE (on_device = 1: the calling thread's current HIP device) or with the same code compiled for
 * the host (0): boxes n_boxes x 8 floats (C.xyz, -, E.xyz, -), rays n_rays x 6 floats (origin, direction),
 * out[b * n_rays + q] = 1 if box b passes for ray q on [tmin, tmax].  Used by the GPU test that holds the
 * device's culling decisions to the host's bit for bit. */
hrt_status hrt_debug_box_test(int32_t form, int32_t on_device, const float* boxes, uint32_t n_boxes, const float* rays,
                              uint32_t n_rays, float tmin, float tmax, uint8_t* out);

#ifdef __cplusplus
}
#endif
#endif /* HRT_HRT_H */
