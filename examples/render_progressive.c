/*
 * render_progressive.c — the reference's tile pipeline on the C ABI: Application::render's tile tasks
 * (application.rs:393-475) send each finished 80x80 Tile over an mpsc channel, and the main thread
 * receives them and uploads each into the frame's texture at its place (:284-306).  Here
 * hrt_render_progressive renders the tile grid in batches on the GPU and hands every finished tile to
 * `receive`, which does what that receiver does with it: copy its pixels into the frame at
 * (x * TILE, y * TILE) and count it.  The frame is written as an exact PFM.
 *
 *   make -C examples && ./examples/render_progressive 400 225 50 out.pfm
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hrt/hrt.h"

#define TILE 80u /* application.rs:363 */

#define CHECK(call)                                                                       \
  do {                                                                                    \
    hrt_status st_ = (call);                                                              \
    if (st_ != HRT_OK) {                                                                  \
      fprintf(stderr, "%s failed (status %d): %s\n", #call, (int)st_, hrt_last_error());  \
      return 1;                                                                           \
    }                                                                                     \
  } while (0)

typedef struct {
  float* frame; /* the "texture": w x h RGBA f32, row 0 = image y 0 */
  uint32_t w, h;
  uint32_t tiles;
  int bad;
} Receiver;

/* the receiving end of the channel (application.rs:284-306): place the tile, count it */
static void receive(const hrt_tile_pixels* t, void* user) {
  Receiver* r = (Receiver*)user;
  const uint32_t x0 = t->x * TILE, y0 = t->y * TILE;
  if (x0 + t->width > r->w || y0 + t->height > r->h) {
    r->bad = 1;
    return;
  }
  for (uint32_t y = 0; y < t->height; y++)
    memcpy(r->frame + 4 * ((size_t)(y0 + y) * r->w + x0), t->pixels + 4 * (size_t)y * t->width,
           sizeof(float) * 4 * t->width);
  r->tiles++;
}

int main(int argc, char** argv) {
  uint32_t w = argc > 1 ? (uint32_t)atoi(argv[1]) : 400;
  uint32_t h = argc > 2 ? (uint32_t)atoi(argv[2]) : 225;
  uint32_t spp = argc > 3 ? (uint32_t)atoi(argv[3]) : 50;
  const char* out = argc > 4 ? argv[4] : "random.pfm";

  hrt_scene* s = NULL;
  hrt_preset_info info;
  CHECK(hrt_scene_create(&s));
  CHECK(hrt_preset_build(s, HRT_PRESET_RANDOM, 1, NULL, 0, 0, 0, &info));
  CHECK(hrt_scene_commit(s, 0));
  hrt_camera cam;
  CHECK(hrt_camera_init(&cam, info.look_from, info.look_at, info.fov, info.aperture, info.focus_dist, info.time0,
                        info.time1, (int32_t)w, (int32_t)h));
  hrt_render_params p = {0};
  p.width = w;
  p.height = h;
  p.samples = spp;
  p.max_depth = 50;
  p.t_min = 0.001f;
  p.background[0] = info.background[0];
  p.background[1] = info.background[1];
  p.background[2] = info.background[2];
  p.seed = 1;

  Receiver r = {0};
  r.w = w;
  r.h = h;
  r.frame = (float*)calloc(4 * (size_t)w * h, sizeof(float));
  if (!r.frame) return 1;
  uint32_t n_tiles = 0;
  CHECK(hrt_tile_grid(w, h, TILE, 0, 1, NULL, 0, &n_tiles));
  hrt_render_stats stats;
  CHECK(hrt_render_progressive(s, &cam, &p, TILE, 0, 1, 4, receive, &r, &stats));
  if (r.bad || r.tiles != n_tiles) {
    fprintf(stderr, "received %u of %u tiles%s\n", r.tiles, n_tiles, r.bad ? " (one outside the frame)" : "");
    return 1;
  }
  CHECK(hrt_image_write(out, r.frame, w, h, HRT_IMAGE_PFM));
  printf("%ux%u, %u spp: %u tiles received, %llu rays -> %s\n", w, h, spp, r.tiles,
         (unsigned long long)stats.segments, out);
  free(r.frame);
  hrt_scene_destroy(s);
  return 0;
}
