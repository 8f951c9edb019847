/*
 * render_random.c — the C ABI end to end, no Python or PyTorch: build the reference's random-spheres
 * scene (application.rs:497-565), commit it to GPU 0, render it and write a PPM.
 *
 *   make -C examples && LD_LIBRARY_PATH=hyper-ray-tracer_amd/lib ./examples/render_random 400 225 50 out.ppm
 *
 * A process that uses only libhrt gets the ROCm HIP runtime libhrt was linked against.
 */
#include <stdio.h>
#include <stdlib.h>

#include "hrt/hrt.h"

#define CHECK(call)                                                                  \
  do {                                                                               \
    hrt_status st_ = (call);                                                         \
    if (st_ != HRT_OK) {                                                             \
      fprintf(stderr, "%s failed (status %d): %s\n", #call, (int)st_, hrt_last_error()); \
      return 1;                                                                      \
    }                                                                                \
  } while (0)

int main(int argc, char** argv) {
  uint32_t w = argc > 1 ? (uint32_t)atoi(argv[1]) : 400;
  uint32_t h = argc > 2 ? (uint32_t)atoi(argv[2]) : 225;
  uint32_t spp = argc > 3 ? (uint32_t)atoi(argv[3]) : 50;
  const char* out = argc > 4 ? argv[4] : "random.ppm";

  hrt_scene* s = NULL;
  hrt_preset_info info;
  CHECK(hrt_scene_create(&s));
  CHECK(hrt_preset_build(s, HRT_PRESET_RANDOM, 1, NULL, 0, 0, 0, &info));
  CHECK(hrt_scene_commit(s, 0));

  hrt_camera cam;
  CHECK(hrt_camera_init(&cam, info.look_from, info.look_at, info.fov, info.aperture, info.focus_dist, info.time0, info.time1,
                        (int32_t)w, (int32_t)h));
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

  float* rgba = (float*)malloc(sizeof(float) * 4 * (size_t)w * h);
  hrt_render_stats stats;
  if (!rgba) return 1;
  CHECK(hrt_render(s, &cam, &p, 0, 0, w, h, rgba, &stats));
  CHECK(hrt_image_write(out, rgba, w, h, HRT_IMAGE_PPM));
  printf("%ux%u, %u spp: %llu rays (world.hit calls), %llu samples -> %s\n", w, h, spp,
         (unsigned long long)stats.segments, (unsigned long long)stats.samples, out);
  free(rgba);
  hrt_scene_destroy(s);
  return 0;
}
