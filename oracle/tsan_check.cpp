/*
 * tsan_check.cpp — TEST INFRASTRUCTURE ONLY: the oracle's thread pools (oracle.cpp render: 80x80 tiles on
 * N workers, as application.rs:404-415 spawns one task per tile; render_rows: row segments) under
 * ThreadSanitizer (`make -C oracle tsan`, scripts/sanitize.sh).  Renders every preset small with 8 threads
 * and checks that the multi-threaded frames equal the one-thread frames bit for bit, so a race would show
 * up either as a TSan report (exit 66) or as a frame difference.
 */
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

extern "C" {
void* oracle_preset_build(int preset, uint64_t seed, const uint8_t* img, uint32_t iw, uint32_t ih, uint32_t ic,
                          float* info);
void oracle_scene_destroy(void* s);
int oracle_render(void* scene, uint32_t W, uint32_t H, uint32_t spp, uint32_t depth, uint32_t sample_offset,
                  uint64_t seed, float t_min, uint32_t x0, uint32_t y0, uint32_t w, uint32_t h, float* out, int nthreads,
                  uint64_t* counters);
int oracle_render_rows(void* scene, uint32_t W, uint32_t H, uint32_t spp, uint32_t depth, uint32_t sample_offset,
                       uint64_t seed, float t_min, const uint32_t* rows, uint32_t n_rows, uint32_t x0, uint32_t w,
                       uint32_t task_w, float* out, int nthreads, uint64_t* counters);
const char* oracle_last_error(void);
}

int main() {
  /* a small RGB8 "earth" so the image-texture presets have an image */
  const uint32_t iw = 64, ih = 32;
  std::vector<uint8_t> img(iw * ih * 3);
  for (size_t i = 0; i < img.size(); i++) img[i] = (uint8_t)((i * 37u) & 255u);
  const uint32_t W = 96, H = 64, spp = 4, depth = 20; /* 2 x 1 tiles of 80 px: the ragged edge too */
  int bad = 0;
  for (int preset = 0; preset <= 12; preset++) {
    if (preset == 11) continue; /* random_40k: large, same code path as random_10k */
    void* s = oracle_preset_build(preset, 1, img.data(), iw, ih, 3, nullptr);
    if (!s) {
      fprintf(stderr, "preset %d: %s\n", preset, oracle_last_error());
      return 1;
    }
    std::vector<float> one(W * H * 4), many(W * H * 4);
    uint64_t c1[16] = {0}, c8[16] = {0};
    if (oracle_render(s, W, H, spp, depth, 0, 3, 0.001f, 0, 0, W, H, one.data(), 1, c1) ||
        oracle_render(s, W, H, spp, depth, 0, 3, 0.001f, 0, 0, W, H, many.data(), 8, c8)) {
      fprintf(stderr, "preset %d: %s\n", preset, oracle_last_error());
      return 1;
    }
    const uint32_t rows[3] = {0, 31, 63};
    std::vector<float> r1(3 * W * 4), r8(3 * W * 4);
    uint64_t d1[16] = {0}, d8[16] = {0};
    oracle_render_rows(s, W, H, spp, depth, 0, 3, 0.001f, rows, 3, 0, W, 16, r1.data(), 1, d1);
    oracle_render_rows(s, W, H, spp, depth, 0, 3, 0.001f, rows, 3, 0, W, 16, r8.data(), 8, d8);
    const bool same = memcmp(one.data(), many.data(), one.size() * 4) == 0 && c1[0] == c8[0] &&
                      memcmp(r1.data(), r8.data(), r1.size() * 4) == 0 && d1[0] == d8[0];
    printf("preset %2d: %llu rays, 1 vs 8 threads %s\n", preset, (unsigned long long)c1[0], same ? "identical" : "DIFFER");
    bad += !same;
    oracle_scene_destroy(s);
  }
  return bad ? 2 : 0;
}
