/*
 * image_io.cpp — frame output for debugging, fixtures and visual diffs.  The reference
 * has no image writer: Application::render (src/application.rs:451-456) uploads sqrt(sum/spp) RGBA to
 * a GL texture whose row 0 is the bottom of the image (y up, :444-445).  PFM keeps those floats and
 * that row order exactly; PPM is the usual 8-bit view of the same (already gamma-2) values.
 */
#include <cmath>
#include <cstdio>
#include <string>
#include <vector>

#include "hrt/hrt.h"
#include "scene_internal.h"

using namespace hrt;

namespace {
hrt_status fail(hrt_status code, const std::string& msg) {
  set_error(msg);
  return code;
}
}  // namespace

extern "C" hrt_status hrt_image_write(const char* path, const float* rgba, uint32_t w, uint32_t h, int32_t format) {
  if (!path || !rgba || w == 0 || h == 0) return fail(HRT_ERR_INVALID_ARG, "bad argument");
  if (format != HRT_IMAGE_PFM && format != HRT_IMAGE_PPM) return fail(HRT_ERR_INVALID_ARG, "unknown image format");
  FILE* f = fopen(path, "wb");
  if (!f) return fail(HRT_ERR_INVALID_ARG, std::string("cannot open ") + path);
  bool ok = true;
  try {
    if (format == HRT_IMAGE_PFM) {
      /* "PF", size, scale < 0 = little-endian; scanlines bottom to top */
      ok = fprintf(f, "PF\n%u %u\n-1.0\n", w, h) > 0;
      std::vector<float> row(3 * (size_t)w);
      for (uint32_t y = 0; y < h && ok; y++) {
        for (uint32_t x = 0; x < w; x++)
          for (int c = 0; c < 3; c++) row[3 * x + c] = rgba[4 * ((size_t)y * w + x) + c];
        ok = fwrite(row.data(), sizeof(float), row.size(), f) == row.size();
      }
    } else {
      ok = fprintf(f, "P6\n%u %u\n255\n", w, h) > 0;
      std::vector<unsigned char> row(3 * (size_t)w);
      for (uint32_t yy = 0; yy < h && ok; yy++) {
        const uint32_t y = h - 1 - yy; /* PPM rows run top to bottom */
        for (uint32_t x = 0; x < w; x++)
          for (int c = 0; c < 3; c++) {
            float v = rgba[4 * ((size_t)y * w + x) + c];
            v = std::isnan(v) ? 0.0f : (v < 0.0f ? 0.0f : (v > 0.999f ? 0.999f : v));
            row[3 * x + c] = (unsigned char)(256.0f * v);
          }
        ok = fwrite(row.data(), 1, row.size(), f) == row.size();
      }
    }
  } catch (const std::bad_alloc&) {
    fclose(f);
    return fail(HRT_ERR_OOM, "out of host memory");
  }
  ok = (fclose(f) == 0) && ok;
  if (!ok) return fail(HRT_ERR_INVALID_ARG, std::string("write failed: ") + path);
  return HRT_OK;
}
