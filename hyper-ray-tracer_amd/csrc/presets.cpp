/*
 * presets.cpp — the reference's scene builders (src/application.rs:497-935) and camera presets
 * (:132-211), written against the world.hpp mirror of the trait surface.  `thread_rng()` becomes one
 * seeded stream (hd_math.h scene_rng) consumed in the reference's draw order, so a scene is a pure
 * function of (preset, seed).  Build-defined presets for BASELINE configs 3 and 4 and a feature
 * coverage scene are documented in DESIGN.md.
 */
#include <memory>

#include "world.hpp"

using namespace hrt;
using namespace hrt::world;

namespace {

struct Ctx {
  Rng rand;
  const uint8_t* img;
  uint32_t iw, ih, ic;
};

TextureP solid(float r, float g, float b) { return std::make_shared<SolidColor>(v3(r, g, b)); }
MaterialP lambert(TextureP t) { return std::make_shared<Lambertian>(std::move(t)); }
TextureP image(Ctx& c) { return std::make_shared<ImageTexture>(c.img, c.iw, c.ih, c.ic); }

template <class T, class... A>
HittableP mk(A&&... a) {
  return HittableP(new T(std::forward<A>(a)...));
}

/* application.rs:497-565; n = 11 (the 10k-sphere config 4 uses n = 50) */
HittableP generate_random_scene(Ctx& c, int n) {
  std::vector<HittableP> objects;
  objects.push_back(mk<Sphere>(v3(0.0f, -1000.0f, 0.0f), 1000.0f,
                               lambert(std::make_shared<CheckerTexture>(solid(0.2f, 0.3f, 0.1f),
                                                                        solid(0.9f, 0.9f, 0.9f)))));
  Rng& rand = c.rand;
  for (int a = -n; a < n; a++) {
    for (int b = -n; b < n; b++) {
      float choose_material = rand.gen_f32();
      float cx = (float)a + 0.9f * rand.gen_f32();
      float cz = (float)b + 0.9f * rand.gen_f32();
      Vec3 center = v3(cx, 0.2f, cz);
      if (magnitude(center - v3(4.0f, 0.2f, 0.0f)) > 0.9f) {
        if (choose_material < 0.8f) {
          float r = rand.gen_f32(), g = rand.gen_f32(), bl = rand.gen_f32();
          Vec3 center_2 = center + v3(0.0f, rand.gen_range_f32(0.0f, 0.5f), 0.0f);
          objects.push_back(
              mk<MovingSphere>(center, center_2, 0.0f, 1.0f, 0.2f, lambert(solid(r, g, bl))));
        } else if (choose_material < 0.95f) {
          float r = rand.gen_range_f32(0.5f, 1.0f), g = rand.gen_range_f32(0.5f, 1.0f),
                bl = rand.gen_range_f32(0.5f, 1.0f);
          float fuzz = rand.gen_range_f32(0.0f, 0.5f);
          objects.push_back(mk<Sphere>(center, 0.2f, std::make_shared<Metal>(v3(r, g, bl), fuzz)));
        } else {
          objects.push_back(mk<Sphere>(center, 0.2f, std::make_shared<Dielectric>(1.5f)));
        }
      }
    }
  }
  objects.push_back(mk<Sphere>(v3(0.0f, 1.0f, 0.0f), 1.0f, std::make_shared<Dielectric>(1.5f)));
  objects.push_back(mk<Sphere>(v3(-4.0f, 1.0f, 0.0f), 1.0f, lambert(solid(0.4f, 0.2f, 0.1f))));
  objects.push_back(
      mk<Sphere>(v3(4.0f, 1.0f, 0.0f), 1.0f, std::make_shared<Metal>(v3(0.7f, 0.6f, 0.5f), 0.0f)));
  return mk<BvhNode>(std::move(objects), 0.0f, 1.0f);
}

/* build-defined: the random scene's grid with every sphere moving over its OWN shutter interval
 * (moving_sphere.rs:53-58 divides by each sphere's time1 - time0), so the kernels' scene-wide motion
 * factor does not apply; oracle.cpp preset 12 draws the same numbers in the same order */
HittableP generate_motion(Ctx& c) {
  std::vector<HittableP> objects;
  objects.push_back(mk<Sphere>(v3(0.0f, -1000.0f, 0.0f), 1000.0f,
                               lambert(std::make_shared<CheckerTexture>(solid(0.2f, 0.3f, 0.1f),
                                                                        solid(0.9f, 0.9f, 0.9f)))));
  Rng& rand = c.rand;
  for (int a = -4; a < 4; a++) {
    for (int b = -4; b < 4; b++) {
      const float choose_material = rand.gen_f32();
      const float cx = (float)a + 0.9f * rand.gen_f32();
      const float cz = (float)b + 0.9f * rand.gen_f32();
      const Vec3 center = v3(cx, 0.2f, cz);
      const float t0 = rand.gen_range_f32(-0.5f, 0.5f);
      const float t1 = t0 + rand.gen_range_f32(0.25f, 1.5f);
      const float dx = rand.gen_range_f32(-0.3f, 0.3f), dy = rand.gen_range_f32(0.0f, 0.5f),
                  dz = rand.gen_range_f32(-0.3f, 0.3f);
      const Vec3 center_2 = center + v3(dx, dy, dz);
      MaterialP m;
      if (choose_material < 0.6f) {
        const float r = rand.gen_f32(), g = rand.gen_f32(), bl = rand.gen_f32();
        m = lambert(solid(r, g, bl));
      } else if (choose_material < 0.85f) {
        const float r = rand.gen_range_f32(0.5f, 1.0f), g = rand.gen_range_f32(0.5f, 1.0f),
                    bl = rand.gen_range_f32(0.5f, 1.0f);
        const float fuzz = rand.gen_range_f32(0.0f, 0.5f);
        m = std::make_shared<Metal>(v3(r, g, bl), fuzz);
      } else {
        m = std::make_shared<Dielectric>(1.5f);
      }
      objects.push_back(mk<MovingSphere>(center, center_2, t0, t1, 0.2f, m));
    }
  }
  objects.push_back(mk<Sphere>(v3(0.0f, 1.0f, 0.0f), 1.0f, std::make_shared<Dielectric>(1.5f)));
  objects.push_back(mk<MovingSphere>(v3(-4.0f, 1.0f, 0.0f), v3(-4.0f, 1.5f, 0.0f), 0.0f, 2.0f, 1.0f,
                                     lambert(solid(0.4f, 0.2f, 0.1f))));
  return mk<BvhNode>(std::move(objects), 0.0f, 1.0f);
}

/* :567-587 */
HittableP generate_two_spheres() {
  MaterialP checker =
      lambert(std::make_shared<CheckerTexture>(solid(0.2f, 0.3f, 0.1f), solid(0.9f, 0.9f, 0.9f)));
  std::vector<HittableP> o;
  o.push_back(mk<Sphere>(v3(0.0f, -10.0f, 0.0f), 10.0f, checker));
  o.push_back(mk<Sphere>(v3(0.0f, 10.0f, 0.0f), 10.0f, checker));
  return mk<BvhNode>(std::move(o), 0.0f, 1.0f);
}

/* :589-602 */
HittableP generate_two_perlin_spheres(Ctx& c) {
  MaterialP noise = lambert(std::make_shared<NoiseTexture>(c.rand, 4.0f));
  std::vector<HittableP> o;
  o.push_back(mk<Sphere>(v3(0.0f, -1000.0f, 0.0f), 1000.0f, noise));
  o.push_back(mk<Sphere>(v3(0.0f, 2.0f, 0.0f), 2.0f, noise));
  return mk<BvhNode>(std::move(o), 0.0f, 1.0f);
}

/* :604-612 */
HittableP generate_earth(Ctx& c) {
  std::vector<HittableP> o;
  o.push_back(mk<Sphere>(v3(0.0f, 0.0f, 0.0f), 2.0f, lambert(image(c))));
  return mk<BvhNode>(std::move(o), 0.0f, 1.0f);
}

/* BASELINE config 3: the Earth sphere moved to (0,2,0) over the Perlin ground of :594-598 */
HittableP generate_earth_perlin(Ctx& c) {
  std::vector<HittableP> o;
  o.push_back(mk<Sphere>(v3(0.0f, -1000.0f, 0.0f), 1000.0f,
                         lambert(std::make_shared<NoiseTexture>(c.rand, 4.0f))));
  o.push_back(mk<Sphere>(v3(0.0f, 2.0f, 0.0f), 2.0f, lambert(image(c))));
  return mk<BvhNode>(std::move(o), 0.0f, 1.0f);
}

/* :614-637 */
HittableP generate_simple_light(Ctx& c) {
  MaterialP noise = lambert(std::make_shared<NoiseTexture>(c.rand, 4.0f));
  std::vector<HittableP> o;
  o.push_back(mk<Sphere>(v3(0.0f, -1000.0f, 0.0f), 1000.0f, noise));
  o.push_back(mk<Sphere>(v3(0.0f, 2.0f, 0.0f), 2.0f, noise));
  o.push_back(mk<Rect>(HRT_PLANE_XY, 3.0f, 5.0f, 1.0f, 3.0f, -2.0f,
                       std::make_shared<DiffuseLight>(solid(4.0f, 4.0f, 4.0f))));
  return mk<BvhNode>(std::move(o), 0.0f, 1.0f);
}

/* :639-815 (smoke = the CornellSmoke variant of :723-815) */
HittableP generate_cornell(bool smoke) {
  MaterialP red = lambert(solid(0.65f, 0.05f, 0.05f));
  MaterialP white = lambert(solid(0.73f, 0.73f, 0.73f));
  MaterialP green = lambert(solid(0.12f, 0.45f, 0.15f));
  MaterialP light = std::make_shared<DiffuseLight>(solid(15.0f, 15.0f, 15.0f));
  std::vector<HittableP> o;
  o.push_back(mk<Rect>(HRT_PLANE_YZ, 0.0f, 555.0f, 0.0f, 555.0f, 555.0f, green));
  o.push_back(mk<Rect>(HRT_PLANE_YZ, 0.0f, 555.0f, 0.0f, 555.0f, 0.0f, red));
  o.push_back(mk<Rect>(HRT_PLANE_ZX, 213.0f, 343.0f, 227.0f, 332.0f, 554.0f, light));
  o.push_back(mk<Rect>(HRT_PLANE_ZX, 0.0f, 555.0f, 0.0f, 555.0f, 0.0f, white));
  o.push_back(mk<Rect>(HRT_PLANE_ZX, 0.0f, 555.0f, 0.0f, 555.0f, 555.0f, white));
  o.push_back(mk<Rect>(HRT_PLANE_XY, 0.0f, 555.0f, 0.0f, 555.0f, 555.0f, white));
  HittableP c1 = mk<Cuboid>(v3(0.0f, 0.0f, 0.0f), v3(165.0f, 330.0f, 165.0f), white);
  c1 = mk<Rotation>(HRT_AXIS_Y, std::move(c1), 15.0f);
  c1 = mk<Translation>(std::move(c1), v3(265.0f, 0.0f, 295.0f));
  if (smoke) c1 = mk<ConstantMedium>(std::move(c1), 0.01f, solid(0.0f, 0.0f, 0.0f));
  o.push_back(std::move(c1));
  HittableP c2 = mk<Cuboid>(v3(0.0f, 0.0f, 0.0f), v3(165.0f, 165.0f, 165.0f), white);
  c2 = mk<Rotation>(HRT_AXIS_Y, std::move(c2), -18.0f);
  c2 = mk<Translation>(std::move(c2), v3(130.0f, 0.0f, 65.0f));
  if (smoke) c2 = mk<ConstantMedium>(std::move(c2), 0.01f, solid(1.0f, 1.0f, 1.0f));
  o.push_back(std::move(c2));
  return mk<BvhNode>(std::move(o), 0.0f, 1.0f);
}

/* :817-935 */
HittableP generate_final_scene(Ctx& c) {
  Rng& rand = c.rand;
  MaterialP ground_material = lambert(solid(0.48f, 0.83f, 0.53f));
  std::vector<HittableP> ground_boxes;
  for (int i = 0; i < 20; i++)
    for (int j = 0; j < 20; j++) {
      float w = 100.0f;
      float x0 = -1000.0f + (float)i * w;
      float z0 = -1000.0f + (float)j * w;
      float y0 = 0.0f;
      float x1 = x0 + w;
      float y1 = rand.gen_range_f32(1.0f, 101.0f);
      float z1 = z0 + w;
      ground_boxes.push_back(mk<Cuboid>(v3(x0, y0, z0), v3(x1, y1, z1), ground_material));
    }
  std::vector<HittableP> o;
  o.push_back(mk<BvhNode>(std::move(ground_boxes), 0.0f, 1.0f));
  o.push_back(mk<Rect>(HRT_PLANE_ZX, 123.0f, 423.0f, 147.0f, 412.0f, 554.0f,
                       std::make_shared<DiffuseLight>(solid(7.0f, 7.0f, 7.0f))));
  Vec3 center_1 = v3(400.0f, 400.0f, 200.0f);
  Vec3 center_2 = center_1 + v3(30.0f, 0.0f, 0.0f);
  o.push_back(mk<MovingSphere>(center_1, center_2, 0.0f, 1.0f, 50.0f, lambert(solid(0.7f, 0.3f, 0.1f))));
  o.push_back(mk<Sphere>(v3(260.0f, 150.0f, 45.0f), 50.0f, std::make_shared<Dielectric>(1.5f)));
  o.push_back(mk<Sphere>(v3(0.0f, 150.0f, 145.0f), 50.0f, std::make_shared<Metal>(v3(0.8f, 0.8f, 0.9f), 1.0f)));
  o.push_back(mk<Sphere>(v3(360.0f, 150.0f, 145.0f), 70.0f, std::make_shared<Dielectric>(1.5f)));
  o.push_back(mk<ConstantMedium>(mk<Sphere>(v3(360.0f, 150.0f, 145.0f), 70.0f, std::make_shared<Dielectric>(1.5f)),
                                 0.2f, solid(0.2f, 0.4f, 0.9f)));
  o.push_back(mk<ConstantMedium>(mk<Sphere>(v3(0.0f, 0.0f, 0.0f), 5000.0f, std::make_shared<Dielectric>(1.5f)),
                                 0.0001f, solid(1.0f, 1.0f, 1.0f)));
  o.push_back(mk<Sphere>(v3(400.0f, 200.0f, 400.0f), 100.0f, lambert(image(c))));
  o.push_back(mk<Sphere>(v3(220.0f, 280.0f, 300.0f), 80.0f, lambert(std::make_shared<NoiseTexture>(rand, 0.1f))));
  MaterialP white = lambert(solid(0.73f, 0.73f, 0.73f));
  std::vector<HittableP> sphere_box;
  for (int k = 0; k < 1000; k++) {
    float x = rand.gen_range_f32(0.0f, 165.0f);
    float y = rand.gen_range_f32(0.0f, 165.0f);
    float z = rand.gen_range_f32(0.0f, 165.0f);
    sphere_box.push_back(mk<Sphere>(v3(x, y, z), 10.0f, white));
  }
  o.push_back(mk<Translation>(
      mk<Rotation>(HRT_AXIS_Y, mk<BvhNode>(std::move(sphere_box), 0.0f, 1.0f), 15.0f),
      v3(-100.0f, 270.0f, 395.0f)));
  return mk<BvhNode>(std::move(o), 0.0f, 1.0f);
}

/* build-defined feature coverage scene: lists, X/Y/Z rotations, nested instances, a
 * medium inside an instance, rects of every plane with image/checker/emissive textures, a moving
 * sphere with a shutter other than [0, 1], a non-black background */
HittableP generate_features(Ctx& c) {
  Rng& rand = c.rand;
  TextureP img = image(c);
  std::vector<HittableP> o;
  o.push_back(mk<Sphere>(v3(0.0f, -1000.0f, 0.0f), 1000.0f,
                         lambert(std::make_shared<CheckerTexture>(std::make_shared<NoiseTexture>(rand, 2.0f),
                                                                  solid(0.8f, 0.8f, 0.8f)))));
  {
    std::vector<HittableP> l;
    l.push_back(mk<Sphere>(v3(-3.0f, 1.0f, 0.0f), 1.0f, std::make_shared<Dielectric>(1.5f)));
    l.push_back(mk<MovingSphere>(v3(-3.0f, 2.5f, 0.0f), v3(-2.5f, 2.5f, 0.0f), 0.25f, 0.75f, 0.4f,
                                 std::make_shared<Metal>(v3(0.8f, 0.6f, 0.2f), 0.3f)));
    o.push_back(mk<List>(std::move(l)));
  }
  o.push_back(mk<Translation>(
      mk<Rotation>(HRT_AXIS_Z, mk<Cuboid>(v3(0.0f, 0.0f, 0.0f), v3(1.0f, 2.0f, 1.0f), lambert(img)), 30.0f),
      v3(1.5f, 0.0f, -1.0f)));
  o.push_back(mk<Translation>(
      mk<Rotation>(HRT_AXIS_X,
                   mk<Cuboid>(v3(-0.5f, 0.0f, -0.5f), v3(0.5f, 1.0f, 0.5f),
                              std::make_shared<Metal>(v3(0.7f, 0.7f, 0.7f), 0.05f)),
                   -20.0f),
      v3(3.0f, 0.5f, 1.0f)));
  o.push_back(mk<ConstantMedium>(
      mk<Translation>(mk<Rotation>(HRT_AXIS_Y,
                                   mk<Cuboid>(v3(0.0f, 0.0f, 0.0f), v3(1.0f, 1.0f, 1.0f),
                                              lambert(solid(0.73f, 0.73f, 0.73f))),
                                   45.0f),
                      v3(-1.0f, 0.0f, 2.0f)),
      0.8f, solid(0.2f, 0.4f, 0.9f)));
  o.push_back(mk<Rect>(HRT_PLANE_XY, -1.0f, 1.0f, 3.0f, 4.0f, -3.0f,
                       std::make_shared<DiffuseLight>(solid(4.0f, 4.0f, 4.0f))));
  o.push_back(mk<Rect>(HRT_PLANE_YZ, 0.0f, 2.0f, -2.0f, 0.0f, -4.0f, lambert(img)));
  o.push_back(mk<Rect>(HRT_PLANE_ZX, -1.0f, 1.0f, -1.0f, 1.0f, 3.5f,
                       std::make_shared<DiffuseLight>(std::make_shared<CheckerTexture>(
                           solid(2.0f, 2.0f, 2.0f), solid(0.5f, 0.5f, 3.0f)))));
  {
    std::vector<HittableP> sb;
    for (int k = 0; k < 20; k++) {
      float x = rand.gen_range_f32(0.0f, 1.5f);
      float y = rand.gen_range_f32(0.0f, 1.5f);
      float z = rand.gen_range_f32(0.0f, 1.5f);
      float r = rand.gen_f32(), g = rand.gen_f32(), b = rand.gen_f32();
      sb.push_back(mk<Sphere>(v3(x, y, z), 0.15f, lambert(solid(r, g, b))));
    }
    o.push_back(mk<Translation>(mk<Rotation>(HRT_AXIS_Y, mk<BvhNode>(std::move(sb), 0.0f, 1.0f), 15.0f),
                                v3(-4.5f, 0.0f, -2.0f)));
  }
  o.push_back(mk<Sphere>(v3(1.0f, 0.7f, 2.0f), 0.7f, lambert(std::make_shared<NoiseTexture>(rand, 4.0f))));
  return mk<BvhNode>(std::move(o), 0.0f, 1.0f);
}

void set3(float* d, float a, float b, float c) { d[0] = a; d[1] = b; d[2] = c; }

}  // namespace

extern "C" hrt_status hrt_preset_build(hrt_scene* s, int32_t preset, uint64_t scene_seed,
                                       const uint8_t* img, uint32_t iw, uint32_t ih, uint32_t ic,
                                       hrt_preset_info* info) {
  try {
    if (!s || !info || preset < 0 || preset >= HRT_PRESET_COUNT) {
      hrt::set_error("hrt_preset_build: bad argument");
      return HRT_ERR_INVALID_ARG;
    }
    Ctx c{scene_rng(scene_seed), img, iw, ih, ic};
    /* application.rs:132-211 */
    set3(info->look_from, 13.0f, 2.0f, 3.0f);
    set3(info->look_at, 0.0f, 0.0f, 0.0f);
    set3(info->background, 0.7f, 0.8f, 1.0f);
    info->fov = 20.0f;
    info->aperture = 0.0f;
    info->focus_dist = 10.0f;
    info->time0 = 0.0f;
    info->time1 = 1.0f;
    HittableP world;
    switch (preset) {
      case HRT_PRESET_RANDOM: info->aperture = 0.1f; world = generate_random_scene(c, 11); break;
      case HRT_PRESET_RANDOM_10K: info->aperture = 0.1f; world = generate_random_scene(c, 50); break;
      case HRT_PRESET_RANDOM_40K: info->aperture = 0.1f; world = generate_random_scene(c, 100); break;
      case HRT_PRESET_MOTION: info->aperture = 0.05f; world = generate_motion(c); break;
      case HRT_PRESET_TWO_SPHERES: world = generate_two_spheres(); break;
      case HRT_PRESET_TWO_PERLIN_SPHERES: world = generate_two_perlin_spheres(c); break;
      case HRT_PRESET_EARTH: world = generate_earth(c); break;
      case HRT_PRESET_EARTH_PERLIN: world = generate_earth_perlin(c); break;
      case HRT_PRESET_SIMPLE_LIGHT:
        set3(info->look_from, 26.0f, 3.0f, 6.0f);
        set3(info->look_at, 0.0f, 2.0f, 0.0f);
        set3(info->background, 0.0f, 0.0f, 0.0f);
        world = generate_simple_light(c);
        break;
      case HRT_PRESET_CORNELL:
      case HRT_PRESET_CORNELL_SMOKE:
        set3(info->look_from, 278.0f, 278.0f, -800.0f);
        set3(info->look_at, 278.0f, 278.0f, 0.0f);
        set3(info->background, 0.0f, 0.0f, 0.0f);
        info->fov = 40.0f;
        world = generate_cornell(preset == HRT_PRESET_CORNELL_SMOKE);
        break;
      case HRT_PRESET_FINAL:
        set3(info->look_from, 478.0f, 278.0f, -600.0f);
        set3(info->look_at, 278.0f, 278.0f, 0.0f);
        set3(info->background, 0.0f, 0.0f, 0.0f);
        info->fov = 40.0f;
        world = generate_final_scene(c);
        break;
      case HRT_PRESET_FEATURES:
        set3(info->look_from, 0.0f, 3.0f, 12.0f);
        set3(info->look_at, 0.0f, 1.0f, 0.0f);
        set3(info->background, 0.15f, 0.18f, 0.25f);
        info->fov = 35.0f;
        info->aperture = 0.05f;
        world = generate_features(c);
        break;
    }
    SceneBuilder b{s, {}};
    uint32_t root = world->lower(b);
    hrt_status st = hrt_scene_set_root(s, root);
    if (st != HRT_OK) return st;
    info->root = root;
    return HRT_OK;
  } catch (const LowerError& e) {
    hrt::set_error(e.what());
    return e.code;
  } catch (const std::exception& e) {
    hrt::set_error(e.what());
    return HRT_ERR_INVALID_ARG;
  }
}
