/*
 * world.hpp — C++ host mirror of the reference's scene-builder surface.
 *
 * The reference builds scenes from concrete types behind three traits (src/hittable/mod.rs:19-25,
 * src/materials/mod.rs:15-19, src/textures/mod.rs:14-16).  Here every concrete type keeps its
 * reference name and constructor arguments and gains one additive method, lower(), which records the
 * object through the C ABI (hrt.h).  Scene builders written against these classes read like
 * application.rs:497-935 and drop in unchanged; the Rust binding of INTEGRATION.md adds the same
 * lower() to the Rust types.
 *
 * Textures and materials are shared (Rust clones them), so lowering caches their ids; hittables are
 * owned (Box<dyn Hittable>) and lowered exactly once.
 */
#pragma once
#include <hrt/hd_math.h>
#include <hrt/hrt.h>

#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace hrt {
void set_error(const std::string& msg); /* scene.cpp: thread-local hrt_last_error text */
namespace world {

struct LowerError : std::runtime_error {
  hrt_status code;
  LowerError(hrt_status c, const std::string& m) : std::runtime_error(m), code(c) {}
};
inline void check(hrt_status st) {
  if (st != HRT_OK) throw LowerError(st, hrt_last_error());
}

struct SceneBuilder {
  hrt_scene* scene;
  std::map<const void*, uint32_t> ids; /* shared textures / materials already lowered */
};

/* ------------------------------------------------------------------ textures */
struct Texture {
  virtual ~Texture() {}
  virtual uint32_t lower_new(SceneBuilder& b) const = 0;
  uint32_t lower(SceneBuilder& b) const {
    auto it = b.ids.find(this);
    if (it != b.ids.end()) return it->second;
    uint32_t id = lower_new(b);
    b.ids[this] = id;
    return id;
  }
};
using TextureP = std::shared_ptr<Texture>;

struct SolidColor : Texture { /* solid_color.rs:9-23 */
  Vec3 color;
  explicit SolidColor(Vec3 c) : color(c) {}
  uint32_t lower_new(SceneBuilder& b) const override {
    uint32_t id;
    check(hrt_tex_solid(b.scene, color.x, color.y, color.z, &id));
    return id;
  }
};

struct CheckerTexture : Texture { /* checker_texture.rs:9-30 */
  TextureP odd, even;
  CheckerTexture(TextureP o, TextureP e) : odd(std::move(o)), even(std::move(e)) {}
  uint32_t lower_new(SceneBuilder& b) const override {
    uint32_t o = odd->lower(b), e = even->lower(b), id;
    check(hrt_tex_checker(b.scene, o, e, &id));
    return id;
  }
};

struct PerlinNoise { /* perlin_noise.rs:12-64: tables drawn from the builder's stream */
  float random_vectors[256][3];
  uint32_t permutation[3][256];
  explicit PerlinNoise(Rng& rand) {
    for (int i = 0; i < 256; i++) {
      float x = rand.gen_range_f32(-1.0f, 1.0f);
      float y = rand.gen_range_f32(-1.0f, 1.0f);
      float z = rand.gen_range_f32(-1.0f, 1.0f);
      Vec3 v = normalize(v3(x, y, z));
      random_vectors[i][0] = v.x;
      random_vectors[i][1] = v.y;
      random_vectors[i][2] = v.z;
    }
    for (int c = 0; c < 3; c++) {
      for (int i = 0; i < 256; i++) permutation[c][i] = (uint32_t)i;
      for (int i = 255; i >= 1; i--) { /* Sattolo, :58-64 */
        uint64_t target = gen_range_u64(rand, 0, (uint64_t)i);
        uint32_t t = permutation[c][i];
        permutation[c][i] = permutation[c][target];
        permutation[c][target] = t;
      }
    }
  }
};

struct NoiseTexture : Texture { /* noise_texture.rs:9-31 */
  std::shared_ptr<PerlinNoise> noise;
  float scale;
  NoiseTexture(Rng& rand, float s) : noise(std::make_shared<PerlinNoise>(rand)), scale(s) {}
  uint32_t lower_new(SceneBuilder& b) const override {
    uint32_t id;
    check(hrt_tex_noise(b.scene, scale, &noise->random_vectors[0][0], &noise->permutation[0][0], &id));
    return id;
  }
};

struct ImageTexture : Texture { /* image_texture.rs:9-33: bytes decoded by the caller */
  const uint8_t* data;
  uint32_t width, height, components;
  ImageTexture(const uint8_t* d, uint32_t w, uint32_t h, uint32_t c)
      : data(d), width(w), height(h), components(c) {}
  uint32_t lower_new(SceneBuilder& b) const override {
    uint32_t id;
    check(hrt_tex_image(b.scene, data, width, height, components, &id));
    return id;
  }
};

/* ------------------------------------------------------------------ materials */
struct Material {
  virtual ~Material() {}
  virtual uint32_t lower_new(SceneBuilder& b) const = 0;
  uint32_t lower(SceneBuilder& b) const {
    auto it = b.ids.find(this);
    if (it != b.ids.end()) return it->second;
    uint32_t id = lower_new(b);
    b.ids[this] = id;
    return id;
  }
};
using MaterialP = std::shared_ptr<Material>;

struct Lambertian : Material { /* lambertian.rs */
  TextureP albedo;
  explicit Lambertian(TextureP a) : albedo(std::move(a)) {}
  uint32_t lower_new(SceneBuilder& b) const override {
    uint32_t t = albedo->lower(b), id;
    check(hrt_mat_lambertian(b.scene, t, &id));
    return id;
  }
};
struct Metal : Material { /* metal.rs */
  Vec3 albedo;
  float fuzz;
  Metal(Vec3 a, float f) : albedo(a), fuzz(f) {}
  uint32_t lower_new(SceneBuilder& b) const override {
    uint32_t id;
    check(hrt_mat_metal(b.scene, albedo.x, albedo.y, albedo.z, fuzz, &id));
    return id;
  }
};
struct Dielectric : Material { /* dielectric.rs */
  float index_of_refraction;
  explicit Dielectric(float ior) : index_of_refraction(ior) {}
  uint32_t lower_new(SceneBuilder& b) const override {
    uint32_t id;
    check(hrt_mat_dielectric(b.scene, index_of_refraction, &id));
    return id;
  }
};
struct DiffuseLight : Material { /* diffuse_light.rs */
  TextureP emit;
  explicit DiffuseLight(TextureP e) : emit(std::move(e)) {}
  uint32_t lower_new(SceneBuilder& b) const override {
    uint32_t t = emit->lower(b), id;
    check(hrt_mat_diffuse_light(b.scene, t, &id));
    return id;
  }
};

/* ------------------------------------------------------------------ hittables */
struct Hittable {
  virtual ~Hittable() {}
  virtual uint32_t lower(SceneBuilder& b) const = 0;
};
using HittableP = std::unique_ptr<Hittable>;

struct Sphere : Hittable { /* sphere.rs */
  Vec3 center;
  float radius;
  MaterialP material;
  Sphere(Vec3 c, float r, MaterialP m) : center(c), radius(r), material(std::move(m)) {}
  uint32_t lower(SceneBuilder& b) const override {
    uint32_t m = material->lower(b), id;
    float c[3] = {center.x, center.y, center.z};
    check(hrt_node_sphere(b.scene, c, radius, m, &id));
    return id;
  }
};
struct MovingSphere : Hittable { /* moving_sphere.rs */
  Vec3 center_start, center_end;
  float time_start, time_end, radius;
  MaterialP material;
  MovingSphere(Vec3 c0, Vec3 c1, float t0, float t1, float r, MaterialP m)
      : center_start(c0), center_end(c1), time_start(t0), time_end(t1), radius(r), material(std::move(m)) {}
  uint32_t lower(SceneBuilder& b) const override {
    uint32_t m = material->lower(b), id;
    float c0[3] = {center_start.x, center_start.y, center_start.z};
    float c1[3] = {center_end.x, center_end.y, center_end.z};
    check(hrt_node_moving_sphere(b.scene, c0, c1, time_start, time_end, radius, m, &id));
    return id;
  }
};
struct Rect : Hittable { /* rect.rs */
  int plane;
  float a0, a1, b0, b1, k;
  MaterialP material;
  Rect(int p, float a0_, float a1_, float b0_, float b1_, float k_, MaterialP m)
      : plane(p), a0(a0_), a1(a1_), b0(b0_), b1(b1_), k(k_), material(std::move(m)) {}
  uint32_t lower(SceneBuilder& b) const override {
    uint32_t m = material->lower(b), id;
    check(hrt_node_rect(b.scene, plane, a0, a1, b0, b1, k, m, &id));
    return id;
  }
};
struct Cuboid : Hittable { /* cuboid.rs */
  Vec3 box_min, box_max;
  MaterialP material;
  Cuboid(Vec3 p0, Vec3 p1, MaterialP m) : box_min(p0), box_max(p1), material(std::move(m)) {}
  uint32_t lower(SceneBuilder& b) const override {
    uint32_t m = material->lower(b), id;
    float p0[3] = {box_min.x, box_min.y, box_min.z}, p1[3] = {box_max.x, box_max.y, box_max.z};
    check(hrt_node_cuboid(b.scene, p0, p1, m, &id));
    return id;
  }
};
struct Translation : Hittable { /* translation.rs */
  HittableP hittable;
  Vec3 displacement;
  Translation(HittableP h, Vec3 d) : hittable(std::move(h)), displacement(d) {}
  uint32_t lower(SceneBuilder& b) const override {
    uint32_t c = hittable->lower(b), id;
    float d[3] = {displacement.x, displacement.y, displacement.z};
    check(hrt_node_translate(b.scene, c, d, &id));
    return id;
  }
};
struct Rotation : Hittable { /* rotation.rs */
  int axis;
  HittableP hittable;
  float angle;
  Rotation(int ax, HittableP h, float a) : axis(ax), hittable(std::move(h)), angle(a) {}
  uint32_t lower(SceneBuilder& b) const override {
    uint32_t c = hittable->lower(b), id;
    check(hrt_node_rotate(b.scene, axis, c, angle, &id));
    return id;
  }
};
struct ConstantMedium : Hittable { /* constant_medium.rs */
  HittableP boundary;
  float density;
  TextureP texture;
  ConstantMedium(HittableP bd, float d, TextureP t) : boundary(std::move(bd)), density(d), texture(std::move(t)) {}
  uint32_t lower(SceneBuilder& b) const override {
    uint32_t c = boundary->lower(b), t = texture->lower(b), id;
    check(hrt_node_constant_medium(b.scene, c, density, t, &id));
    return id;
  }
};
struct List : Hittable { /* list.rs */
  std::vector<HittableP> objects;
  explicit List(std::vector<HittableP> o) : objects(std::move(o)) {}
  uint32_t lower(SceneBuilder& b) const override {
    std::vector<uint32_t> ids;
    for (const auto& o : objects) ids.push_back(o->lower(b));
    uint32_t id;
    check(hrt_node_list(b.scene, ids.data(), (uint32_t)ids.size(), &id));
    return id;
  }
};
struct BvhNode : Hittable { /* bvh_node.rs: built by hrt_node_bvh at lowering time */
  std::vector<HittableP> objects;
  float time_start, time_end;
  BvhNode(std::vector<HittableP> o, float t0, float t1) : objects(std::move(o)), time_start(t0), time_end(t1) {}
  uint32_t lower(SceneBuilder& b) const override {
    std::vector<uint32_t> ids;
    for (const auto& o : objects) ids.push_back(o->lower(b));
    uint32_t id;
    check(hrt_node_bvh(b.scene, ids.data(), (uint32_t)ids.size(), time_start, time_end, &id));
    return id;
  }
};

}  // namespace world
}  // namespace hrt
