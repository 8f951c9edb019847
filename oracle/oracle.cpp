/*
 * oracle.cpp — TEST INFRASTRUCTURE ONLY (the parity checker and the CPU baseline).
 *
 * A C++ CPU restatement of the reference renderer (SkillerRaptor/hyper-ray-tracer, Rust), kept in the
 * reference's own shape: trait objects (virtual dispatch), a recursive BvhNode, a recursive
 * ray_color, 80x80 tiles on a thread pool.  Every function cites the reference file:line it follows.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library; the
 * product (hyper-ray-tracer_amd/) never links or calls it.
 *
 * Pinning: the reference is a Rust binary (no cargo/rustc in this image, needs a GLFW window, and is
 * unseeded: rand::thread_rng), it has no tests or fixtures, so no golden image of it can exist.
 * => parity UNPINNED against the reference binary.  What pins this restatement instead:
 *    - tests/golden/kat_*.json: an independent numpy-float32 restatement of each unit function
 *      (tests/golden/make_kats.py), compared bit-exactly;
 *    - the shared transcendentals against correctly rounded f64 values;
 *    - statistical checks (tests/test_oracle.py).
 * Substitutions (documented in DESIGN.md): thread_rng -> keyed xoshiro128** (hd_math.h); Rust
 * sort_unstable -> stable sort (identical for < 21 elements, where Rust uses insertion sort).
 */
#include <hrt/hd_math.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <thread>
#include <vector>

using namespace hrt;

namespace oracle {

/* ---- the platform-libm variant (tests/test_libm.py) --------------------------------------------
 * The reference's f32::{sin, cos, tan, acos, atan2, ln, powf} are calls into the platform libm: glibc's
 * sinf / cosf / tanf / acosf / atan2f / logf / powf on Linux (Rust std lowers them to the C symbols).
 * The restatement (and the kernel) use hd_math's deterministic f64 evaluations instead, which host and
 * gfx950 compute bit for bit alike.  oracle_set_libm(1) switches THIS oracle to glibc's f32 functions,
 * so the GPU frame can be compared with an oracle on the reference platform's arithmetic.  Optional
 * input recording (single-threaded renders) collects the arguments the scenes actually produce. */
static int g_libm = 0;
enum { OP_SIN, OP_COS, OP_ACOS, OP_ATAN2, OP_LN, OP_POW5, OP_TAN, OP_N };
static float* g_rec[OP_N] = {};
static uint32_t g_rec_cap = 0;
static std::atomic<uint32_t> g_rec_n[OP_N];
static inline void rec1(int op, float a, float b = 0.0f) {
  if (!g_rec[op]) return;
  const uint32_t i = g_rec_n[op].fetch_add(1);
  if (i < g_rec_cap) { g_rec[op][2 * i] = a; g_rec[op][2 * i + 1] = b; }
}
static inline float m_sin(float x) { rec1(OP_SIN, x); return g_libm ? sinf(x) : sin_f(x); }
static inline float m_cos(float x) { rec1(OP_COS, x); return g_libm ? cosf(x) : cos_f(x); }
static inline float m_tan(float x) { rec1(OP_TAN, x); return g_libm ? tanf(x) : tan_f(x); }
static inline float m_acos(float x) { rec1(OP_ACOS, x); return g_libm ? acosf(x) : acos_f(x); }
static inline float m_atan2(float y, float x) { rec1(OP_ATAN2, y, x); return g_libm ? atan2f(y, x) : atan2_f(y, x); }
static inline float m_ln(float x) { rec1(OP_LN, x); return g_libm ? logf(x) : ln_f(x); }
static inline float m_pow5(float x) { rec1(OP_POW5, x); return g_libm ? powf(x, 5.0f) : pow5_f(x); }
/* math.rs:58-62 with the switchable powf */
static inline float m_reflectance(float cosine, float refraction_index) {
  float r0 = (1.0f - refraction_index) / (1.0f + refraction_index);
  r0 = r0 * r0;
  return r0 + (1.0f - r0) * m_pow5(1.0f - cosine);
}


static const float INF_F = u2f(0x7f800000u);

/* ---------------------------------------------------------------- counters (instrumentation) */
enum {
  C_SEGMENTS = 0, C_AABB, C_SPHERE, C_MOVING, C_RECT, C_MEDIUM, C_TEX_SOLID, C_TEX_CHECKER,
  C_TEX_NOISE, C_TEX_IMAGE, C_SAMPLES, C_PIXELS, C_COUNT
};
struct Counters { uint64_t c[C_COUNT] = {}; };

/* per-path context: what the reference keeps in thread_rng + instrumentation */
struct Ctx {
  Rng rng;
  uint64_t pkey = 0;
  uint32_t segment = 0;
  Counters* cnt = nullptr;
};

/* ---------------------------------------------------------------- ray.rs:10-39 */
struct Ray {
  Vec3 origin, direction;
  float time;
  Vec3 at(float t) const { return origin + t * direction; }
};

struct Material;

/* ---------------------------------------------------------------- hit_record.rs:11-29 */
struct HitRecord {
  Vec3 point, normal;
  float t, u, v;
  bool front_face;
  const Material* material;
  void set_face_normal(const Ray& ray, Vec3 outward_normal) {
    front_face = dot(ray.direction, outward_normal) < 0.0f;
    normal = front_face ? outward_normal : -outward_normal;
  }
};

/* ---------------------------------------------------------------- aabb.rs:9-80 */
struct Aabb {
  Vec3 minimum, maximum;
  /* aabb.rs:20-47. time_min/time_max are NOT narrowed across axes (each axis is tested on its own
   * against the caller's interval); 1/d is recomputed per call. */
  bool hit(const Ray& ray, float time_min, float time_max, Ctx& ctx) const {
    ctx.cnt->c[C_AABB]++;
    for (int a = 0; a < 3; a++) {
      float inverse_direction = 1.0f / ray.direction[a];
      float time_start = (minimum[a] - ray.origin[a]) * inverse_direction;
      float time_end = (maximum[a] - ray.origin[a]) * inverse_direction;
      if (inverse_direction < 0.0f) std::swap(time_start, time_end);
      float t_min = time_start > time_min ? time_start : time_min;
      float t_max = time_end < time_max ? time_end : time_max;
      if (t_max <= t_min) return false;
    }
    return true;
  }
  /* aabb.rs:49-63 (f32::min / f32::max) */
  static Aabb surrounding_box(const Aabb& b0, const Aabb& b1) {
    Aabb r;
    r.minimum = v3(fminf(b0.minimum.x, b1.minimum.x), fminf(b0.minimum.y, b1.minimum.y),
                   fminf(b0.minimum.z, b1.minimum.z));
    r.maximum = v3(fmaxf(b0.maximum.x, b1.maximum.x), fmaxf(b0.maximum.y, b1.maximum.y),
                   fmaxf(b0.maximum.z, b1.maximum.z));
    return r;
  }
};

/* ---------------------------------------------------------------- textures/mod.rs:14-16 */
struct Texture {
  virtual ~Texture() {}
  virtual Vec3 value(float u, float v, Vec3 point, Ctx& ctx) const = 0;
};
using TexP = std::shared_ptr<Texture>;

/* solid_color.rs:20-23 */
struct SolidColor : Texture {
  Vec3 color;
  explicit SolidColor(Vec3 c) : color(c) {}
  Vec3 value(float, float, Vec3, Ctx& ctx) const override {
    ctx.cnt->c[C_TEX_SOLID]++;
    return color;
  }
};

/* checker_texture.rs:21-30 */
struct CheckerTexture : Texture {
  TexP odd, even;
  CheckerTexture(TexP o, TexP e) : odd(std::move(o)), even(std::move(e)) {}
  Vec3 value(float u, float v, Vec3 p, Ctx& ctx) const override {
    ctx.cnt->c[C_TEX_CHECKER]++;
    float sines = m_sin(10.0f * p.x) * m_sin(10.0f * p.y) * m_sin(10.0f * p.z);
    if (sines < 0.0f) return odd->value(u, v, p, ctx);
    return even->value(u, v, p, ctx);
  }
};

/* perlin_noise.rs:12-123 */
struct PerlinNoise {
  static const int POINT_COUNT = 256;
  Vec3 random_vectors[POINT_COUNT];
  uint32_t permutation_x[POINT_COUNT], permutation_y[POINT_COUNT], permutation_z[POINT_COUNT];

  /* :28-64, drawn from the scene stream in the reference's order */
  explicit PerlinNoise(Rng& rand) {
    for (int i = 0; i < POINT_COUNT; i++) {
      float x = rand.gen_range_f32(-1.0f, 1.0f);
      float y = rand.gen_range_f32(-1.0f, 1.0f);
      float z = rand.gen_range_f32(-1.0f, 1.0f);
      random_vectors[i] = normalize(v3(x, y, z));
    }
    generate_permutation(rand, permutation_x);
    generate_permutation(rand, permutation_y);
    generate_permutation(rand, permutation_z);
  }
  PerlinNoise(const float* ranvec, const uint32_t* perm) {
    for (int i = 0; i < POINT_COUNT; i++) {
      random_vectors[i] = v3(ranvec[3 * i], ranvec[3 * i + 1], ranvec[3 * i + 2]);
      permutation_x[i] = perm[i];
      permutation_y[i] = perm[256 + i];
      permutation_z[i] = perm[512 + i];
    }
  }
  static void generate_permutation(Rng& rand, uint32_t* p) {
    for (int i = 0; i < POINT_COUNT; i++) p[i] = (uint32_t)i;
    /* Sattolo: i from 255 down to 1, target = gen_range(0..i) (:58-64) */
    for (int i = POINT_COUNT - 1; i >= 1; i--) {
      uint64_t target = gen_range_u64(rand, 0, (uint64_t)i);
      std::swap(p[i], p[target]);
    }
  }
  /* :66-78 */
  float turbulence(Vec3 point, uint32_t depth) const {
    float accumulator = 0.0f;
    float weight = 1.0f;
    for (uint32_t k = 0; k < depth; k++) {
      accumulator += weight * noise(point);
      weight *= 0.5f;
      point = point * 2.0f;
    }
    return fabsf(accumulator);
  }
  /* :80-102 */
  float noise(Vec3 point) const {
    int32_t i = sat_f2i32(floorf(point.x));
    int32_t j = sat_f2i32(floorf(point.y));
    int32_t k = sat_f2i32(floorf(point.z));
    Vec3 c[2][2][2];
    for (int index = 0; index < 8; index++) {
      int i_x = index / 4, i_y = (index / 2) % 2, i_z = index % 2;
      /* i32 `i + i_x` wraps in a Rust release build (i = i32::MAX after the saturating cast of a huge
       * coordinate): the same bits in u32, without C++'s signed-overflow UB */
      uint32_t x = permutation_x[((uint32_t)i + (uint32_t)i_x) & (uint32_t)(POINT_COUNT - 1)];
      uint32_t y = permutation_y[((uint32_t)j + (uint32_t)i_y) & (uint32_t)(POINT_COUNT - 1)];
      uint32_t z = permutation_z[((uint32_t)k + (uint32_t)i_z) & (uint32_t)(POINT_COUNT - 1)];
      c[i_x][i_y][i_z] = random_vectors[x ^ y ^ z];
    }
    float u = point.x - floorf(point.x);
    float v = point.y - floorf(point.y);
    float w = point.z - floorf(point.z);
    return trilinear_interpolation(c, u, v, w);
  }
  /* :104-123 (smoothed u,v,w also used in the weight vector) */
  static float trilinear_interpolation(const Vec3 c[2][2][2], float u, float v, float w) {
    u = u * u * (3.0f - 2.0f * u);
    v = v * v * (3.0f - 2.0f * v);
    w = w * w * (3.0f - 2.0f * w);
    float accumulator = 0.0f;
    for (int i = 0; i < 8; i++) {
      int x = i / 4, y = (i / 2) % 2, z = i % 2;
      Vec3 weight = v3(u - (float)x, v - (float)y, w - (float)z);
      accumulator += ((float)x * u + (float)(1 - x) * (1.0f - u)) *
                     ((float)y * v + (float)(1 - y) * (1.0f - v)) *
                     ((float)z * w + (float)(1 - z) * (1.0f - w)) * dot(c[x][y][z], weight);
    }
    return accumulator;
  }
};

/* noise_texture.rs:24-31 */
struct NoiseTexture : Texture {
  std::shared_ptr<PerlinNoise> noise;
  float scale;
  NoiseTexture(std::shared_ptr<PerlinNoise> n, float s) : noise(std::move(n)), scale(s) {}
  Vec3 value(float, float, Vec3 p, Ctx& ctx) const override {
    ctx.cnt->c[C_TEX_NOISE]++;
    float s = 1.0f + m_sin((scale * p.z) + (10.0f * noise->turbulence(scale * p, 7)));
    return (v3(1.0f, 1.0f, 1.0f) * 0.5f) * s;
  }
};

/* image_texture.rs:19-63 */
struct ImageTexture : Texture {
  std::vector<uint8_t> data;
  uint32_t components = 0, width = 0, height = 0, bytes_per_scanline = 0;
  ImageTexture(const uint8_t* d, uint32_t w, uint32_t h, uint32_t c) {
    if (d && w && h && c) data.assign(d, d + (size_t)w * h * c);
    width = w; height = h; components = c; bytes_per_scanline = c * w;
  }
  Vec3 value(float u, float v, Vec3, Ctx& ctx) const override {
    ctx.cnt->c[C_TEX_IMAGE]++;
    if (data.empty()) return v3(1.0f, 0.0f, 1.0f);
    /* f32::clamp keeps NaN */
    u = u < 0.0f ? 0.0f : (u > 1.0f ? 1.0f : u);
    float vc = v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v);
    v = 1.0f - vc;
    uint32_t i = sat_f2u32(u * (float)width);
    uint32_t j = sat_f2u32(v * (float)height);
    if (i >= width) i = width - 1;
    if (j >= height) j = height - 1;
    const float color_scale = 1.0f / 255.0f;
    size_t offset = (size_t)j * bytes_per_scanline + (size_t)i * components;
    return v3(color_scale * (float)data[offset], color_scale * (float)data[offset + 1],
              color_scale * (float)data[offset + 2]);
  }
};

/* ---------------------------------------------------------------- materials/mod.rs:15-19 */
struct Material {
  virtual ~Material() {}
  virtual bool scatter(const Ray& ray, const HitRecord& rec, Vec3& attenuation, Ray& scattered,
                       Ctx& ctx) const = 0;
  virtual Vec3 emitted(float, float, Vec3, Ctx&) const { return v3(0.0f, 0.0f, 0.0f); }
};
using MatP = std::shared_ptr<Material>;

/* lambertian.rs:27-38 */
struct Lambertian : Material {
  TexP albedo;
  explicit Lambertian(TexP a) : albedo(std::move(a)) {}
  bool scatter(const Ray& ray, const HitRecord& rec, Vec3& att, Ray& sc, Ctx& ctx) const override {
    Vec3 scatter_direction = rec.normal + random_unit_vector(ctx.rng);
    if (near_zero(scatter_direction)) scatter_direction = rec.normal;
    att = albedo->value(rec.u, rec.v, rec.point, ctx);
    sc = Ray{rec.point, scatter_direction, ray.time};
    return true;
  }
};

/* metal.rs:29-42 */
struct Metal : Material {
  Vec3 albedo;
  float fuzz;
  Metal(Vec3 a, float f) : albedo(a), fuzz(f) {}
  bool scatter(const Ray& ray, const HitRecord& rec, Vec3& att, Ray& sc, Ctx& ctx) const override {
    Vec3 reflected = reflect(normalize(ray.direction), rec.normal);
    sc = Ray{rec.point, reflected + fuzz * random_in_unit_sphere(ctx.rng), ray.time};
    if (dot(sc.direction, rec.normal) > 0.0f) {
      att = albedo;
      return true;
    }
    return false;
  }
};

/* dielectric.rs:31-55 */
struct Dielectric : Material {
  float index_of_refraction;
  explicit Dielectric(float ior) : index_of_refraction(ior) {}
  bool scatter(const Ray& ray, const HitRecord& rec, Vec3& att, Ray& sc, Ctx& ctx) const override {
    float refraction_ratio = rec.front_face ? (1.0f / index_of_refraction) : index_of_refraction;
    Vec3 unit_direction = normalize(ray.direction);
    float cos_theta = min_rs(dot(-unit_direction, rec.normal), 1.0f);
    float sin_theta = sqrtf(1.0f - cos_theta * cos_theta);
    bool cannot_refract = (refraction_ratio * sin_theta) > 1.0f;
    Vec3 direction;
    /* the xi draw happens only when refraction is possible (|| short-circuits) */
    if (cannot_refract || m_reflectance(cos_theta, refraction_ratio) > ctx.rng.gen_f32())
      direction = reflect(unit_direction, rec.normal);
    else
      direction = refract(unit_direction, rec.normal, refraction_ratio);
    att = v3(1.0f, 1.0f, 1.0f);
    sc = Ray{rec.point, direction, ray.time};
    return true;
  }
};

/* diffuse_light.rs:20-28 */
struct DiffuseLight : Material {
  TexP emit;
  explicit DiffuseLight(TexP e) : emit(std::move(e)) {}
  bool scatter(const Ray&, const HitRecord&, Vec3&, Ray&, Ctx&) const override { return false; }
  Vec3 emitted(float u, float v, Vec3 p, Ctx& ctx) const override { return emit->value(u, v, p, ctx); }
};

/* isotropic.rs:26-33 */
struct Isotropic : Material {
  TexP albedo;
  explicit Isotropic(TexP a) : albedo(std::move(a)) {}
  bool scatter(const Ray& ray, const HitRecord& rec, Vec3& att, Ray& sc, Ctx& ctx) const override {
    att = albedo->value(rec.u, rec.v, rec.point, ctx);
    sc = Ray{rec.point, random_in_unit_sphere(ctx.rng), ray.time};
    return true;
  }
};

/* ---------------------------------------------------------------- hittable/mod.rs:19-25 */
struct Hittable {
  virtual ~Hittable() {}
  virtual bool hit(const Ray& ray, float tmin, float tmax, HitRecord& rec, Ctx& ctx) const = 0;
  virtual bool bounding_box(float t0, float t1, Aabb& out) const = 0;
  virtual uint32_t count() const = 0;
};
using HitP = std::unique_ptr<Hittable>;

/* sphere.rs:31-35 */
static void sphere_uv(Vec3 p, float& u, float& v) {
  float theta = m_acos(-p.y);
  float phi = m_atan2(-p.z, p.x) + PI_F;
  u = phi / (2.0f * PI_F);
  v = theta / PI_F;
}

/* sphere.rs:38-87 */
struct Sphere : Hittable {
  Vec3 center;
  float radius;
  MatP material;
  Sphere(Vec3 c, float r, MatP m) : center(c), radius(r), material(std::move(m)) {}
  bool hit(const Ray& ray, float tmin, float tmax, HitRecord& rec, Ctx& ctx) const override {
    ctx.cnt->c[C_SPHERE]++;
    Vec3 oc = ray.origin - center;
    float a = dot(ray.direction, ray.direction);
    float half_b = dot(oc, ray.direction);
    float c = dot(oc, oc) - radius * radius;
    float discriminant = half_b * half_b - a * c;
    if (discriminant < 0.0f) return false;
    float sqrtd = sqrtf(discriminant);
    float root = (-half_b - sqrtd) / a;
    if (root < tmin || tmax < root) {
      root = (-half_b + sqrtd) / a;
      if (root < tmin || tmax < root) return false;
    }
    Vec3 outward_normal = (ray.at(root) - center) / radius;
    sphere_uv(outward_normal, rec.u, rec.v);
    rec.point = ray.at(root);
    rec.t = root;
    rec.material = material.get();
    rec.set_face_normal(ray, outward_normal);
    return true;
  }
  bool bounding_box(float, float, Aabb& out) const override {
    Vec3 rv = v3(radius, radius, radius);
    out.minimum = center - rv;
    out.maximum = center + rv;
    return true;
  }
  uint32_t count() const override { return 1; }
};

/* moving_sphere.rs:50-114 */
struct MovingSphere : Hittable {
  Vec3 center_start, center_end;
  float time_start, time_end, radius;
  MatP material;
  MovingSphere(Vec3 c0, Vec3 c1, float t0, float t1, float r, MatP m)
      : center_start(c0), center_end(c1), time_start(t0), time_end(t1), radius(r),
        material(std::move(m)) {}
  Vec3 center(float time) const {
    return center_start +
           ((time - time_start) / (time_end - time_start)) * (center_end - center_start);
  }
  bool hit(const Ray& ray, float tmin, float tmax, HitRecord& rec, Ctx& ctx) const override {
    ctx.cnt->c[C_MOVING]++;
    Vec3 oc = ray.origin - center(ray.time);
    float a = dot(ray.direction, ray.direction);
    float half_b = dot(oc, ray.direction);
    float c = dot(oc, oc) - radius * radius;
    float discriminant = half_b * half_b - a * c;
    if (discriminant < 0.0f) return false;
    float sqrtd = sqrtf(discriminant);
    float root = (-half_b - sqrtd) / a;
    if (root < tmin || tmax < root) {
      root = (-half_b + sqrtd) / a;
      if (root < tmin || tmax < root) return false;
    }
    Vec3 outward_normal = (ray.at(root) - center(ray.time)) / radius;
    sphere_uv(outward_normal, rec.u, rec.v);
    rec.point = ray.at(root);
    rec.t = root;
    rec.material = material.get();
    rec.set_face_normal(ray, outward_normal);
    return true;
  }
  bool bounding_box(float t0, float t1, Aabb& out) const override {
    Vec3 rv = v3(radius, radius, radius);
    Aabb b0{center(t0) - rv, center(t0) + rv};
    Aabb b1{center(t1) - rv, center(t1) + rv};
    out = Aabb::surrounding_box(b0, b1);
    return true;
  }
  uint32_t count() const override { return 1; }
};

/* rect.rs:19-108 */
struct Rect : Hittable {
  int plane; /* 0 XY, 1 YZ, 2 ZX */
  float a0, a1, b0, b1, k;
  MatP material;
  Rect(int p, float a0_, float a1_, float b0_, float b1_, float k_, MatP m)
      : plane(p), a0(a0_), a1(a1_), b0(b0_), b1(b1_), k(k_), material(std::move(m)) {}
  bool hit(const Ray& ray, float tmin, float tmax, HitRecord& rec, Ctx& ctx) const override {
    ctx.cnt->c[C_RECT]++;
    int k_axis, a_axis, b_axis;
    if (plane == 0) { k_axis = 2; a_axis = 0; b_axis = 1; }
    else if (plane == 1) { k_axis = 0; a_axis = 1; b_axis = 2; }
    else { k_axis = 1; a_axis = 2; b_axis = 0; }
    float t = (k - ray.origin[k_axis]) / ray.direction[k_axis];
    if (t < tmin || t > tmax) return false;
    float a = ray.origin[a_axis] + t * ray.direction[a_axis];
    float b = ray.origin[b_axis] + t * ray.direction[b_axis];
    if (a < a0 || a > a1 || b < b0 || b > b1) return false;
    rec.point = ray.at(t);
    rec.t = t;
    rec.u = (a - a0) / (a1 - a0);
    rec.v = (b - b0) / (b1 - b0);
    rec.material = material.get();
    Vec3 outward = v3(0.0f, 0.0f, 0.0f);
    outward[k_axis] = 1.0f;
    rec.set_face_normal(ray, outward);
    return true;
  }
  bool bounding_box(float, float, Aabb& out) const override {
    if (plane == 0) out = Aabb{v3(a0, b0, k - 0.0001f), v3(a1, b1, k + 0.0001f)};
    else if (plane == 1) out = Aabb{v3(k - 0.0001f, a0, b0), v3(k + 0.0001f, a1, b1)};
    else out = Aabb{v3(a0, k - 0.0001f, b0), v3(a1, k + 0.0001f, b1)};
    return true;
  }
  uint32_t count() const override { return 1; }
};

/* list.rs:9-49 */
struct List : Hittable {
  std::vector<HitP> objects;
  explicit List(std::vector<HitP> o) : objects(std::move(o)) {}
  bool hit(const Ray& ray, float tmin, float tmax, HitRecord& rec, Ctx& ctx) const override {
    float closest = tmax;
    bool hit_anything = false;
    HitRecord tmp;
    for (const auto& o : objects) {
      if (o->hit(ray, tmin, closest, tmp, ctx)) {
        closest = tmp.t;
        rec = tmp;
        hit_anything = true;
      }
    }
    return hit_anything;
  }
  bool bounding_box(float t0, float t1, Aabb& out) const override {
    if (objects.empty()) return false;
    Aabb acc;
    if (!objects[0]->bounding_box(t0, t1, acc)) return false;
    for (size_t i = 1; i < objects.size(); i++) {
      Aabb b;
      if (!objects[i]->bounding_box(t0, t1, b)) return false;
      acc = Aabb::surrounding_box(acc, b);
    }
    out = acc;
    return true;
  }
  uint32_t count() const override {
    uint32_t n = 0;
    for (const auto& o : objects) n += o->count();
    return n;
  }
};

/* cuboid.rs:22-110: a List of 6 rects in this order */
struct Cuboid : Hittable {
  Vec3 box_min, box_max;
  std::unique_ptr<List> sides;
  Cuboid(Vec3 p0, Vec3 p1, MatP m) : box_min(p0), box_max(p1) {
    std::vector<HitP> s;
    s.emplace_back(new Rect(0, p0.x, p1.x, p0.y, p1.y, p1.z, m));
    s.emplace_back(new Rect(0, p0.x, p1.x, p0.y, p1.y, p0.z, m));
    s.emplace_back(new Rect(2, p0.z, p1.z, p0.x, p1.x, p1.y, m));
    s.emplace_back(new Rect(2, p0.z, p1.z, p0.x, p1.x, p0.y, m));
    s.emplace_back(new Rect(1, p0.y, p1.y, p0.z, p1.z, p1.x, m));
    s.emplace_back(new Rect(1, p0.y, p1.y, p0.z, p1.z, p0.x, m));
    sides.reset(new List(std::move(s)));
  }
  bool hit(const Ray& ray, float tmin, float tmax, HitRecord& rec, Ctx& ctx) const override {
    return sides->hit(ray, tmin, tmax, rec, ctx);
  }
  bool bounding_box(float, float, Aabb& out) const override {
    out = Aabb{box_min, box_max};
    return true;
  }
  uint32_t count() const override { return sides->count(); }
};

/* translation.rs:9-53 */
struct Translation : Hittable {
  HitP hittable;
  Vec3 displacement;
  Translation(HitP h, Vec3 d) : hittable(std::move(h)), displacement(d) {}
  bool hit(const Ray& ray, float tmin, float tmax, HitRecord& rec, Ctx& ctx) const override {
    Ray moved{ray.origin - displacement, ray.direction, ray.time};
    if (!hittable->hit(moved, tmin, tmax, rec, ctx)) return false;
    rec.point = rec.point + displacement;
    rec.set_face_normal(moved, rec.normal);
    return true;
  }
  bool bounding_box(float t0, float t1, Aabb& out) const override {
    Aabb b;
    if (!hittable->bounding_box(t0, t1, b)) return false;
    out = Aabb{b.minimum + displacement, b.maximum + displacement};
    return true;
  }
  uint32_t count() const override { return hittable->count(); }
};

/* rotation.rs:10-143 */
struct Rotation : Hittable {
  HitP hittable;
  float sin_theta, cos_theta;
  bool has_box;
  Aabb bbox;
  int axis;
  static void axes(int axis, int& r, int& a, int& b) {
    if (axis == 0) { r = 0; a = 1; b = 2; }
    else if (axis == 1) { r = 1; a = 2; b = 0; }
    else { r = 2; a = 0; b = 1; }
  }
  Rotation(int ax, HitP h, float angle) : hittable(std::move(h)), axis(ax) {
    int r_axis, a_axis, b_axis;
    axes(axis, r_axis, a_axis, b_axis);
    float radians = (PI_F / 180.0f) * angle;
    sin_theta = m_sin(radians);
    cos_theta = m_cos(radians);
    Aabb b;
    has_box = hittable->bounding_box(0.0f, 1.0f, b);
    if (has_box) {
      const float FMAX = 3.40282347e+38f;
      Vec3 mn = v3(FMAX, FMAX, FMAX), mx = v3(-FMAX, -FMAX, -FMAX);
      for (int i = 0; i < 2; i++)
        for (int j = 0; j < 2; j++)
          for (int k = 0; k < 2; k++) {
            float r = (float)k * b.maximum[r_axis] + (float)(1 - k) * b.minimum[r_axis];
            float a = (float)i * b.maximum[a_axis] + (float)(1 - i) * b.minimum[a_axis];
            float bb = (float)j * b.maximum[b_axis] + (float)(1 - j) * b.minimum[b_axis];
            float new_a = cos_theta * a - sin_theta * bb;
            float new_b = sin_theta * a + cos_theta * bb;
            if (new_a < mn[a_axis]) mn[a_axis] = new_a;
            if (new_b < mn[b_axis]) mn[b_axis] = new_b;
            if (r < mn[r_axis]) mn[r_axis] = r;
            if (new_a > mx[a_axis]) mx[a_axis] = new_a;
            if (new_b > mx[b_axis]) mx[b_axis] = new_b;
            if (r > mx[r_axis]) mx[r_axis] = r;
          }
      bbox = Aabb{mn, mx};
    }
  }
  bool hit(const Ray& ray, float tmin, float tmax, HitRecord& rec, Ctx& ctx) const override {
    int r_axis, a_axis, b_axis;
    axes(axis, r_axis, a_axis, b_axis);
    Vec3 origin = ray.origin, direction = ray.direction;
    origin[a_axis] = cos_theta * ray.origin[a_axis] + sin_theta * ray.origin[b_axis];
    origin[b_axis] = -sin_theta * ray.origin[a_axis] + cos_theta * ray.origin[b_axis];
    direction[a_axis] = cos_theta * ray.direction[a_axis] + sin_theta * ray.direction[b_axis];
    direction[b_axis] = -sin_theta * ray.direction[a_axis] + cos_theta * ray.direction[b_axis];
    Ray rotated{origin, direction, ray.time};
    if (!hittable->hit(rotated, tmin, tmax, rec, ctx)) return false;
    Vec3 point = rec.point, normal = rec.normal;
    point[a_axis] = cos_theta * rec.point[a_axis] - sin_theta * rec.point[b_axis];
    point[b_axis] = sin_theta * rec.point[a_axis] + cos_theta * rec.point[b_axis];
    normal[a_axis] = cos_theta * rec.normal[a_axis] - sin_theta * rec.normal[b_axis];
    normal[b_axis] = sin_theta * rec.normal[a_axis] + cos_theta * rec.normal[b_axis];
    rec.point = point;
    rec.normal = normal;
    return true;
  }
  bool bounding_box(float, float, Aabb& out) const override {
    if (!has_box) return false;
    out = bbox;
    return true;
  }
  uint32_t count() const override { return 1; }
};

/* constant_medium.rs:17-85 */
struct ConstantMedium : Hittable {
  HitP boundary;
  float negative_inverse_density;
  std::unique_ptr<Isotropic> phase_function;
  uint32_t medium_id; /* creation order; keys the medium's RNG sub-stream */
  ConstantMedium(HitP b, float density, TexP tex, uint32_t id)
      : boundary(std::move(b)), negative_inverse_density(-1.0f / density),
        phase_function(new Isotropic(std::move(tex))), medium_id(id) {}
  bool hit(const Ray& ray, float tmin, float tmax, HitRecord& rec, Ctx& ctx) const override {
    ctx.cnt->c[C_MEDIUM]++;
    HitRecord r1, r2;
    if (!boundary->hit(ray, -INF_F, INF_F, r1, ctx)) return false;
    if (!boundary->hit(ray, r1.t + 0.0001f, INF_F, r2, ctx)) return false;
    if (r1.t < tmin) r1.t = tmin;
    if (r2.t > tmax) r2.t = tmax;
    if (r1.t >= r2.t) return false;
    if (r1.t < 0.0f) r1.t = 0.0f;
    float ray_length = magnitude(ray.direction);
    float distance_inside_boundary = (r2.t - r1.t) * ray_length;
    /* rand.gen::<f32>().log(E) == ln(xi) / ln(E) (Rust f32::log) */
    float xi = medium_xi(ctx.pkey, ctx.segment, medium_id);
    float hit_distance = negative_inverse_density * (m_ln(xi) / (g_libm ? logf(E_F) : ln_f(E_F)));
    if (hit_distance > distance_inside_boundary) return false;
    float t = r1.t + hit_distance / ray_length;
    rec.point = ray.at(t);
    rec.normal = v3(0.0f, 0.0f, 0.0f);
    rec.t = t;
    rec.u = 0.0f;
    rec.v = 0.0f;
    rec.front_face = false;
    rec.material = phase_function.get();
    return true;
  }
  bool bounding_box(float t0, float t1, Aabb& out) const override {
    return boundary->bounding_box(t0, t1, out);
  }
  uint32_t count() const override { return boundary->count(); }
};

/* bvh_node.rs:10-139 */
struct BvhNode : Hittable {
  HitP left, right; /* branch */
  HitP leaf;        /* leaf */
  Aabb box;
  static float axis_range(const std::vector<HitP>& objects, float t0, float t1, int axis) {
    float mn = 3.40282347e+38f, mx = -3.40282347e+38f; /* f32::MAX, f32::MIN */
    for (const auto& o : objects) {
      Aabb b;
      if (!o->bounding_box(t0, t1, b)) continue;
      mn = fminf(mn, b.minimum[axis]);
      mx = fmaxf(mx, b.maximum[axis]);
    }
    return mx - mn;
  }
  BvhNode(std::vector<HitP> objects, float t0, float t1) {
    int order[3] = {0, 1, 2};
    float ranges[3];
    for (int a = 0; a < 3; a++) {
      ranges[a] = axis_range(objects, t0, t1, a);
      if (ranges[a] != ranges[a]) throw std::runtime_error("NaN axis range");
    }
    /* sort_unstable_by descending on 3 elements == stable insertion sort */
    std::stable_sort(order, order + 3, [&](int a, int b) { return ranges[a] > ranges[b]; });
    int axis = order[0];
    std::vector<std::pair<float, size_t>> keys(objects.size());
    for (size_t i = 0; i < objects.size(); i++) {
      Aabb b;
      if (!objects[i]->bounding_box(t0, t1, b)) throw std::runtime_error("no bounding box");
      float key = b.minimum[axis] + b.maximum[axis];
      if (key != key) throw std::runtime_error("NaN bounding box");
      keys[i] = {key, i};
    }
    std::stable_sort(keys.begin(), keys.end(),
                     [](const std::pair<float, size_t>& a, const std::pair<float, size_t>& b) {
                       return a.first < b.first;
                     });
    std::vector<HitP> sorted;
    sorted.reserve(objects.size());
    for (auto& k : keys) sorted.push_back(std::move(objects[k.second]));
    size_t len = sorted.size();
    if (len == 0) throw std::runtime_error("no elements in scene");
    if (len == 1) {
      leaf = std::move(sorted[0]);
      if (!leaf->bounding_box(t0, t1, box)) throw std::runtime_error("no bounding box");
      return;
    }
    std::vector<HitP> upper;
    for (size_t i = len / 2; i < len; i++) upper.push_back(std::move(sorted[i]));
    sorted.resize(len / 2);
    right.reset(new BvhNode(std::move(upper), t0, t1));
    left.reset(new BvhNode(std::move(sorted), t0, t1));
    box = Aabb::surrounding_box(static_cast<BvhNode*>(left.get())->box,
                                static_cast<BvhNode*>(right.get())->box);
  }
  bool hit(const Ray& ray, float tmin, float tmax, HitRecord& rec, Ctx& ctx) const override {
    if (!box.hit(ray, tmin, tmax, ctx)) return false;
    if (leaf) return leaf->hit(ray, tmin, tmax, rec, ctx);
    HitRecord lrec;
    bool lhit = left->hit(ray, tmin, tmax, lrec, ctx);
    float t_max = lhit ? lrec.t : tmax;
    HitRecord rrec;
    if (right->hit(ray, tmin, t_max, rrec, ctx)) { rec = rrec; return true; }
    if (lhit) { rec = lrec; return true; }
    return false;
  }
  bool bounding_box(float, float, Aabb& out) const override { out = box; return true; }
  uint32_t count() const override { return leaf ? leaf->count() : left->count() + right->count(); }
};

/* ---------------------------------------------------------------- camera.rs:16-96 */
struct Camera {
  Vec3 origin, lower_left_corner, horizontal, vertical, look_from, look_at;
  float fov, focus_dist;
  Vec3 w, u, v;
  float lens_radius, time_0, time_1;
  Camera(Vec3 from, Vec3 at, float fov_, float aperture, float focus, float t0, float t1, int width,
         int height)
      : look_from(from), look_at(at), fov(fov_), focus_dist(focus), lens_radius(aperture / 2.0f),
        time_0(t0), time_1(t1) {
    resize(width, height);
  }
  /* camera.rs:67-83; f32::to_radians == x * (PI / 180) */
  void resize(int width, int height) {
    float aspect_ratio = (float)width / (float)height;
    float theta = fov * (PI_F / 180.0f);
    float h = m_tan(theta / 2.0f);
    float viewport_height = 2.0f * h;
    float viewport_width = aspect_ratio * viewport_height;
    w = normalize(look_from - look_at);
    u = normalize(cross(v3(0.0f, 1.0f, 0.0f), w));
    v = cross(w, u);
    origin = look_from;
    horizontal = (focus_dist * viewport_width) * u;
    vertical = (focus_dist * viewport_height) * v;
    lower_left_corner = ((origin - horizontal / 2.0f) - vertical / 2.0f) - focus_dist * w;
  }
  /* camera.rs:85-95, with the two random quantities passed in */
  Ray ray_from(float s, float t, Vec3 disk, float time) const {
    Vec3 rd = lens_radius * disk;
    Vec3 offset = u * rd.x + v * rd.y;
    return Ray{origin + offset,
               (((lower_left_corner + s * horizontal) + t * vertical) - origin) - offset, time};
  }
  Ray get_ray(float s, float t, Rng& rng) const {
    Vec3 disk = random_in_unit_disk(rng);
    float time = rng.gen_range_f32(time_0, time_1);
    return ray_from(s, t, disk, time);
  }
};

/* ---------------------------------------------------------------- scene + builders */
struct PresetInfo {
  Vec3 look_from, look_at;
  float fov, aperture, focus_dist, time0, time1;
  Vec3 background;
};

struct Scene {
  HitP world;
  PresetInfo info;
  uint32_t n_media = 0;
};

static TexP solid(float r, float g, float b) { return std::make_shared<SolidColor>(v3(r, g, b)); }
static MatP lambert(TexP t) { return std::make_shared<Lambertian>(std::move(t)); }

struct Builder {
  Rng rand;
  uint32_t n_media = 0;
  const uint8_t* img;
  uint32_t iw, ih, ic;
  HitP medium(HitP boundary, float density, TexP tex) {
    return HitP(new ConstantMedium(std::move(boundary), density, std::move(tex), n_media++));
  }
  TexP noise(float scale) {
    return std::make_shared<NoiseTexture>(std::make_shared<PerlinNoise>(rand), scale);
  }
  TexP image() { return std::make_shared<ImageTexture>(img, iw, ih, ic); }
};

/* application.rs:497-565 (grid half-extent n = 11; the 10k variant uses n = 50) */
static HitP random_scene(Builder& B, int n) {
  std::vector<HitP> objects;
  objects.emplace_back(new Sphere(v3(0.0f, -1000.0f, 0.0f), 1000.0f,
                                  lambert(std::make_shared<CheckerTexture>(solid(0.2f, 0.3f, 0.1f),
                                                                           solid(0.9f, 0.9f, 0.9f)))));
  Rng& rand = B.rand;
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
          objects.emplace_back(
              new MovingSphere(center, center_2, 0.0f, 1.0f, 0.2f, lambert(solid(r, g, bl))));
        } else if (choose_material < 0.95f) {
          float r = rand.gen_range_f32(0.5f, 1.0f), g = rand.gen_range_f32(0.5f, 1.0f),
                bl = rand.gen_range_f32(0.5f, 1.0f);
          float fuzz = rand.gen_range_f32(0.0f, 0.5f);
          objects.emplace_back(new Sphere(center, 0.2f, std::make_shared<Metal>(v3(r, g, bl), fuzz)));
        } else {
          objects.emplace_back(new Sphere(center, 0.2f, std::make_shared<Dielectric>(1.5f)));
        }
      }
    }
  }
  objects.emplace_back(new Sphere(v3(0.0f, 1.0f, 0.0f), 1.0f, std::make_shared<Dielectric>(1.5f)));
  objects.emplace_back(new Sphere(v3(-4.0f, 1.0f, 0.0f), 1.0f, lambert(solid(0.4f, 0.2f, 0.1f))));
  objects.emplace_back(
      new Sphere(v3(4.0f, 1.0f, 0.0f), 1.0f, std::make_shared<Metal>(v3(0.7f, 0.6f, 0.5f), 0.0f)));
  return HitP(new BvhNode(std::move(objects), 0.0f, 1.0f));
}

/* build-defined (library presets.cpp generate_motion): moving spheres with their own shutter intervals,
 * drawn in the library's order; moving_sphere.rs:53-58 per sphere */
static HitP motion_scene(Builder& B) {
  std::vector<HitP> objects;
  objects.emplace_back(new Sphere(v3(0.0f, -1000.0f, 0.0f), 1000.0f,
                                  lambert(std::make_shared<CheckerTexture>(solid(0.2f, 0.3f, 0.1f),
                                                                           solid(0.9f, 0.9f, 0.9f)))));
  Rng& rand = B.rand;
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
      MatP m;
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
      objects.emplace_back(new MovingSphere(center, center_2, t0, t1, 0.2f, m));
    }
  }
  objects.emplace_back(new Sphere(v3(0.0f, 1.0f, 0.0f), 1.0f, std::make_shared<Dielectric>(1.5f)));
  objects.emplace_back(new MovingSphere(v3(-4.0f, 1.0f, 0.0f), v3(-4.0f, 1.5f, 0.0f), 0.0f, 2.0f, 1.0f,
                                        lambert(solid(0.4f, 0.2f, 0.1f))));
  return HitP(new BvhNode(std::move(objects), 0.0f, 1.0f));
}

static void cornell_walls(std::vector<HitP>& objects, MatP& white) {
  MatP red = lambert(solid(0.65f, 0.05f, 0.05f));
  white = lambert(solid(0.73f, 0.73f, 0.73f));
  MatP green = lambert(solid(0.12f, 0.45f, 0.15f));
  MatP light = std::make_shared<DiffuseLight>(solid(15.0f, 15.0f, 15.0f));
  objects.emplace_back(new Rect(1, 0.0f, 555.0f, 0.0f, 555.0f, 555.0f, green));
  objects.emplace_back(new Rect(1, 0.0f, 555.0f, 0.0f, 555.0f, 0.0f, red));
  objects.emplace_back(new Rect(2, 213.0f, 343.0f, 227.0f, 332.0f, 554.0f, light));
  objects.emplace_back(new Rect(2, 0.0f, 555.0f, 0.0f, 555.0f, 0.0f, white));
  objects.emplace_back(new Rect(2, 0.0f, 555.0f, 0.0f, 555.0f, 555.0f, white));
  objects.emplace_back(new Rect(0, 0.0f, 555.0f, 0.0f, 555.0f, 555.0f, white));
}

static Scene* build_preset(int preset, uint64_t seed, const uint8_t* img, uint32_t iw, uint32_t ih,
                           uint32_t ic) {
  std::unique_ptr<Scene> sc(new Scene());
  Builder B{scene_rng(seed), 0, img, iw, ih, ic};
  PresetInfo& I = sc->info;
  I.focus_dist = 10.0f; /* application.rs:201-211 */
  I.time0 = 0.0f;
  I.time1 = 1.0f;
  I.aperture = 0.0f;
  I.fov = 20.0f;
  I.look_from = v3(13.0f, 2.0f, 3.0f);
  I.look_at = v3(0.0f, 0.0f, 0.0f);
  I.background = v3(0.7f, 0.8f, 1.0f);
  switch (preset) {
    case 0: /* Random, application.rs:133-139 */
      I.aperture = 0.1f;
      sc->world = random_scene(B, 11);
      break;
    case 9: /* config 4: 10k spheres */
      I.aperture = 0.1f;
      sc->world = random_scene(B, 50);
      break;
    case 12: /* moving spheres with their own shutter intervals */
      I.aperture = 0.05f;
      sc->world = motion_scene(B);
      break;
    case 11: /* 40k spheres (a device-built walk hierarchy in the library) */
      I.aperture = 0.1f;
      sc->world = random_scene(B, 100);
      break;
    case 1: { /* TwoSpheres :567-587 */
      MatP checker = lambert(
          std::make_shared<CheckerTexture>(solid(0.2f, 0.3f, 0.1f), solid(0.9f, 0.9f, 0.9f)));
      std::vector<HitP> o;
      o.emplace_back(new Sphere(v3(0.0f, -10.0f, 0.0f), 10.0f, checker));
      o.emplace_back(new Sphere(v3(0.0f, 10.0f, 0.0f), 10.0f, checker));
      sc->world.reset(new BvhNode(std::move(o), 0.0f, 1.0f));
      break;
    }
    case 2: { /* TwoPerlinSpheres :589-602 */
      MatP noise = lambert(B.noise(4.0f));
      std::vector<HitP> o;
      o.emplace_back(new Sphere(v3(0.0f, -1000.0f, 0.0f), 1000.0f, noise));
      o.emplace_back(new Sphere(v3(0.0f, 2.0f, 0.0f), 2.0f, noise));
      sc->world.reset(new BvhNode(std::move(o), 0.0f, 1.0f));
      break;
    }
    case 3: { /* Earth :604-612 */
      std::vector<HitP> o;
      o.emplace_back(new Sphere(v3(0.0f, 0.0f, 0.0f), 2.0f, lambert(B.image())));
      sc->world.reset(new BvhNode(std::move(o), 0.0f, 1.0f));
      break;
    }
    case 8: { /* config 3: Earth at (0,2,0) over the Perlin ground */
      std::vector<HitP> o;
      o.emplace_back(new Sphere(v3(0.0f, -1000.0f, 0.0f), 1000.0f, lambert(B.noise(4.0f))));
      o.emplace_back(new Sphere(v3(0.0f, 2.0f, 0.0f), 2.0f, lambert(B.image())));
      sc->world.reset(new BvhNode(std::move(o), 0.0f, 1.0f));
      break;
    }
    case 4: { /* SimpleLight :614-637, camera :165-171 */
      I.look_from = v3(26.0f, 3.0f, 6.0f);
      I.look_at = v3(0.0f, 2.0f, 0.0f);
      I.background = v3(0.0f, 0.0f, 0.0f);
      MatP noise = lambert(B.noise(4.0f));
      std::vector<HitP> o;
      o.emplace_back(new Sphere(v3(0.0f, -1000.0f, 0.0f), 1000.0f, noise));
      o.emplace_back(new Sphere(v3(0.0f, 2.0f, 0.0f), 2.0f, noise));
      o.emplace_back(new Rect(0, 3.0f, 5.0f, 1.0f, 3.0f, -2.0f,
                              std::make_shared<DiffuseLight>(solid(4.0f, 4.0f, 4.0f))));
      sc->world.reset(new BvhNode(std::move(o), 0.0f, 1.0f));
      break;
    }
    case 5:   /* Cornell :639-721 */
    case 6: { /* CornellSmoke :723-815; camera :173-187 */
      I.look_from = v3(278.0f, 278.0f, -800.0f);
      I.look_at = v3(278.0f, 278.0f, 0.0f);
      I.fov = 40.0f;
      I.background = v3(0.0f, 0.0f, 0.0f);
      std::vector<HitP> o;
      MatP white;
      cornell_walls(o, white);
      HitP c1(new Cuboid(v3(0.0f, 0.0f, 0.0f), v3(165.0f, 330.0f, 165.0f), white));
      c1.reset(new Rotation(1, std::move(c1), 15.0f));
      c1.reset(new Translation(std::move(c1), v3(265.0f, 0.0f, 295.0f)));
      if (preset == 6) c1 = B.medium(std::move(c1), 0.01f, solid(0.0f, 0.0f, 0.0f));
      o.push_back(std::move(c1));
      HitP c2(new Cuboid(v3(0.0f, 0.0f, 0.0f), v3(165.0f, 165.0f, 165.0f), white));
      c2.reset(new Rotation(1, std::move(c2), -18.0f));
      c2.reset(new Translation(std::move(c2), v3(130.0f, 0.0f, 65.0f)));
      if (preset == 6) c2 = B.medium(std::move(c2), 0.01f, solid(1.0f, 1.0f, 1.0f));
      o.push_back(std::move(c2));
      sc->world.reset(new BvhNode(std::move(o), 0.0f, 1.0f));
      break;
    }
    case 7: { /* Final :817-935, camera :189-195 */
      I.look_from = v3(478.0f, 278.0f, -600.0f);
      I.look_at = v3(278.0f, 278.0f, 0.0f);
      I.fov = 40.0f;
      I.background = v3(0.0f, 0.0f, 0.0f);
      Rng& rand = B.rand;
      MatP ground = lambert(solid(0.48f, 0.83f, 0.53f));
      std::vector<HitP> boxes;
      for (int i = 0; i < 20; i++)
        for (int j = 0; j < 20; j++) {
          float w = 100.0f;
          float x0 = -1000.0f + (float)i * w;
          float z0 = -1000.0f + (float)j * w;
          float y0 = 0.0f;
          float x1 = x0 + w;
          float y1 = rand.gen_range_f32(1.0f, 101.0f);
          float z1 = z0 + w;
          boxes.emplace_back(new Cuboid(v3(x0, y0, z0), v3(x1, y1, z1), ground));
        }
      std::vector<HitP> o;
      o.emplace_back(new BvhNode(std::move(boxes), 0.0f, 1.0f));
      o.emplace_back(new Rect(2, 123.0f, 423.0f, 147.0f, 412.0f, 554.0f,
                              std::make_shared<DiffuseLight>(solid(7.0f, 7.0f, 7.0f))));
      Vec3 center_1 = v3(400.0f, 400.0f, 200.0f);
      Vec3 center_2 = center_1 + v3(30.0f, 0.0f, 0.0f);
      o.emplace_back(new MovingSphere(center_1, center_2, 0.0f, 1.0f, 50.0f,
                                      lambert(solid(0.7f, 0.3f, 0.1f))));
      o.emplace_back(
          new Sphere(v3(260.0f, 150.0f, 45.0f), 50.0f, std::make_shared<Dielectric>(1.5f)));
      o.emplace_back(new Sphere(v3(0.0f, 150.0f, 145.0f), 50.0f,
                                std::make_shared<Metal>(v3(0.8f, 0.8f, 0.9f), 1.0f)));
      o.emplace_back(
          new Sphere(v3(360.0f, 150.0f, 145.0f), 70.0f, std::make_shared<Dielectric>(1.5f)));
      o.push_back(B.medium(
          HitP(new Sphere(v3(360.0f, 150.0f, 145.0f), 70.0f, std::make_shared<Dielectric>(1.5f))),
          0.2f, solid(0.2f, 0.4f, 0.9f)));
      o.push_back(B.medium(
          HitP(new Sphere(v3(0.0f, 0.0f, 0.0f), 5000.0f, std::make_shared<Dielectric>(1.5f))),
          0.0001f, solid(1.0f, 1.0f, 1.0f)));
      o.emplace_back(new Sphere(v3(400.0f, 200.0f, 400.0f), 100.0f, lambert(B.image())));
      o.emplace_back(new Sphere(v3(220.0f, 280.0f, 300.0f), 80.0f, lambert(B.noise(0.1f))));
      MatP white = lambert(solid(0.73f, 0.73f, 0.73f));
      std::vector<HitP> sb;
      for (int k = 0; k < 1000; k++) {
        float x = rand.gen_range_f32(0.0f, 165.0f);
        float y = rand.gen_range_f32(0.0f, 165.0f);
        float z = rand.gen_range_f32(0.0f, 165.0f);
        sb.emplace_back(new Sphere(v3(x, y, z), 10.0f, white));
      }
      o.emplace_back(new Translation(
          HitP(new Rotation(1, HitP(new BvhNode(std::move(sb), 0.0f, 1.0f)), 15.0f)),
          v3(-100.0f, 270.0f, 395.0f)));
      sc->world.reset(new BvhNode(std::move(o), 0.0f, 1.0f));
      break;
    }
    case 10: { /* build-defined feature coverage scene */
      I.look_from = v3(0.0f, 3.0f, 12.0f);
      I.look_at = v3(0.0f, 1.0f, 0.0f);
      I.fov = 35.0f;
      I.aperture = 0.05f;
      I.background = v3(0.15f, 0.18f, 0.25f);
      Rng& rand = B.rand;
      TexP img = B.image();
      std::vector<HitP> o;
      o.emplace_back(new Sphere(v3(0.0f, -1000.0f, 0.0f), 1000.0f,
                                lambert(std::make_shared<CheckerTexture>(B.noise(2.0f),
                                                                         solid(0.8f, 0.8f, 0.8f)))));
      {
        std::vector<HitP> l;
        l.emplace_back(new Sphere(v3(-3.0f, 1.0f, 0.0f), 1.0f, std::make_shared<Dielectric>(1.5f)));
        l.emplace_back(new MovingSphere(v3(-3.0f, 2.5f, 0.0f), v3(-2.5f, 2.5f, 0.0f), 0.25f, 0.75f,
                                        0.4f, std::make_shared<Metal>(v3(0.8f, 0.6f, 0.2f), 0.3f)));
        o.emplace_back(new List(std::move(l)));
      }
      o.emplace_back(new Translation(
          HitP(new Rotation(2, HitP(new Cuboid(v3(0.0f, 0.0f, 0.0f), v3(1.0f, 2.0f, 1.0f), lambert(img))),
                            30.0f)),
          v3(1.5f, 0.0f, -1.0f)));
      o.emplace_back(new Translation(
          HitP(new Rotation(0,
                            HitP(new Cuboid(v3(-0.5f, 0.0f, -0.5f), v3(0.5f, 1.0f, 0.5f),
                                            std::make_shared<Metal>(v3(0.7f, 0.7f, 0.7f), 0.05f))),
                            -20.0f)),
          v3(3.0f, 0.5f, 1.0f)));
      o.push_back(B.medium(
          HitP(new Translation(
              HitP(new Rotation(1,
                                HitP(new Cuboid(v3(0.0f, 0.0f, 0.0f), v3(1.0f, 1.0f, 1.0f),
                                                lambert(solid(0.73f, 0.73f, 0.73f)))),
                                45.0f)),
              v3(-1.0f, 0.0f, 2.0f))),
          0.8f, solid(0.2f, 0.4f, 0.9f)));
      o.emplace_back(new Rect(0, -1.0f, 1.0f, 3.0f, 4.0f, -3.0f,
                              std::make_shared<DiffuseLight>(solid(4.0f, 4.0f, 4.0f))));
      o.emplace_back(new Rect(1, 0.0f, 2.0f, -2.0f, 0.0f, -4.0f, lambert(img)));
      o.emplace_back(new Rect(
          2, -1.0f, 1.0f, -1.0f, 1.0f, 3.5f,
          std::make_shared<DiffuseLight>(
              std::make_shared<CheckerTexture>(solid(2.0f, 2.0f, 2.0f), solid(0.5f, 0.5f, 3.0f)))));
      {
        std::vector<HitP> sb;
        for (int k = 0; k < 20; k++) {
          float x = rand.gen_range_f32(0.0f, 1.5f);
          float y = rand.gen_range_f32(0.0f, 1.5f);
          float z = rand.gen_range_f32(0.0f, 1.5f);
          float r = rand.gen_f32(), g = rand.gen_f32(), b = rand.gen_f32();
          sb.emplace_back(new Sphere(v3(x, y, z), 0.15f, lambert(solid(r, g, b))));
        }
        o.emplace_back(new Translation(
            HitP(new Rotation(1, HitP(new BvhNode(std::move(sb), 0.0f, 1.0f)), 15.0f)),
            v3(-4.5f, 0.0f, -2.0f)));
      }
      o.emplace_back(new Sphere(v3(1.0f, 0.7f, 2.0f), 0.7f, lambert(B.noise(4.0f))));
      sc->world.reset(new BvhNode(std::move(o), 0.0f, 1.0f));
      break;
    }
    default:
      throw std::runtime_error("unknown preset");
  }
  sc->n_media = B.n_media;
  return sc.release();
}

/* ---------------------------------------------------------------- application.rs:477-495 */
static Vec3 ray_color(const Ray& ray, Vec3 background, const Hittable& world, uint32_t depth,
                      float t_min, Ctx& ctx) {
  if (depth == 0) return v3(0.0f, 0.0f, 0.0f);
  HitRecord rec;
  ctx.cnt->c[C_SEGMENTS]++;
  bool h = world.hit(ray, t_min, INF_F, rec, ctx);
  ctx.segment++;
  if (!h) return background;
  Vec3 emitted = rec.material->emitted(rec.u, rec.v, rec.point, ctx);
  Vec3 attenuation;
  Ray scattered;
  if (!rec.material->scatter(ray, rec, attenuation, scattered, ctx)) return emitted;
  Vec3 c = ray_color(scattered, background, world, depth - 1, t_min, ctx);
  return mul_elem(attenuation, c) + emitted;
}

struct RenderArgs {
  uint32_t W, H, spp, depth, sample_offset;
  uint64_t seed;
  float t_min;
  uint32_t x0, y0, w, h;
  float* out;
};

/* application.rs:393-475: 80x80 tiles over the region, one task per tile on a worker pool. */
static void render(const Scene& sc, const Camera& cam, const RenderArgs& A, int nthreads,
                   Counters& total) {
  const uint32_t tile = 80;
  uint32_t tx = (A.w + tile - 1) / tile, ty = (A.h + tile - 1) / tile;
  uint32_t ntiles = tx * ty;
  std::atomic<uint32_t> next(0);
  std::vector<Counters> per(nthreads > 0 ? nthreads : 1);
  float scale = 1.0f / (float)A.spp; /* application.rs:403 */
  auto worker = [&](int wid) {
    Counters& cnt = per[wid];
    for (;;) {
      uint32_t ti = next.fetch_add(1);
      if (ti >= ntiles) break;
      uint32_t lx = (ti % tx) * tile, ly = (ti / tx) * tile;
      uint32_t tw = std::min(tile, A.w - lx), th = std::min(tile, A.h - ly);
      for (uint32_t i = 0; i < tw * th; i++) {
        uint32_t x = A.x0 + lx + i % tw, y = A.y0 + ly + i / tw;
        uint32_t pixel = y * A.W + x;
        Vec3 pixel_color = v3(0.0f, 0.0f, 0.0f);
        for (uint32_t s = 0; s < A.spp; s++) {
          Ctx ctx;
          ctx.pkey = path_key(A.seed, pixel, A.sample_offset + s);
          ctx.rng = rng_from_key(ctx.pkey);
          ctx.cnt = &cnt;
          ctx.segment = 0;
          float u = ((float)x + ctx.rng.gen_f32()) / ((float)A.W - 1.0f);
          float v = ((float)y + ctx.rng.gen_f32()) / ((float)A.H - 1.0f);
          Ray ray = cam.get_ray(u, v, ctx.rng);
          pixel_color = pixel_color +
                        ray_color(ray, sc.info.background, *sc.world, A.depth, A.t_min, ctx);
          cnt.c[C_SAMPLES]++;
        }
        size_t o = 4 * ((size_t)(x - A.x0) + (size_t)A.w * (y - A.y0));
        A.out[o + 0] = sqrtf(pixel_color.x * scale);
        A.out[o + 1] = sqrtf(pixel_color.y * scale);
        A.out[o + 2] = sqrtf(pixel_color.z * scale);
        A.out[o + 3] = 1.0f;
        cnt.c[C_PIXELS]++;
      }
    }
  };
  if (nthreads <= 1) {
    worker(0);
  } else {
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; t++) th.emplace_back(worker, t);
    for (auto& t : th) t.join();
  }
  for (auto& p : per)
    for (int k = 0; k < C_COUNT; k++) total.c[k] += p.c[k];
}

static thread_local std::string g_err;

}  // namespace oracle

/* ======================================================================== C API (ctypes) */
using namespace oracle;

extern "C" {

const char* oracle_last_error(void) { return g_err.c_str(); }

/* info[0..15]: look_from(3) look_at(3) fov aperture focus_dist time0 time1 background(3) n_media */
void* oracle_preset_build(int preset, uint64_t seed, const uint8_t* img, uint32_t iw, uint32_t ih,
                          uint32_t ic, float* info) {
  try {
    Scene* s = build_preset(preset, seed, img, iw, ih, ic);
    if (info) {
      const PresetInfo& I = s->info;
      float v[16] = {I.look_from.x, I.look_from.y, I.look_from.z, I.look_at.x, I.look_at.y,
                     I.look_at.z, I.fov, I.aperture, I.focus_dist, I.time0, I.time1,
                     I.background.x, I.background.y, I.background.z, (float)s->n_media, 0.0f};
      memcpy(info, v, sizeof(v));
    }
    return s;
  } catch (const std::exception& e) {
    g_err = e.what();
    return nullptr;
  }
}

void oracle_scene_destroy(void* s) { delete static_cast<Scene*>(s); }

uint32_t oracle_scene_count(void* s) { return static_cast<Scene*>(s)->world->count(); }

int oracle_scene_bbox(void* s, float* out6) {
  Aabb b;
  if (!static_cast<Scene*>(s)->world->bounding_box(0.0f, 1.0f, b)) return 0;
  float v[6] = {b.minimum.x, b.minimum.y, b.minimum.z, b.maximum.x, b.maximum.y, b.maximum.z};
  memcpy(out6, v, sizeof(v));
  return 1;
}

/* counters[0..C_COUNT): segments aabb sphere moving rect medium tex_solid tex_checker tex_noise
 * tex_image samples pixels */
int oracle_render(void* scene, uint32_t W, uint32_t H, uint32_t spp, uint32_t depth,
                  uint32_t sample_offset, uint64_t seed, float t_min, uint32_t x0, uint32_t y0,
                  uint32_t w, uint32_t h, float* out, int nthreads, uint64_t* counters) {
  try {
    Scene* s = static_cast<Scene*>(scene);
    if (!s || !out || W < 2 || H < 2 || spp == 0 || x0 + w > W || y0 + h > H)
      throw std::runtime_error("bad render arguments");
    const PresetInfo& I = s->info;
    Camera cam(I.look_from, I.look_at, I.fov, I.aperture, I.focus_dist, I.time0, I.time1, (int)W,
               (int)H);
    RenderArgs A{W, H, spp, depth, sample_offset, seed, t_min, x0, y0, w, h, out};
    Counters total;
    render(*s, cam, A, nthreads, total);
    if (counters) memcpy(counters, total.c, sizeof(total.c));
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    return 1;
  }
}

/* Columns [x0, x0 + w) of a set of rows of the W x H frame (bench.py's CPU baseline and parity band:
 * full-width rows spread over the image, so the sample's rays per sample match the frame's; the GPU
 * config tests: short windows of a row).  Same per-pixel computation as render(); the tasks are
 * task_w-pixel row segments (80 = the reference's tile width) on the pool.  out: [n_rows][w][4]. */
int oracle_render_rows(void* scene, uint32_t W, uint32_t H, uint32_t spp, uint32_t depth,
                       uint32_t sample_offset, uint64_t seed, float t_min, const uint32_t* rows,
                       uint32_t n_rows, uint32_t x0, uint32_t w, uint32_t task_w, float* out, int nthreads,
                       uint64_t* counters) {
  try {
    Scene* s = static_cast<Scene*>(scene);
    if (!s || !out || !rows || W < 2 || H < 2 || spp == 0 || w == 0 || task_w == 0 || x0 + w > W)
      throw std::runtime_error("bad render arguments");
    for (uint32_t r = 0; r < n_rows; r++)
      if (rows[r] >= H) throw std::runtime_error("row outside the image");
    const PresetInfo& I = s->info;
    Camera cam(I.look_from, I.look_at, I.fov, I.aperture, I.focus_dist, I.time0, I.time1, (int)W, (int)H);
    const uint32_t seg = task_w, per_row = (w + seg - 1) / seg, ntasks = per_row * n_rows;
    std::atomic<uint32_t> next(0);
    const int nt = nthreads > 0 ? nthreads : 1;
    std::vector<Counters> per(nt);
    std::vector<std::string> errs(nt);
    auto worker = [&](int wid) {
      try {
        for (;;) {
          const uint32_t t = next.fetch_add(1);
          if (t >= ntasks) break;
          const uint32_t r = t / per_row, lx = (t % per_row) * seg;
          RenderArgs A{W, H, spp, depth, sample_offset, seed, t_min, x0 + lx, rows[r], std::min(seg, w - lx), 1u,
                       out + 4 * ((size_t)r * w + lx)};
          render(*s, cam, A, 1, per[wid]);
        }
      } catch (const std::exception& e) {
        errs[wid] = e.what();
      }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; t++) th.emplace_back(worker, t);
    worker(0);
    for (auto& t : th) t.join();
    for (auto& e : errs)
      if (!e.empty()) throw std::runtime_error(e);
    Counters total;
    for (auto& p : per)
      for (int k = 0; k < C_COUNT; k++) total.c[k] += p.c[k];
    if (counters) memcpy(counters, total.c, sizeof(total.c));
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    return 1;
  }
}

/* ---- unit entry points for the KAT fixtures (tests/golden) ---- */
/* out: origin llc horizontal vertical u v w (21) lens_radius t0 t1 */
void oracle_camera(const float* from, const float* at, float fov, float aperture, float focus,
                   float t0, float t1, int W, int H, float* out) {
  Camera c(v3(from[0], from[1], from[2]), v3(at[0], at[1], at[2]), fov, aperture, focus, t0, t1, W, H);
  Vec3 vs[7] = {c.origin, c.lower_left_corner, c.horizontal, c.vertical, c.u, c.v, c.w};
  for (int i = 0; i < 7; i++) { out[3 * i] = vs[i].x; out[3 * i + 1] = vs[i].y; out[3 * i + 2] = vs[i].z; }
  out[21] = c.lens_radius; out[22] = c.time_0; out[23] = c.time_1;
}
/* camera ray from explicit (s, t, disk, time): out origin(3) direction(3) time */
void oracle_camera_ray(const float* from, const float* at, float fov, float aperture, float focus,
                       int W, int H, float s, float t, const float* disk, float time, float* out) {
  Camera c(v3(from[0], from[1], from[2]), v3(at[0], at[1], at[2]), fov, aperture, focus, 0.0f, 1.0f, W, H);
  Ray r = c.ray_from(s, t, v3(disk[0], disk[1], disk[2]), time);
  float v[7] = {r.origin.x, r.origin.y, r.origin.z, r.direction.x, r.direction.y, r.direction.z, r.time};
  memcpy(out, v, sizeof(v));
}
int oracle_aabb_hit(const float* mn, const float* mx, const float* o, const float* d, float tmin,
                    float tmax) {
  Counters c;
  Ctx ctx;
  ctx.cnt = &c;
  Aabb b{v3(mn[0], mn[1], mn[2]), v3(mx[0], mx[1], mx[2])};
  Ray r{v3(o[0], o[1], o[2]), v3(d[0], d[1], d[2]), 0.0f};
  return b.hit(r, tmin, tmax, ctx) ? 1 : 0;
}
static void rec_out(const HitRecord& rec, float* out) {
  float v[10] = {rec.t, rec.point.x, rec.point.y, rec.point.z, rec.normal.x, rec.normal.y,
                 rec.normal.z, rec.u, rec.v, rec.front_face ? 1.0f : 0.0f};
  memcpy(out, v, sizeof(v));
}
/* kind 0 sphere (p: c3 r), 1 moving sphere (p: c0 c1 t0 t1 r), 2 rect (p: plane a0 a1 b0 b1 k);
 * ray: o3 d3 time; out: t point3 normal3 u v front_face */
int oracle_prim_hit(int kind, const float* p, const float* ray, float tmin, float tmax, float* out) {
  Counters c;
  Ctx ctx;
  ctx.cnt = &c;
  MatP m = lambert(solid(1.0f, 1.0f, 1.0f));
  Ray r{v3(ray[0], ray[1], ray[2]), v3(ray[3], ray[4], ray[5]), ray[6]};
  HitRecord rec;
  bool h;
  if (kind == 0) h = Sphere(v3(p[0], p[1], p[2]), p[3], m).hit(r, tmin, tmax, rec, ctx);
  else if (kind == 1)
    h = MovingSphere(v3(p[0], p[1], p[2]), v3(p[3], p[4], p[5]), p[6], p[7], p[8], m).hit(r, tmin, tmax, rec, ctx);
  else h = Rect((int)p[0], p[1], p[2], p[3], p[4], p[5], m).hit(r, tmin, tmax, rec, ctx);
  if (h) rec_out(rec, out);
  return h ? 1 : 0;
}
/* op 0 reflect(v,n) 1 refract(v,n,eta) 2 reflectance(cos,ri)->out[0] 3 normalize(v) 4 near_zero */
void oracle_vec_op(int op, const float* a, const float* b, float s, float* out) {
  Vec3 va = v3(a[0], a[1], a[2]), vb = v3(b[0], b[1], b[2]), r = v3(0, 0, 0);
  if (op == 0) r = reflect(va, vb);
  else if (op == 1) r = refract(va, vb, s);
  else if (op == 2) r.x = reflectance(a[0], s);
  else if (op == 3) r = normalize(va);
  else if (op == 4) r.x = near_zero(va) ? 1.0f : 0.0f;
  out[0] = r.x; out[1] = r.y; out[2] = r.z;
}
/* Perlin with explicit tables: op 0 noise(p), 1 turbulence(p, depth) */
float oracle_perlin(const float* ranvec, const uint32_t* perm, int op, const float* p, uint32_t depth) {
  PerlinNoise n(ranvec, perm);
  Vec3 q = v3(p[0], p[1], p[2]);
  return op == 0 ? n.noise(q) : n.turbulence(q, depth);
}
/* Perlin tables drawn from the scene stream (checks the Sattolo/normalize draw order) */
void oracle_perlin_tables(uint64_t seed, float* ranvec, uint32_t* perm) {
  Rng r = scene_rng(seed);
  PerlinNoise n(r);
  for (int i = 0; i < 256; i++) {
    ranvec[3 * i] = n.random_vectors[i].x; ranvec[3 * i + 1] = n.random_vectors[i].y;
    ranvec[3 * i + 2] = n.random_vectors[i].z;
    perm[i] = n.permutation_x[i]; perm[256 + i] = n.permutation_y[i]; perm[512 + i] = n.permutation_z[i];
  }
}
/* textures: op 0 checker((0.2,0.3,0.1),(0.9,0.9,0.9)) at p; 1 noise(scale) with tables; 2 image */
void oracle_texture(int op, const float* p, float u, float v, float scale, const float* ranvec,
                    const uint32_t* perm, const uint8_t* img, uint32_t iw, uint32_t ih, uint32_t ic,
                    float* out) {
  Counters c;
  Ctx ctx;
  ctx.cnt = &c;
  Vec3 q = v3(p[0], p[1], p[2]), r;
  if (op == 0) r = CheckerTexture(solid(0.2f, 0.3f, 0.1f), solid(0.9f, 0.9f, 0.9f)).value(u, v, q, ctx);
  else if (op == 1) r = NoiseTexture(std::make_shared<PerlinNoise>(ranvec, perm), scale).value(u, v, q, ctx);
  else r = ImageTexture(img, iw, ih, ic).value(u, v, q, ctx);
  out[0] = r.x; out[1] = r.y; out[2] = r.z;
}
/* shared deterministic math on the host (op as hrt_debug_device_math) */
void oracle_math(int op, const float* x, const float* y, float* out, uint32_t n) {
  for (uint32_t i = 0; i < n; i++) {
    float a = x[i], b = y ? y[i] : 0.0f, r = 0.0f;
    switch (op) {
      case 0: r = sin_f(a); break;
      case 1: r = cos_f(a); break;
      case 2: r = acos_f(a); break;
      case 3: r = atan2_f(a, b); break;
      case 4: r = ln_f(a); break;
      case 5: r = pow5_f(a); break;
      case 6: r = tan_f(a); break;
    }
    out[i] = r;
  }
}
/* glibc's f32 functions (the reference platform's arithmetic), op as oracle_math */
void oracle_math_libm(int op, const float* x, const float* y, float* out, uint32_t n) {
  for (uint32_t i = 0; i < n; i++) {
    float a = x[i], b = y ? y[i] : 0.0f, r = 0.0f;
    switch (op) {
      case 0: r = sinf(a); break;
      case 1: r = cosf(a); break;
      case 2: r = acosf(a); break;
      case 3: r = atan2f(a, b); break;
      case 4: r = logf(a); break;
      case 5: r = powf(a, 5.0f); break;
      case 6: r = tanf(a); break;
    }
    out[i] = r;
  }
}
/* 1: renders (and scene builds) use glibc's f32 transcendentals; 0: hd_math (the kernel's) */
void oracle_set_libm(int on) { g_libm = on ? 1 : 0; }
/* Record the arguments of every transcendental call into bufs[op] (pairs (a, b), up to cap per op;
 * bufs == NULL stops recording).  counts[op] receives the number of calls seen. */
void oracle_record_math(float** bufs, uint32_t cap, uint32_t* counts) {
  if (counts)
    for (int k = 0; k < OP_N; k++) counts[k] = g_rec_n[k].load();
  for (int k = 0; k < OP_N; k++) {
    g_rec[k] = bufs ? bufs[k] : nullptr;
    g_rec_n[k] = 0;
  }
  g_rec_cap = bufs ? cap : 0;
}
/* raw RNG streams: mode 0 gen_f32, 1 gen_range(-1,1), 2 next_u32 (as float bits) */
void oracle_rng(uint64_t seed, uint32_t pixel, uint32_t sample, int mode, uint32_t n, float* out) {
  Rng r = rng_from_key(path_key(seed, pixel, sample));
  for (uint32_t i = 0; i < n; i++) {
    if (mode == 0) out[i] = r.gen_f32();
    else if (mode == 1) out[i] = r.gen_range_f32(-1.0f, 1.0f);
    else out[i] = u2f(r.next_u32());
  }
}

}  // extern "C"
