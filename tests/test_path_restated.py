"""The whole per-pixel path of the headline scene restated a third time, in Python, from the Rust sources, and held
bit for bit to the CPU oracle (which the GPU is held to by tests/test_gpu_parity.py and bench.py's parity band).

The oracle (oracle/oracle.cpp) and the library (csrc/lane.h) share include/hrt/hd_math.h, so a misreading of the
path itself -- the sample loop's draw order (application.rs:443-453), Camera::get_ray (camera.rs:85-95),
BvhNode::hit's left-then-right walk with the shrinking t_max (bvh_node.rs:104-127), ray_color's recursion
(application.rs:477-495), the materials' scatter and their draws (lambertian.rs:27-38, metal.rs:29-42,
dielectric.rs:31-55), the checker texture -- would be shared by both.  This test restates that path on numpy
float32 scalars (one IEEE rounding per operation, cgmath's operation order) with the unit functions of the KAT
generator (tests/golden/make_kats.py: aabb.rs, sphere.rs, moving_sphere.rs, camera.rs, math.rs, checker_texture.rs,
the seeded per-sample RNG with rand 0.8.5's transforms) and the scene of tests/test_scene_builders.py (which is
held to the library's lowered scene), renders a few pixels of the Random scene (configs 1-2) and of Cornell (config
5: rect.rs, list.rs, rotation.rs -- whose hit turns the normal back without set_face_normal -- translation.rs,
diffuse_light.rs), and compares colour and world.hit count with the oracle's render of the same pixels: equal
bits, equal counts.  Parity against the reference binary
stays unpinned (it cannot run here); this pins the C++ restatements against an independent reading."""
import os
import sys

import numpy as np
import pytest

import hrt
from oracle import oracle as O

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import test_scene_builders as SB  # noqa: E402

K = SB.K
f = np.float32
INF = f(np.inf)


class Bvh:
    """BvhNode::new's tree (bvh_node.rs:27-63) over the scene's objects, with each node's box."""

    def __init__(self, objs, t0=0.0, t1=1.0):
        objs = list(objs)
        ranges = []
        for axis in range(3):
            mn, mx = f(np.finfo(np.float32).max), f(np.finfo(np.float32).min)
            for o in objs:
                b = SB.bbox(o, t0, t1)
                mn, mx = min(mn, b[0][axis]), max(mx, b[1][axis])
            ranges.append((axis, mx - mn))
        ranges.sort(key=lambda ar: -ar[1])
        axis = ranges[0][0]
        objs.sort(key=lambda o: SB.bbox(o, t0, t1)[0][axis] + SB.bbox(o, t0, t1)[1][axis])
        if len(objs) == 1:
            self.leaf, self.left, self.right = objs[0], None, None
            self.box = SB.bbox(objs[0], t0, t1)
            return
        half = len(objs) // 2
        self.leaf = None
        self.right = Bvh(objs[half:], t0, t1)
        self.left = Bvh(objs[:half], t0, t1)
        self.box = SB.surrounding(self.left.box, self.right.box)

    def hit(self, o, d, time, tmin, tmax):
        """BvhNode::hit (bvh_node.rs:104-127): the box, then the left child, the right one with t_max shrunk."""
        if not K.aabb_hit(self.box[0], self.box[1], o, d, tmin, tmax):
            return None
        if self.leaf is not None:
            kind, c0, c1, r, mat = self.leaf
            c = c0 if kind == "sphere" else K.moving_center(c0, c1, f(0), f(1), time)  # moving_sphere.rs:53-58
            h = K.sphere_hit(c, r, o, d, tmin, tmax)
            return None if h is None else (h, mat)
        left = self.left.hit(o, d, time, tmin, tmax)
        right = self.right.hit(o, d, time, tmin, left[0][0] if left is not None else tmax)
        return right if right is not None else left


def random_in_unit_sphere(rng):  # math.rs:16-30 (Uniform(-1, 1): the gen_range bits, no retry needed)
    while True:
        p = (rng.gen_range(-1.0, 1.0), rng.gen_range(-1.0, 1.0), rng.gen_range(-1.0, 1.0))
        if K.dot(p, p) < f(1):
            return p


def random_in_unit_disk(rng):  # math.rs:32-40
    while True:
        p = (rng.gen_range(-1.0, 1.0), rng.gen_range(-1.0, 1.0), f(0))
        if K.dot(p, p) < f(1):
            return p


def scatter(mat, rng, d, rec):
    """(attenuation, direction) or None (materials/*.rs scatter)."""
    t, px, py, pz, nx, ny, nz, u, v, front = rec
    p, n = (px, py, pz), (nx, ny, nz)
    kind = mat[0]
    if kind in ("lambertian", "lambertian_checker"):  # lambertian.rs:27-38
        sd = K.add(n, K.norm(random_in_unit_sphere(rng)))
        if K.near_zero(sd):
            sd = n
        att = mat[1] if kind == "lambertian" else (mat[1] if K.checker(p) == K.F3((0.2, 0.3, 0.1)) else mat[2])
        return att, sd
    if kind == "metal":  # metal.rs:29-42
        refl = K.reflect(K.norm(d), n)
        sd = K.add(refl, K.smul(mat[2], random_in_unit_sphere(rng)))
        return (mat[1], sd) if K.dot(sd, n) > f(0) else None
    ratio = (f(1) / mat[1]) if front else mat[1]  # dielectric.rs:31-55
    ud = K.norm(d)
    cos_t = min(K.dot(K.neg(ud), n), f(1))
    sin_t = np.sqrt(f(1) - cos_t * cos_t)
    if (ratio * sin_t) > f(1) or K.reflectance(cos_t, ratio) > rng.gen_f32():
        sd = K.reflect(ud, n)
    else:
        sd = K.refract(ud, n, ratio)
    return (f(1), f(1), f(1)), sd


def ray_color(world, o, d, time, background, depth, rng, count):
    """application.rs:477-495, recursive as the reference is."""
    if depth == 0:
        return (f(0), f(0), f(0))
    count[0] += 1
    h = world.hit(o, d, time, f(0.001), INF)
    if h is None:
        return background
    rec, mat = h
    s = scatter(mat, rng, d, rec)
    emitted = (f(0), f(0), f(0))
    if s is None:
        return emitted
    att, sd = s
    col = ray_color(world, (rec[1], rec[2], rec[3]), sd, time, background, depth - 1, rng, count)
    return K.add((att[0] * col[0], att[1] * col[1], att[2] * col[2]), emitted)


def render_pixel(world, cam, bg, W, H, x, y, spp, depth, seed, count):
    """The sample loop (application.rs:443-456) for one pixel: each sample on its own keyed stream (the thread_rng
    substitution), u and v jitter, Camera::get_ray (lens disk, then the shutter time), the colours summed."""
    total = (f(0), f(0), f(0))
    for s in range(spp):
        rng = K.Rng(K.path_key(seed, y * W + x, s))
        u = (f(x) + rng.gen_f32()) / (f(W) - f(1))
        v = (f(y) + rng.gen_f32()) / (f(H) - f(1))
        disk = random_in_unit_disk(rng)
        time = rng.gen_range(0.0, 1.0)
        r = K.camera_ray(cam, u, v, disk, time)
        total = K.add(total, ray_color(world, tuple(r[0:3]), tuple(r[3:6]), r[6], bg, depth, rng, count))
    scale = f(1) / f(spp)
    return tuple(np.sqrt(c * scale) for c in total)


@pytest.mark.parametrize("x,y", [(20, 10), (45, 22), (5, 30), (33, 17), (60, 2), (31, 12)])
def test_random_scene_path_equals_oracle_bit_for_bit(x, y):
    """Pixels of the Random scene at 64 x 36, 16 spp, depth 50 (spheres, moving spheres, Lambertian solid and
    checker, Metal, Dielectric): the restated path's colour and world.hit count equal the oracle's exactly."""
    W, H, spp, depth, seed = 64, 36, 16, 50, 3
    s = hrt.preset("random", 1)
    info = s.info
    world = Bvh(SB.random_scene(K.scene_rng(1)))
    cam = K.camera(K.F3(info.look_from), K.F3(info.look_at), f(info.fov), f(info.aperture), f(info.focus_dist), W, H)
    bg = K.F3(info.background)
    count = [0]
    got = render_pixel(world, cam, bg, W, H, x, y, spp, depth, seed, count)
    ref, cnt = O.OracleScene(hrt.PRESETS["random"], 1).render(W, H, spp, depth, seed=seed, region=(x, y, 1, 1), threads=1)
    assert count[0] == cnt["segments"], (count[0], cnt["segments"])
    for c in range(3):
        assert np.float32(got[c]).view(np.uint32) == np.float32(ref[0, 0, c]).view(np.uint32), (c, got, ref[0, 0, :3])


def test_restated_path_has_teeth():
    """One misreading in the sample loop (v's jitter drawn before u's) changes the restated pixel: the equality
    above is not a comparison that anything passes."""
    W, H, spp, depth, seed, x, y = 64, 36, 16, 50, 3, 33, 17
    info = hrt.preset("random", 1).info
    world = Bvh(SB.random_scene(K.scene_rng(1)))
    cam = K.camera(K.F3(info.look_from), K.F3(info.look_at), f(info.fov), f(info.aperture), f(info.focus_dist), W, H)
    bg = K.F3(info.background)
    good = render_pixel(world, cam, bg, W, H, x, y, spp, depth, seed, [0])
    total = (f(0), f(0), f(0))
    for s in range(spp):
        rng = K.Rng(K.path_key(seed, y * W + x, s))
        v = (f(y) + rng.gen_f32()) / (f(H) - f(1))
        u = (f(x) + rng.gen_f32()) / (f(W) - f(1))
        r = K.camera_ray(cam, u, v, random_in_unit_disk(rng), rng.gen_range(0.0, 1.0))
        total = K.add(total, ray_color(world, tuple(r[0:3]), tuple(r[3:6]), r[6], bg, depth, rng, [0]))
    bad = tuple(np.sqrt(c * (f(1) / f(spp))) for c in total)
    assert good != bad


# ------------------------------------------------------------------------------- Cornell (application.rs:639-721)
class Rect:  # rect.rs:53-102
    def __init__(self, r, mat):
        self.r, self.mat = r, mat

    def box(self):
        return SB.rect_box(self.r)

    def hit(self, o, d, time, tmin, tmax):
        h = K.rect_hit(*self.r, o, d, tmin, tmax)
        return None if h is None else (h, self.mat)


class HList:  # list.rs:20-31 (a Cuboid's sides, cuboid.rs)
    def __init__(self, items):
        self.items = items

    def hit(self, o, d, time, tmin, tmax):
        closest, best = tmax, None
        for it in self.items:
            h = it.hit(o, d, time, tmin, closest)
            if h is not None:
                closest, best = h[0][0], h
        return best


class Rotate:  # rotation.rs:38-134 (the normal turned back, no set_face_normal)
    def __init__(self, axis, child, angle, child_box):
        import math

        self.child = child
        _, self.a, self.b = {0: (0, 1, 2), 1: (1, 2, 0), 2: (2, 0, 1)}[axis]
        radians = (f(math.pi) / f(180.0)) * f(angle)
        self.s, self.c = f(math.sin(float(radians))), f(math.cos(float(radians)))
        self.bx = SB.rotated_box(child_box, axis, angle)

    def box(self):
        return self.bx

    def hit(self, o, d, time, tmin, tmax):
        a, b, s, c = self.a, self.b, self.s, self.c
        o2, d2 = list(o), list(d)
        o2[a], o2[b] = c * o[a] + s * o[b], -s * o[a] + c * o[b]
        d2[a], d2[b] = c * d[a] + s * d[b], -s * d[a] + c * d[b]
        h = self.child.hit(tuple(o2), tuple(d2), time, tmin, tmax)
        if h is None:
            return None
        rec, mat = h
        p, n = list(rec[1:4]), list(rec[4:7])
        p[a], p[b] = c * rec[1 + a] - s * rec[1 + b], s * rec[1 + a] + c * rec[1 + b]
        n[a], n[b] = c * rec[4 + a] - s * rec[4 + b], s * rec[4 + a] + c * rec[4 + b]
        return [rec[0], *p, *n, *rec[7:]], mat


class Translate:  # translation.rs:24-47
    def __init__(self, child, off):
        self.child, self.off = child, off

    def box(self):
        b = self.child.box()
        return SB.vadd(b[0], self.off), SB.vadd(b[1], self.off)

    def hit(self, o, d, time, tmin, tmax):
        mo = SB.vsub(o, self.off)
        h = self.child.hit(mo, d, time, tmin, tmax)
        if h is None:
            return None
        rec, mat = h
        front, n = K.face(d, tuple(rec[4:7]))  # set_face_normal(moved_ray, normal)
        return [rec[0], *SB.vadd(tuple(rec[1:4]), self.off), *n, rec[7], rec[8], f(1) if front else f(0)], mat


class Bvh2:
    """BvhNode::new / ::hit over objects with box() and hit() (bvh_node.rs:27-127)."""

    def __init__(self, idx, objs):
        ranges = []
        for axis in range(3):
            mn, mx = f(np.finfo(np.float32).max), f(np.finfo(np.float32).min)
            for i in idx:
                b = objs[i].box()
                mn, mx = min(mn, b[0][axis]), max(mx, b[1][axis])
            ranges.append((axis, mx - mn))
        ranges.sort(key=lambda ar: -ar[1])
        axis = ranges[0][0]
        idx = sorted(idx, key=lambda i: objs[i].box()[0][axis] + objs[i].box()[1][axis])
        if len(idx) == 1:
            self.leaf, self.bx = objs[idx[0]], objs[idx[0]].box()
            return
        half = len(idx) // 2
        self.leaf = None
        self.right, self.left = Bvh2(idx[half:], objs), Bvh2(idx[:half], objs)
        self.bx = SB.surrounding(self.left.bx, self.right.bx)

    def hit(self, o, d, time, tmin, tmax):
        if not K.aabb_hit(self.bx[0], self.bx[1], o, d, tmin, tmax):
            return None
        if self.leaf is not None:
            return self.leaf.hit(o, d, time, tmin, tmax)
        left = self.left.hit(o, d, time, tmin, tmax)
        right = self.right.hit(o, d, time, tmin, left[0][0] if left is not None else tmax)
        return right if right is not None else left


def cornell_world(smoke=False):
    red, white, green = ("lambertian", SB.v3(0.65, 0.05, 0.05)), ("lambertian", SB.v3(0.73, 0.73, 0.73)), \
        ("lambertian", SB.v3(0.12, 0.45, 0.15))
    light = ("light", SB.v3(15, 15, 15))
    F = lambda *x: tuple(f(v) for v in x)  # noqa: E731
    objs = [Rect(F(1, 0, 555, 0, 555, 555), green), Rect(F(1, 0, 555, 0, 555, 0), red),
            Rect(F(2, 213, 343, 227, 332, 554), light), Rect(F(2, 0, 555, 0, 555, 0), white),
            Rect(F(2, 0, 555, 0, 555, 555), white), Rect(F(0, 0, 555, 0, 555, 555), white)]
    for size, angle, off in ((SB.v3(165, 330, 165), 15.0, SB.v3(265, 0, 295)), (SB.v3(165, 165, 165), -18.0, SB.v3(130, 0, 65))):
        sides = HList([Rect(tuple(f(v) for v in r), white) for r in SB.cuboid_rects(SB.v3(0, 0, 0), size)])
        obj = Translate(Rotate(1, sides, angle, (SB.v3(0, 0, 0), size)), off)
        if smoke:  # application.rs:723-815: each box a ConstantMedium of density 0.01, black then white smoke
            n = len(objs) - 6
            obj = Medium(obj, 0.01, SB.v3(0, 0, 0) if n == 0 else SB.v3(1, 1, 1), n)
        objs.append(obj)
    return Bvh2(list(range(len(objs))), objs)


def ray_color_full(world, o, d, time, background, depth, rng, count):
    """application.rs:477-495 with emission (DiffuseLight: no scatter, emitted = its colour, diffuse_light.rs)."""
    if depth == 0:
        return (f(0), f(0), f(0))
    count[0] += 1
    h = world.hit(o, d, time, f(0.001), INF)
    if h is None:
        return background
    rec, mat = h
    if mat[0] == "light":
        return mat[1]
    s = scatter(mat, rng, d, rec)
    if s is None:
        return (f(0), f(0), f(0))
    att, sd = s
    col = ray_color_full(world, (rec[1], rec[2], rec[3]), sd, time, background, depth - 1, rng, count)
    return K.add((att[0] * col[0], att[1] * col[1], att[2] * col[2]), (f(0), f(0), f(0)))


@pytest.mark.parametrize("x,y", [(20, 10), (30, 12), (8, 30), (25, 5), (14, 20)])
def test_cornell_path_equals_oracle_bit_for_bit(x, y):
    """Pixels of Cornell (config 5's scene) at 40 x 40, 24 spp: the restated path -- Rects (rect.rs), the cuboids'
    sides as Lists, Rotation without set_face_normal and Translation with it, the light's emission -- equals the
    oracle's colours and world.hit counts exactly."""
    W, H, spp, depth, seed = 40, 40, 24, 50, 5
    info = hrt.preset("cornell", 1).info
    world = cornell_world()
    cam = K.camera(K.F3(info.look_from), K.F3(info.look_at), f(info.fov), f(info.aperture), f(info.focus_dist), W, H)
    bg = K.F3(info.background)
    count = [0]
    total = (f(0), f(0), f(0))
    for s in range(spp):
        rng = K.Rng(K.path_key(seed, y * W + x, s))
        u = (f(x) + rng.gen_f32()) / (f(W) - f(1))
        v = (f(y) + rng.gen_f32()) / (f(H) - f(1))
        r = K.camera_ray(cam, u, v, random_in_unit_disk(rng), rng.gen_range(float(info.time0), float(info.time1)))
        total = K.add(total, ray_color_full(world, tuple(r[0:3]), tuple(r[3:6]), r[6], bg, depth, rng, count))
    got = tuple(np.sqrt(c * (f(1) / f(spp))) for c in total)
    ref, cnt = O.OracleScene(hrt.PRESETS["cornell"], 1).render(W, H, spp, depth, seed=seed, region=(x, y, 1, 1), threads=1)
    assert count[0] == cnt["segments"], (count[0], cnt["segments"])
    for c in range(3):
        assert np.float32(got[c]).view(np.uint32) == np.float32(ref[0, 0, c]).view(np.uint32), (c, got, ref[0, 0, :3])


# ------------------------------------------------------------------------------- Final (application.rs:817-935)
class Sphere:  # sphere.rs / moving_sphere.rs (a moving one when c1 is given, over the shutter [0, 1])
    def __init__(self, c0, r, mat, c1=None):
        self.c0, self.c1, self.r, self.mat = c0, c1, f(r), mat

    def centre(self, time):
        return self.c0 if self.c1 is None else K.moving_center(self.c0, self.c1, f(0), f(1), time)

    def box(self):
        if self.c1 is None:
            return SB.sphere_box(self.c0, self.r)
        return SB.surrounding(SB.sphere_box(self.centre(f(0)), self.r), SB.sphere_box(self.centre(f(1)), self.r))

    def hit(self, o, d, time, tmin, tmax):
        h = K.sphere_hit(self.centre(time), self.r, o, d, tmin, tmax)
        return None if h is None else (h, self.mat)


class Cuboid(HList):  # cuboid.rs: its six sides as a List, its box (box_min, box_max)
    def __init__(self, p0, p1, mat):
        super().__init__([Rect(r, mat) for r in SB.cuboid_rects(p0, p1)])
        self.bx = (p0, p1)

    def box(self):
        return self.bx


class Medium:  # constant_medium.rs:34-76; the draw keyed by (path, segment, medium id): hd_math.h medium_xi
    def __init__(self, boundary, density, albedo, medium_id):
        self.boundary, self.nid, self.mat, self.id = boundary, f(-1.0) / f(density), ("isotropic", albedo), medium_id

    def box(self):
        return self.boundary.box()

    def hit(self, o, d, time, tmin, tmax, key=None):
        r1 = self.boundary.hit(o, d, time, -INF, INF)
        if r1 is None:
            return None
        r2 = self.boundary.hit(o, d, time, r1[0][0] + f(0.0001), INF)
        if r2 is None:
            return None
        t1, t2 = r1[0][0], r2[0][0]
        t1 = tmin if t1 < tmin else t1
        t2 = tmax if t2 > tmax else t2
        if t1 >= t2:
            return None
        t1 = f(0) if t1 < f(0) else t1
        length = np.sqrt(K.dot(d, d))
        inside = (t2 - t1) * length
        pkey, segment = PATH[0], PATH[1]
        k = K.mix64(pkey ^ K.mix64(0xC2B2AE3D27D4EB4F ^ ((segment << 32) | self.id)))
        xi = f((k >> 32) >> 8) * f(2.0 ** -24)
        hit_distance = self.nid * (f(np.log(np.float64(xi))) / f(np.log(np.float64(f(np.e)))))
        if hit_distance > inside:
            return None
        t = t1 + hit_distance / length
        return [t, *K.at(o, d, t), f(0), f(0), f(0), f(0), f(0), f(0)], self.mat


PATH = [0, 0]  # the current sample's path key and segment index (the medium draw's key)


def final_world(earth):
    ground, (ranvec, perms), centres = SB.final_draws(K.scene_rng(1))
    green = ("lambertian", SB.v3(0.48, 0.83, 0.53))
    objs = [Bvh2(list(range(400)), [Cuboid(p0, p1, green) for p0, p1 in ground])]
    F = lambda *x: tuple(f(v) for v in x)  # noqa: E731
    objs.append(Rect(F(2, 123, 423, 147, 412, 554), ("light", SB.v3(7, 7, 7))))
    objs.append(Sphere(SB.v3(400, 400, 200), 50, ("lambertian", SB.v3(0.7, 0.3, 0.1)), c1=SB.vadd(SB.v3(400, 400, 200), SB.v3(30, 0, 0))))
    objs.append(Sphere(SB.v3(260, 150, 45), 50, ("dielectric", f(1.5))))
    objs.append(Sphere(SB.v3(0, 150, 145), 50, ("metal", SB.v3(0.8, 0.8, 0.9), f(1.0))))
    objs.append(Sphere(SB.v3(360, 150, 145), 70, ("dielectric", f(1.5))))
    objs.append(Medium(Sphere(SB.v3(360, 150, 145), 70, ("dielectric", f(1.5))), 0.2, SB.v3(0.2, 0.4, 0.9), 0))
    objs.append(Medium(Sphere(SB.v3(0, 0, 0), 5000, ("dielectric", f(1.5))), 0.0001, SB.v3(1, 1, 1), 1))
    objs.append(Sphere(SB.v3(400, 200, 400), 100, ("image", earth)))
    objs.append(Sphere(SB.v3(220, 280, 300), 80, ("noise", f(0.1), ranvec, perms)))
    white = ("lambertian", SB.v3(0.73, 0.73, 0.73))
    inner = Bvh2(list(range(1000)), [Sphere(c, 10, white) for c in centres])
    inner.box = lambda: inner.bx
    objs.append(Translate(Rotate(1, inner, 15.0, inner.bx), SB.v3(-100, 270, 395)))
    for o in objs:
        if isinstance(o, Bvh2):
            o.box = (lambda b: (lambda: b))(o.bx)
    return Bvh2(list(range(len(objs))), objs)


def shade_final(mat, rng, d, rec):
    """(attenuation, direction) or None, with the Next-Week materials and textures (noise_texture.rs:24-31,
    image_texture.rs:36-62, isotropic.rs:26-33)."""
    p = tuple(rec[1:4])
    if mat[0] == "image":
        return K.image_tex(mat[1], rec[7], rec[8]), scatter(("lambertian", (f(0), f(0), f(0))), rng, d, rec)[1]
    if mat[0] == "noise":
        att = K.noise_tex(mat[2], mat[3], mat[1], p)
        return att, scatter(("lambertian", (f(0), f(0), f(0))), rng, d, rec)[1]
    if mat[0] == "isotropic":
        return mat[1], random_in_unit_sphere(rng)
    return scatter(mat, rng, d, rec)


def ray_color_final(world, o, d, time, background, depth, rng, count):
    if depth == 0:
        return (f(0), f(0), f(0))
    count[0] += 1
    h = world.hit(o, d, time, f(0.001), INF)
    PATH[1] += 1
    if h is None:
        return background
    rec, mat = h
    if mat[0] == "light":
        return mat[1]
    s = shade_final(mat, rng, d, rec)
    if s is None:
        return (f(0), f(0), f(0))
    att, sd = s
    col = ray_color_final(world, tuple(rec[1:4]), sd, time, background, depth - 1, rng, count)
    return K.add((att[0] * col[0], att[1] * col[1], att[2] * col[2]), (f(0), f(0), f(0)))


@pytest.mark.parametrize("x,y", [(20, 12), (12, 25), (28, 20), (6, 8), (3, 15), (18, 18), (33, 12), (9, 36), (24, 15)])
def test_final_path_equals_oracle_bit_for_bit(x, y, earth):
    """Pixels of Final at 40 x 40, 4 spp: the ground's Cuboids, the light, a moving sphere, glass, metal, the blue
    medium inside its glass sphere and the fog (ConstantMedium: two boundary hits, the logarithm of the keyed draw),
    the Earth (image texture through the sphere's u, v), the Perlin sphere (turbulence) and the 1000 spheres in a
    rotated, translated BvhNode (pixels chosen so that primary rays hit each of them): colours and world.hit counts
    equal the oracle's exactly."""
    W, H, spp, depth, seed = 40, 40, 4, 50, 7
    info = hrt.preset("final", 1, earth).info
    world = final_world(np.ascontiguousarray(earth, np.uint8))
    cam = K.camera(K.F3(info.look_from), K.F3(info.look_at), f(info.fov), f(info.aperture), f(info.focus_dist), W, H)
    bg = K.F3(info.background)
    count = [0]
    total = (f(0), f(0), f(0))
    for s in range(spp):
        PATH[0], PATH[1] = K.path_key(seed, y * W + x, s), 0
        rng = K.Rng(PATH[0])
        u = (f(x) + rng.gen_f32()) / (f(W) - f(1))
        v = (f(y) + rng.gen_f32()) / (f(H) - f(1))
        r = K.camera_ray(cam, u, v, random_in_unit_disk(rng), rng.gen_range(float(info.time0), float(info.time1)))
        total = K.add(total, ray_color_final(world, tuple(r[0:3]), tuple(r[3:6]), r[6], bg, depth, rng, count))
    got = tuple(np.sqrt(c * (f(1) / f(spp))) for c in total)
    ref, cnt = O.OracleScene(hrt.PRESETS["final"], 1, earth).render(W, H, spp, depth, seed=seed, region=(x, y, 1, 1),
                                                                    threads=1)
    assert count[0] == cnt["segments"], (count[0], cnt["segments"])
    for c in range(3):
        assert np.float32(got[c]).view(np.uint32) == np.float32(ref[0, 0, c]).view(np.uint32), (c, got, ref[0, 0, :3])


@pytest.mark.parametrize("x,y", [(20, 10), (12, 14), (28, 16), (8, 30)])
def test_cornell_smoke_path_equals_oracle_bit_for_bit(x, y):
    """Cornell-smoke (application.rs:723-815): the two boxes are ConstantMedium boundaries inside Rotation and
    Translation -- the boundary queried twice through the instance chain, the keyed draw, the Isotropic scatter --
    the restated path equals the oracle's colours and world.hit counts exactly (40 x 40, 24 spp)."""
    W, H, spp, depth, seed = 40, 40, 24, 50, 11
    info = hrt.preset("cornell_smoke", 1).info
    world = cornell_world(smoke=True)
    cam = K.camera(K.F3(info.look_from), K.F3(info.look_at), f(info.fov), f(info.aperture), f(info.focus_dist), W, H)
    bg = K.F3(info.background)
    count = [0]
    total = (f(0), f(0), f(0))
    for s in range(spp):
        PATH[0], PATH[1] = K.path_key(seed, y * W + x, s), 0
        rng = K.Rng(PATH[0])
        u = (f(x) + rng.gen_f32()) / (f(W) - f(1))
        v = (f(y) + rng.gen_f32()) / (f(H) - f(1))
        r = K.camera_ray(cam, u, v, random_in_unit_disk(rng), rng.gen_range(float(info.time0), float(info.time1)))
        total = K.add(total, ray_color_final(world, tuple(r[0:3]), tuple(r[3:6]), r[6], bg, depth, rng, count))
    got = tuple(np.sqrt(c * (f(1) / f(spp))) for c in total)
    ref, cnt = O.OracleScene(hrt.PRESETS["cornell_smoke"], 1).render(W, H, spp, depth, seed=seed, region=(x, y, 1, 1),
                                                                     threads=1)
    assert count[0] == cnt["segments"], (count[0], cnt["segments"])
    for c in range(3):
        assert np.float32(got[c]).view(np.uint32) == np.float32(ref[0, 0, c]).view(np.uint32), (c, got, ref[0, 0, :3])
