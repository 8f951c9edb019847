"""The reference's scene builders restated a THIRD time, independently of the library (csrc/presets.cpp) and of
the oracle (oracle/oracle.cpp), and held to the library's lowered scene (What's weak 1: the product's
builders and the oracle's are twins, so a shared misreading of application.rs would pass every parity test).

This file is written from the Rust sources alone, in numpy float32 (one IEEE rounding per operation, cgmath's
operation order), on the seeded stream of tests/golden/make_kats.py (its own restatement of the RNG that replaces
thread_rng, with rand 0.8.5's transforms):
  - generate_random_scene (src/application.rs:497-565) and its 10k-sphere variant (config 4: a, b in [-50, 50));
  - Sphere / MovingSphere bounding boxes (src/hittable/sphere.rs:57-63, moving_sphere.rs:53-58, 98-110) and
    Aabb::surrounding_box (src/aabb.rs:49-66);
  - BvhNode::new (src/hittable/bvh_node.rs:27-63): the axis of the largest range (the ranges sorted descending,
    ties in axis order), the objects sorted by min + max on that axis (a stable sort: the substitution for
    sort_unstable_by documented in DESIGN.md section 2, identical below 21 objects), the right half built from
    objects[len / 2 ..], the left from the rest, leaves visited left first.
The library's flattened scene (hrt_debug_scene_blob, no device) lists its primitives in the reference's
pre-order; every leaf's primitive record (centre(s), radius, shutter) and its material and texture records must
equal the restatement's, bit for bit, in that order.  Final (application.rs:817-935): its draws (the ground boxes'
heights, the noise sphere's Perlin tables, the 1000 spheres), the ground's BvhNode of Cuboids (cuboid.rs's six
sides) and the instanced BvhNode of spheres, likewise.  Parity stays unpinned against the reference BINARY (it
cannot run here); this pins the builders against a reading of the source that shares no code
with either C++ side."""
import importlib.util
import os

import numpy as np
import pytest

import hrt

HERE = os.path.dirname(os.path.abspath(__file__))
_spec = importlib.util.spec_from_file_location("make_kats", os.path.join(HERE, "golden", "make_kats.py"))
K = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(K)
f = np.float32


def v3(x, y, z):
    return (f(x), f(y), f(z))


def vsub(a, b):
    return (a[0] - b[0], a[1] - b[1], a[2] - b[2])


def vadd(a, b):
    return (a[0] + b[0], a[1] + b[1], a[2] + b[2])


def magnitude(a):  # cgmath InnerSpace::magnitude: sqrt(dot), dot = (x x + y y) + z z
    return np.sqrt((a[0] * a[0] + a[1] * a[1]) + a[2] * a[2])


# ------------------------------------------------------------------------------- application.rs:497-565
def random_scene(rand, n=11):
    """objects of generate_random_scene: (kind, c0, c1, radius, material) with material = (kind, params)."""
    objs = [("sphere", v3(0, -1000, 0), None, f(1000), ("lambertian_checker", v3(0.2, 0.3, 0.1), v3(0.9, 0.9, 0.9)))]
    for a in range(-n, n):
        for b in range(-n, n):
            choose = rand.gen_f32()
            cx = f(a) + f(0.9) * rand.gen_f32()
            cz = f(b) + f(0.9) * rand.gen_f32()
            center = (cx, f(0.2), cz)
            if magnitude(vsub(center, v3(4, 0.2, 0))) > f(0.9):
                if choose < f(0.8):
                    albedo = (rand.gen_f32(), rand.gen_f32(), rand.gen_f32())
                    c2 = vadd(center, (f(0), rand.gen_range(0.0, 0.5), f(0)))
                    objs.append(("moving", center, c2, f(0.2), ("lambertian", albedo)))
                elif choose < f(0.95):
                    albedo = (rand.gen_range(0.5, 1.0), rand.gen_range(0.5, 1.0), rand.gen_range(0.5, 1.0))
                    fuzz = rand.gen_range(0.0, 0.5)
                    objs.append(("sphere", center, None, f(0.2), ("metal", albedo, fuzz)))
                else:
                    objs.append(("sphere", center, None, f(0.2), ("dielectric", f(1.5))))
    objs.append(("sphere", v3(0, 1, 0), None, f(1), ("dielectric", f(1.5))))
    objs.append(("sphere", v3(-4, 1, 0), None, f(1), ("lambertian", v3(0.4, 0.2, 0.1))))
    objs.append(("sphere", v3(4, 1, 0), None, f(1), ("metal", v3(0.7, 0.6, 0.5), f(0))))
    return objs


# ------------------------------------------------------------------------------- bounding boxes
def sphere_box(c, r):  # sphere.rs:57-63
    rv = (r, r, r)
    return vsub(c, rv), vadd(c, rv)


def moving_center(c0, c1, t0, t1, time):  # moving_sphere.rs:53-58
    s = (f(time) - f(t0)) / (f(t1) - f(t0))
    d = vsub(c1, c0)
    return vadd(c0, (s * d[0], s * d[1], s * d[2]))


def surrounding(b0, b1):  # aabb.rs:49-66
    return (tuple(np.minimum(b0[0][k], b1[0][k]) for k in range(3)),
            tuple(np.maximum(b0[1][k], b1[1][k]) for k in range(3)))


def bbox(o, t0=0.0, t1=1.0):
    kind, c0, c1, r, _ = o
    if kind == "sphere":
        return sphere_box(c0, r)
    # moving_sphere.rs:98-110: the boxes at time_start and time_end of the BvhNode::new call, surrounded; the
    # scene's moving spheres run over [0, 1]
    return surrounding(sphere_box(moving_center(c0, c1, 0.0, 1.0, t0), r),
                       sphere_box(moving_center(c0, c1, 0.0, 1.0, t1), r))


# ------------------------------------------------------------------------------- bvh_node.rs:27-63
def bvh_leaves(objs, t0=0.0, t1=1.0, box=None):
    """The leaves of BvhNode::new(objs) in the order BvhNode::hit visits them (left subtree first); box(o, t0, t1)
    is the objects' Hittable::bounding_box (default: spheres and moving spheres)."""
    box = box or bbox
    objs = list(objs)
    ranges = []
    for axis in range(3):
        mn, mx = f(np.finfo(np.float32).max), f(np.finfo(np.float32).min)  # f32::MAX, f32::MIN
        for o in objs:
            b = box(o, t0, t1)
            mn, mx = min(mn, b[0][axis]), max(mx, b[1][axis])
        ranges.append((axis, mx - mn))
    ranges.sort(key=lambda ar: -ar[1])  # descending; 3 elements: Rust's insertion sort keeps ties in order
    axis = ranges[0][0]
    objs.sort(key=lambda o: box(o, t0, t1)[0][axis] + box(o, t0, t1)[1][axis])
    if len(objs) == 1:
        return objs
    half = len(objs) // 2
    right = bvh_leaves(objs[half:], t0, t1, box)
    left = bvh_leaves(objs[:half], t0, t1, box)
    return left + right


# ------------------------------------------------------------------------------- the library's records
def _records(name, seed=1):
    s = hrt.preset(name, seed)
    buf, info = hrt.scene_blob(s)
    b = np.frombuffer(buf.raw, np.uint8)
    prims = b[info.off_prims:info.off_prims + 48 * info.n_prims].view(np.float32).reshape(-1, 12)
    sec = lambda lo, hi, rec: b[lo:lo + (hi - lo) // rec * rec].view(np.float32).reshape(-1, rec // 4)  # noqa: E731
    mats = sec(info.off_mats, info.off_texs, 32)  # sections may end in alignment padding
    texs = sec(info.off_texs, info.off_perlin, 48)
    return prims, mats, texs, info


def _u(x):
    return int(np.float32(x).view(np.uint32))


def _same(a, b):
    return np.float32(a).view(np.uint32) == np.float32(b).view(np.uint32)


def _check_material(mat, mats, texs, mi):
    m = mats[mi]
    kind, tex = _u(m[4]), _u(m[5])
    if mat[0] == "metal":
        assert kind == 1 and all(_same(m[k], mat[1][k]) for k in range(3)) and _same(m[3], mat[2])
    elif mat[0] == "dielectric":
        assert kind == 2 and _same(m[0], mat[1])
    elif mat[0] == "lambertian":
        t = texs[tex]
        assert kind == 0 and _u(t[4]) == 0 and all(_same(t[k], mat[1][k]) for k in range(3))  # SolidColor
    else:  # Lambertian(CheckerTexture(odd, even))
        t = texs[tex]
        assert kind == 0 and _u(t[4]) == 1
        odd, even = texs[_u(t[5])], texs[_u(t[6])]
        assert all(_same(odd[k], mat[1][k]) for k in range(3)) and all(_same(even[k], mat[2][k]) for k in range(3))


@pytest.mark.parametrize("name,n", [("random", 11), ("random_10k", 50)])
def test_random_scene_builder_restated_independently(name, n):
    """application.rs:497-565 (config 4: n = 50) and BvhNode::new restated here, against the library's lowered
    scene: the same objects in the same pre-order, every centre, radius, shutter and material bit for bit."""
    leaves = bvh_leaves(random_scene(K.scene_rng(1), n))
    prims, mats, texs, info = _records(name)
    assert len(leaves) == info.n_prims == len(prims)
    for k, (kind, c0, c1, r, mat) in enumerate(leaves):
        p = prims[k]
        km = _u(p[11])
        assert all(_same(p[j], c0[j]) for j in range(3)) and _same(p[3], r), (k, p[:4], c0, r)
        if kind == "moving":  # layout.h: p1 = (c1 - c0, time_start), p2[0] = time_end - time_start
            d = vsub(c1, c0)
            assert km & 3 == 1 and all(_same(p[4 + j], d[j]) for j in range(3)), (k, p[4:7], d)
            assert _same(p[7], 0.0) and _same(p[8], 1.0)
        else:
            assert km & 3 == 0, k
        _check_material(mat, mats, texs, km >> 4)


def test_restatement_sees_a_misreading():
    """The check has teeth: one draw out of the reference's order (the moving sphere's albedo drawn after its
    second centre) changes the restated scene, and the comparison above would fail on it."""
    good = bvh_leaves(random_scene(K.scene_rng(1)))

    def misread(rand, n=11):
        objs = random_scene(K.scene_rng(1), 0)[:1]
        for a in range(-n, n):
            for b in range(-n, n):
                choose = rand.gen_f32()
                center = (f(a) + f(0.9) * rand.gen_f32(), f(0.2), f(b) + f(0.9) * rand.gen_f32())
                if magnitude(vsub(center, v3(4, 0.2, 0))) > f(0.9):
                    if choose < f(0.8):
                        c2 = vadd(center, (f(0), rand.gen_range(0.0, 0.5), f(0)))
                        albedo = (rand.gen_f32(), rand.gen_f32(), rand.gen_f32())
                        objs.append(("moving", center, c2, f(0.2), ("lambertian", albedo)))
                    elif choose < f(0.95):
                        albedo = (rand.gen_range(0.5, 1.0), rand.gen_range(0.5, 1.0), rand.gen_range(0.5, 1.0))
                        objs.append(("sphere", center, None, f(0.2), ("metal", albedo, rand.gen_range(0.0, 0.5))))
                    else:
                        objs.append(("sphere", center, None, f(0.2), ("dielectric", f(1.5))))
        return objs + random_scene(K.scene_rng(1), 0)[1:]

    bad = bvh_leaves(misread(K.scene_rng(1)))
    assert len(bad) == len(good)
    assert any(x[1] != y[1] or x[4] != y[4] for x, y in zip(good, bad))


# ------------------------------------------------------------------------------- application.rs:817-935 (Final)
def cuboid_rects(p0, p1):
    """cuboid.rs: the six sides as (plane, a0, a1, b0, b1, k), in its order (HRT_PLANE_XY 0, YZ 1, ZX 2)."""
    (x0, y0, z0), (x1, y1, z1) = p0, p1
    return [(0, x0, x1, y0, y1, z1), (0, x0, x1, y0, y1, z0), (2, z0, z1, x0, x1, y1), (2, z0, z1, x0, x1, y0),
            (1, y0, y1, z0, z1, x1), (1, y0, y1, z0, z1, x0)]


def final_draws(rand):
    """The Final scene's draws from the scene stream, in the reference's order: the 20 x 20 ground boxes' heights
    (application.rs:822-836), the noise sphere's Perlin tables (:912, NoiseTexture::new's perlin_noise.rs:28-45 on
    the scene stream: the documented substitution for its own thread_rng), the 1000 spheres' centres (:917-927)."""
    ground = []
    for i in range(20):
        for j in range(20):
            w = f(100)
            x0 = f(-1000) + f(i) * w
            z0 = f(-1000) + f(j) * w
            y1 = rand.gen_range(1.0, 101.0)
            ground.append(((x0, f(0), z0), (x0 + w, y1, z0 + w)))
    ranvec, perms = K.perlin_tables(rand)
    centres = []
    for _ in range(1000):
        x = rand.gen_range(0.0, 165.0)
        y = rand.gen_range(0.0, 165.0)
        z = rand.gen_range(0.0, 165.0)
        centres.append((x, y, z))
    return ground, (ranvec, perms), centres


def test_final_scene_draws_and_structure_restated_independently():
    """Final (application.rs:817-935): the ground boxes (a BvhNode of 400 Cuboids, each lowered to its six sides
    in cuboid.rs's order), the Perlin tables of the noise sphere and the 1000 spheres of the rotated, translated
    BvhNode, restated here from the scene stream, against the library's lowered scene: every rect of the ground
    in its BvhNode pre-order, every instanced sphere in its BvhNode pre-order, and the Perlin tables, bit for bit."""
    earth = np.zeros((2, 2, 3), np.uint8)
    s = hrt.preset("final", 1, earth)
    buf, info = hrt.scene_blob(s)
    b = np.frombuffer(buf.raw, np.uint8)
    prims = b[info.off_prims:info.off_prims + 48 * info.n_prims].view(np.float32).reshape(-1, 12)
    pu = prims.view(np.uint32)
    ground, (ranvec, perms), centres = final_draws(K.scene_rng(1))

    # the ground: BvhNode::new over the cuboids (box = (box_min, box_max), cuboid.rs), six sides per leaf
    leaves = bvh_leaves([("cuboid", p0, p1, None, None) for p0, p1 in ground], box=lambda o, t0, t1: (o[1], o[2]))
    spheres = bvh_leaves([("sphere", c, None, f(10), None) for c in centres])
    want = [r for o in leaves for r in cuboid_rects(o[1], o[2])]
    world = pu[:, 10] == 0xFFFFFFFF
    rect = (pu[:, 11] & 3) == 2
    got = [k for k in range(len(prims)) if world[k] and rect[k]]
    start = next(k for k in range(len(got)) if all(_same(prims[got[k]][j], want[0][1 + j]) for j in range(4)))
    run = got[start:start + len(want)]
    assert len(run) == len(want) == 2400
    for k, (plane, a0, a1, b0, b1, kk) in zip(run, want):
        p = prims[k]
        assert (pu[k, 11] >> 2) & 3 == plane, k
        assert all(_same(p[j], v) for j, v in enumerate((a0, a1, b0, b1))) and _same(p[4], kk), (k, p[:5])
        assert _same(p[5], a1 - a0) and _same(p[6], b1 - b0)
    # the 1000 spheres inside Translation(Rotation(BvhNode)): their own frame's centres, in the BvhNode's pre-order
    inst = [k for k in range(len(prims)) if not world[k]]
    assert len(inst) == 1000
    for k, o in zip(inst, spheres):
        assert all(_same(prims[k][j], o[1][j]) for j in range(3)) and _same(prims[k][3], 10.0), (k, prims[k][:4])
    # the noise texture's Perlin tables (layout.h Perlin: ranvec[256][4] f32, then perm[3][512] u32: each
    # permutation twice over)
    pt = b[info.off_perlin:info.off_perlin + 4096 + 3 * 512 * 4]
    rv = pt[:4096].view(np.float32).reshape(256, 4)
    pm = pt[4096:].view(np.uint32).reshape(3, 512)
    assert all(_same(rv[i][j], ranvec[i][j]) for i in range(256) for j in range(3))
    assert [list(map(int, pm[c, :256])) for c in range(3)] == perms
    assert [list(map(int, pm[c, 256:])) for c in range(3)] == perms


# ------------------------------------------------------------------------------- application.rs:639-721 (Cornell)
def rect_box(r):  # rect.rs:88-102 (the ZX box transposed relative to its hit test: G17, kept)
    plane, a0, a1, b0, b1, k = r
    e = f(0.0001)
    if plane == 0:
        return (a0, b0, k - e), (a1, b1, k + e)
    if plane == 1:
        return (k - e, a0, b0), (k + e, a1, b1)
    return (a0, k - e, b0), (a1, k + e, b1)


def rotated_box(box, axis, angle):  # rotation.rs:38-90: the eight corners turned, f32 sin / cos of the angle
    import math

    r_axis, a_axis, b_axis = {0: (0, 1, 2), 1: (1, 2, 0), 2: (2, 0, 1)}[axis]
    radians = (f(math.pi) / f(180.0)) * f(angle)  # (PI / 180.0) * angle, std::f32::consts::PI
    sin_t, cos_t = f(math.sin(float(radians))), f(math.cos(float(radians)))
    mn = [f(np.finfo(np.float32).max)] * 3
    mx = [f(-np.finfo(np.float32).max)] * 3
    for i in range(2):
        for j in range(2):
            for k in range(2):
                r = f(k) * box[1][r_axis] + f(1 - k) * box[0][r_axis]
                a = f(i) * box[1][a_axis] + f(1 - i) * box[0][a_axis]
                b = f(j) * box[1][b_axis] + f(1 - j) * box[0][b_axis]
                na = cos_t * a - sin_t * b
                nb = sin_t * a + cos_t * b
                mn[a_axis], mn[b_axis], mn[r_axis] = min(mn[a_axis], na), min(mn[b_axis], nb), min(mn[r_axis], r)
                mx[a_axis], mx[b_axis], mx[r_axis] = max(mx[a_axis], na), max(mx[b_axis], nb), max(mx[r_axis], r)
    return tuple(mn), tuple(mx)


def test_cornell_scene_structure_restated_independently():
    """Cornell (application.rs:639-721): five walls and the light as Rects, two Cuboids each in a Rotation (Y, 15
    and -18 degrees) inside a Translation, all under one BvhNode (its sort keys from rect.rs's boxes, the rotated
    corners of rotation.rs and translation.rs's offset): the library's primitives in that pre-order, the walls at
    world level with their materials, each cuboid's six sides in its own frame, bit for bit."""
    prims, mats, texs, info = _records("cornell")
    pu = prims.view(np.uint32)
    red, white, green = v3(0.65, 0.05, 0.05), v3(0.73, 0.73, 0.73), v3(0.12, 0.45, 0.15)
    F = lambda *x: tuple(f(v) for v in x)  # noqa: E731
    objs = [("rect", F(1, 0, 555, 0, 555, 555), green), ("rect", F(1, 0, 555, 0, 555, 0), red),
            ("rect", F(2, 213, 343, 227, 332, 554), "light"), ("rect", F(2, 0, 555, 0, 555, 0), white),
            ("rect", F(2, 0, 555, 0, 555, 555), white), ("rect", F(0, 0, 555, 0, 555, 555), white)]
    for size, angle, off in ((v3(165, 330, 165), 15.0, v3(265, 0, 295)), (v3(165, 165, 165), -18.0, v3(130, 0, 65))):
        cb = (v3(0, 0, 0), size)
        rb = rotated_box(cb, 1, angle)
        objs.append(("box", cb, (vadd(rb[0], off), vadd(rb[1], off))))

    def box(o, t0, t1):
        return rect_box(o[1]) if o[0] == "rect" else o[2]
    leaves = bvh_leaves(objs, box=box)
    want = []
    for o in leaves:
        if o[0] == "rect":
            want.append((o[1], o[2], True))
        else:
            want += [(tuple(f(v) for v in r), white, False) for r in cuboid_rects(*o[1])]
    assert len(want) == len(prims) == 18
    for k, (r, mat, world) in enumerate(want):
        p = prims[k]
        assert (pu[k, 11] & 3) == 2 and ((pu[k, 11] >> 2) & 3) == int(r[0]), k
        assert all(_same(p[j], r[1 + j]) for j in range(4)) and _same(p[4], r[5]), (k, p[:5], r)
        assert (pu[k, 10] == 0xFFFFFFFF) == world, k
        m = mats[pu[k, 11] >> 4]
        t = texs[_u(m[5])]
        if mat == "light":
            assert _u(m[4]) == 3 and all(_same(t[j], 15.0) for j in range(3))
        else:
            assert _u(m[4]) == 0 and all(_same(t[j], mat[j]) for j in range(3)), k


@pytest.mark.parametrize("name", ["two_perlin_spheres", "earth_perlin", "simple_light"])
def test_noise_scenes_restated_independently(name):
    """The Perlin scenes (application.rs:589-602, :614-637, and config 3's Earth over that ground): the noise
    texture's tables drawn first from the scene stream (perlin_noise.rs:28-45, the thread_rng substitution), the
    ground sphere and the small sphere under one BvhNode (the ground first on the y axis), with NoiseTexture's
    scale 4: the library's records bit for bit."""
    prims, mats, texs, info = _records(name)
    pu = prims.view(np.uint32)
    ranvec, perms = K.perlin_tables(K.scene_rng(1))
    b = np.frombuffer(hrt.scene_blob(hrt.preset(name, 1))[0].raw, np.uint8)
    pt = b[info.off_perlin:info.off_perlin + 4096 + 3 * 512 * 4]
    rv = pt[:4096].view(np.float32).reshape(256, 4)
    pm = pt[4096:].view(np.uint32).reshape(3, 512)  # each permutation twice over (layout.h Perlin)
    assert all(_same(rv[i][j], ranvec[i][j]) for i in range(256) for j in range(3))
    assert [list(map(int, pm[c, :256])) for c in range(3)] == perms
    assert [list(map(int, pm[c, 256:])) for c in range(3)] == perms
    objs = [("sphere", v3(0, -1000, 0), None, f(1000), "noise"),
            ("sphere", v3(0, 2, 0), None, f(2), "image" if name == "earth_perlin" else "noise")]
    spheres = [p for p in range(len(prims)) if (pu[p, 11] & 3) == 0]
    for k, o in zip(spheres, bvh_leaves(objs)):
        assert all(_same(prims[k][j], o[1][j]) for j in range(3)) and _same(prims[k][3], o[3])
        t = texs[_u(mats[pu[k, 11] >> 4][5])]
        if o[4] == "noise":
            assert _u(t[4]) == 2 and _same(t[0], 4.0)
        else:
            assert _u(t[4]) == 3
    assert len(spheres) == 2
