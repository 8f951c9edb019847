"""Test scenes built through the C ABI's constructors (hrt_tex_* / hrt_mat_* / hrt_node_*), for kernel-choice
and stream-layout cases the reference presets do not reach.  Test infrastructure: they have no oracle preset,
so the tests hold the default path to the verbatim reference traversal (HRT_RENDER_REFERENCE_CULL, the
segment kernel walking the reference node stream, itself held to the oracle on every preset) bit for bit.

- sphere_lists: a sphere-only scene whose BvhNodes hold Lists (application.rs never builds one, but
  BvhNode::new takes any Hittable, bvh_node.rs:27-63, and List::hit tests its members with no box of their
  own, list.rs:20-31), including a List whose members come before and after a nested BvhNode that holds a
  List of its own (the group-box state's contiguity, scene.cpp gwalk_leaves_grouped).
- big_textured: a sphere scene whose walk stream exceeds the LDS budget (layout.h LDS_SCENE_MAX_BYTES)
  with noise- and image-textured spheres: the sphere kernel's HEAVY walk over an LDS + global stream.
"""
import numpy as np

import hrt

PEND = 1 << 31
GL_BOX = 1
GL_ONE = 32
GL_MED = 64


def perlin_tables(seed):
    """Any valid NoiseTexture tables (perlin_noise.rs:14-19): 256 unit vectors, three permutations."""
    rng = np.random.default_rng(seed)
    v = rng.uniform(-1, 1, (256, 3))
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    perm = np.stack([rng.permutation(256) for _ in range(3)]).astype(np.uint32)
    return v.astype(np.float32), perm


def _mat(s, rng, kind):
    if kind == 0:
        return s.lambertian(s.solid(*rng.uniform(0, 1, 3)))
    if kind == 1:
        return s.metal(rng.uniform(0.5, 1, 3), float(rng.uniform(0, 0.5)))
    return s.dielectric(1.5)


def sphere_lists(seed=5):
    """Random-scene-like spheres grouped into Lists inside a BvhNode (application.rs:497-565 materials)."""
    rng = np.random.default_rng(seed)
    s = hrt.Scene()
    checker = s.checker(s.solid(0.2, 0.3, 0.1), s.solid(0.9, 0.9, 0.9))
    objs = [s.sphere((0, -1000, 0), 1000, s.lambertian(checker))]
    cells = [(a, b) for a in range(-6, 6) for b in range(-6, 6)]
    spheres = []
    for a, b in cells:
        c = (a + 0.9 * rng.uniform(), 0.2, b + 0.9 * rng.uniform())
        spheres.append(s.sphere(c, 0.2, _mat(s, rng, int(rng.integers(0, 3)))))
    k = 0
    while k < len(spheres):  # Lists of 1-4 members, every fifth one a nested list around a BvhNode of lists
        n = int(rng.integers(2, 5)) if len(objs) % 5 == 4 else int(rng.integers(1, 5))
        group = spheres[k:k + n]
        k += n
        if len(objs) % 5 == 4 and k + 4 <= len(spheres):
            # a BvhNode whose Leaf holds a List with a box-less member and a BvhNode (a box): a group of
            # box-less leaves of its own, between members of the outer List before and after it
            inner = s.bvh([s.list([spheres[k], s.bvh(spheres[k + 1:k + 3])]), spheres[k + 3]])
            k += 4
            group = group[:1] + [inner] + group[1:]
        elif len(objs) % 5 == 2 and k + 2 <= len(spheres):
            group = group + [s.bvh(spheres[k:k + 2])]  # box-less members and a BvhNode: one group box
            k += 2
        objs.append(s.list(group) if len(group) > 1 or rng.uniform() < 0.5 else group[0])
    objs.append(s.list([s.sphere((0, 1, 0), 1.0, s.dielectric(1.5)), s.sphere((-4, 1, 0), 1.0, s.lambertian(s.solid(0.4, 0.2, 0.1)))]))
    objs.append(s.sphere((4, 1, 0), 1.0, s.metal((0.7, 0.6, 0.5), 0.0)))
    root = s.bvh(objs, 0.0, 1.0)
    s.set_root(root)
    return s


def big_textured(seed=7, grid=26):
    """grid^2 small spheres (over the LDS budget from grid ~ 18) on a Perlin-noise ground, an image-textured
    earth and a noise-textured sphere among them (application.rs:589-612 textures)."""
    rng = np.random.default_rng(seed)
    s = hrt.Scene()
    rv, perm = perlin_tables(seed)
    noise = s.noise(4.0, rv, perm)
    objs = [s.sphere((0, -1000, 0), 1000, s.lambertian(noise))]
    earth = s.lambertian(s.image(hrt.synthetic_earth(64, 32)))
    objs.append(s.sphere((0, 1.2, 0), 1.2, earth))
    objs.append(s.sphere((-3, 1, 1), 1.0, s.lambertian(s.noise(2.0, rv, perm))))
    half = grid // 2
    for a in range(-half, grid - half):
        for b in range(-half, grid - half):
            c = (a * 0.6 + 0.5 * rng.uniform(), 0.15, b * 0.6 + 0.5 * rng.uniform())
            kind = int(rng.integers(0, 4))
            mat = earth if kind == 3 else _mat(s, rng, kind)
            objs.append(s.sphere(c, 0.15, mat))
    s.set_root(s.bvh(objs, 0.0, 1.0))
    return s


def foggy(seed=3):
    """Constant media of every shape the general walk stream distinguishes (constant_medium.rs:34-76), among
    spheres, rects and a light: a world-level medium over one sphere and one over a MOVING sphere (flat GL_MED
    programs), a medium that is a box-less List member (its program is the medium node alone), a medium over a
    Cuboid (two boundary walks) and a fog sphere around the whole scene, as in application.rs:884-895."""
    rng = np.random.default_rng(seed)
    s = hrt.Scene()
    white = s.solid(0.73, 0.73, 0.73)
    objs = [s.sphere((0, -1000, 0), 1000, s.lambertian(s.checker(s.solid(0.2, 0.3, 0.1), white)))]
    objs.append(s.rect(hrt.PLANE_ZX, -2, 2, -2, 2, 6.0, s.diffuse_light(s.solid(7, 7, 7))))
    objs.append(s.constant_medium(s.sphere((0, 1, 0), 1.0, s.dielectric(1.5)), 0.8, s.solid(0.2, 0.4, 0.9)))
    objs.append(s.constant_medium(s.moving_sphere((3, 0.8, -1), (3, 1.1, -1), 0.0, 1.0, 0.8, s.dielectric(1.5)),
                                  1.2, s.solid(0.9, 0.3, 0.2)))
    objs.append(s.constant_medium(s.cuboid((-4, 0, -1), (-2.5, 1.5, 0.5), white), 0.5, s.solid(0.1, 0.1, 0.1)))
    member = s.constant_medium(s.sphere((-1.5, 0.5, 2.5), 0.5, s.dielectric(1.5)), 2.0, s.solid(0.8, 0.8, 0.2))
    objs.append(s.list([member, s.sphere((1.5, 0.4, 2.5), 0.4, s.metal((0.7, 0.6, 0.5), 0.1))]))
    for _ in range(12):
        c = (float(rng.uniform(-5, 5)), 0.25, float(rng.uniform(-5, 5)))
        objs.append(s.sphere(c, 0.25, _mat(s, rng, int(rng.integers(0, 3)))))
    objs.append(s.constant_medium(s.sphere((0, 0, 0), 50.0, s.dielectric(1.5)), 0.002, s.solid(1, 1, 1)))
    s.set_root(s.bvh(objs, 0.0, 1.0))
    return s


def camera(w, h):
    return hrt.camera((13, 2, 3), (0, 0, 0), 20.0, 0.1, 10.0, 0.0, 1.0, w, h)


def general_stream_leaves(blob, info):
    """The general walk stream's leaves in walk (pre-)order: (begin, end, flags, group) per leaf (a GL_ONE leaf
    keeps its node's kind word in place of end, a GL_MED leaf its medium: layout.h)."""
    raw = np.frombuffer(bytes(blob), np.uint8)
    base = int(info.off_walk)
    end = int(info.walk_bytes)
    u32 = lambda off: raw[base + off:base + off + 16].view(np.uint32)  # noqa: E731
    out, o = [], 0
    while o < end:
        c, e = u32(o), u32(o + 16)
        skip, link = int(c[3]), int(e[3])
        if link & PEND:
            p = link & ~PEND
            h, bmx = u32(p), u32(p + 32)
            fl = int(h[2])
            last = int(h[0]) + 1 if fl & GL_ONE else int(h[0]) + 2 if fl & GL_MED else int(h[1])
            out.append((int(h[0]), last, fl, int(bmx[3])))
            o = skip
        else:
            o = link
    return out
