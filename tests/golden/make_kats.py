"""Generate tests/golden/kats.json: known-answer vectors for the oracle's unit functions.

This is a SECOND, independent restatement of the reference formulas (numpy float32 scalars, one IEEE
rounding per operation, Python's libm for the transcendentals) written from the Rust sources:
  aabb.rs:20-47, sphere.rs:31-75, moving_sphere.rs:53-96, rect.rs:53-86, math.rs:12-62,
  camera.rs:67-95, perlin_noise.rs:28-123, checker_texture.rs:21-30, noise_texture.rs:24-31,
  image_texture.rs:36-62, hit_record.rs:22-29,
plus the seeded RNG that replaces thread_rng (include/hrt/hd_math.h) and rand 0.8.5's distribution
transforms.  tests/test_oracle_kats.py checks liboracle.so against these vectors bit for bit.
The reference itself cannot run here (Rust toolchain absent, window required, unseeded), so these
vectors -- not reference outputs -- are what pins the oracle.

Run:  python tests/golden/make_kats.py   (deterministic; rewrites kats.json)
"""
import json
import math
import os
import struct

import numpy as np

np.seterr(all="ignore")
f = np.float32
M32, M64 = (1 << 32) - 1, (1 << 64) - 1
PI = f(math.pi)


def bits(x):
    return int(np.float32(x).view(np.uint32))


def fbits(u):
    return np.uint32(u).view(np.float32)


def cr(fn, *xs):
    """libm in f64, rounded once to f32 (the 'correctly rounded' answer hd_math targets)."""
    try:
        return f(fn(*[float(x) for x in xs]))
    except ValueError:
        return f(np.nan)


# ----------------------------------------------------------------------------- vectors (cgmath order)
def add(a, b): return (a[0] + b[0], a[1] + b[1], a[2] + b[2])
def sub(a, b): return (a[0] - b[0], a[1] - b[1], a[2] - b[2])
def neg(a): return (-a[0], -a[1], -a[2])
def smul(s, a): return (s * a[0], s * a[1], s * a[2])
def sdiv(a, s): return (a[0] / s, a[1] / s, a[2] / s)
def dot(a, b): return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]
def cross(a, b): return (a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0])
def norm(a): return smul(f(1) / np.sqrt(dot(a, a)), a)
def F3(v): return tuple(f(x) for x in v)


# ----------------------------------------------------------------------------- math.rs
def reflect(v, n): return sub(v, smul(f(2) * dot(v, n), n))


def refract(uv, n, eta):
    c = np.fmin(dot(neg(uv), n), f(1))
    perp = smul(eta, add(uv, smul(c, n)))
    par = smul(-np.sqrt(np.abs(f(1) - dot(perp, perp))), n)
    return add(perp, par)


def reflectance(cosine, ri):
    r0 = (f(1) - ri) / (f(1) + ri)
    r0 = r0 * r0
    x = float(f(1) - cosine)
    return r0 + (f(1) - r0) * f(x ** 5)


def near_zero(v): return all(abs(c) < f(1e-8) for c in v)


# ----------------------------------------------------------------------------- RNG (hd_math.h)
def mix64(z):
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def rotl(x, k): return ((x << k) | (x >> (32 - k))) & M32


class Rng:
    def __init__(self, key):
        s = (key + 0x9E3779B97F4A7C15) & M64
        a = mix64(s)
        s = (s + 0x9E3779B97F4A7C15) & M64
        b = mix64(s)
        self.s = [a & M32, a >> 32, b & M32, b >> 32]
        if not any(self.s):
            self.s[0] = 1

    def u32(self):
        s0, s1, s2, s3 = self.s
        r = (rotl((s1 * 5) & M32, 7) * 9) & M32
        t = (s1 << 9) & M32
        s2 ^= s0
        s3 ^= s1
        s1 ^= s2
        s0 ^= s3
        s2 ^= t
        s3 = rotl(s3, 11)
        self.s = [s0, s1, s2, s3]
        return r

    def u64(self):
        lo = self.u32()
        hi = self.u32()
        return (hi << 32) | lo

    def gen_f32(self): return f(self.u32() >> 8) * f(2.0 ** -24)

    def gen_range(self, lo, hi):
        lo, hi = f(lo), f(hi)
        scale = hi - lo
        while True:
            v = fbits(0x3F800000 | (self.u32() >> 9)) - f(1)
            res = v * scale + lo
            if res < hi:
                return res
            scale = fbits(int(scale.view(np.uint32)) - 1)

    def gen_range_u64(self, lo, hi):
        rng = hi - lo
        zone = ((rng << (64 - rng.bit_length())) & M64) - 1
        while True:
            m = self.u64() * rng
            if (m & M64) <= zone:
                return lo + (m >> 64)


def path_key(seed, pixel, sample): return mix64(mix64(seed) ^ ((pixel << 32) | sample))
def scene_rng(seed): return Rng(mix64(seed ^ 0x5343454E45))


# ----------------------------------------------------------------------------- aabb.rs / hittables
def aabb_hit(mn, mx, o, d, tmin, tmax):
    for a in range(3):
        inv = f(1) / d[a]
        ts = (mn[a] - o[a]) * inv
        te = (mx[a] - o[a]) * inv
        if inv < f(0):
            ts, te = te, ts
        lo = ts if ts > tmin else tmin
        hi = te if te < tmax else tmax
        if hi <= lo:
            return 0
    return 1


def at(o, d, t): return add(o, smul(t, d))


def sphere_uv(p):
    theta = cr(math.acos, -p[1]) if abs(float(p[1])) <= 1 else f(np.nan)
    phi = cr(math.atan2, -p[2], p[0]) + PI
    return phi / (f(2) * PI), theta / PI


def face(d, outward):
    front = dot(d, outward) < f(0)
    return front, (outward if front else neg(outward))


def sphere_hit(center, radius, o, d, tmin, tmax):
    oc = sub(o, center)
    a = dot(d, d)
    half_b = dot(oc, d)
    c = dot(oc, oc) - radius * radius
    disc = half_b * half_b - a * c
    if disc < f(0):
        return None
    sq = np.sqrt(disc)
    root = (-half_b - sq) / a
    if root < tmin or tmax < root:
        root = (-half_b + sq) / a
        if root < tmin or tmax < root:
            return None
    outward = sdiv(sub(at(o, d, root), center), radius)
    u, v = sphere_uv(outward)
    front, n = face(d, outward)
    return [root, *at(o, d, root), *n, u, v, f(1) if front else f(0)]


def moving_center(c0, c1, t0, t1, time): return add(c0, smul((time - t0) / (t1 - t0), sub(c1, c0)))


def rect_hit(plane, a0, a1, b0, b1, k, o, d, tmin, tmax):
    ka, aa, ba = {0: (2, 0, 1), 1: (0, 1, 2), 2: (1, 2, 0)}[plane]
    t = (k - o[ka]) / d[ka]
    if t < tmin or t > tmax:
        return None
    av = o[aa] + t * d[aa]
    bv = o[ba] + t * d[ba]
    if av < a0 or av > a1 or bv < b0 or bv > b1:
        return None
    outward = [f(0), f(0), f(0)]
    outward[ka] = f(1)
    front, n = face(d, tuple(outward))
    return [t, *at(o, d, t), *n, (av - a0) / (a1 - a0), (bv - b0) / (b1 - b0), f(1) if front else f(0)]


# ----------------------------------------------------------------------------- camera.rs
def camera(frm, at_, fov, aperture, focus, W, H):
    aspect = f(W) / f(H)
    theta = fov * (PI / f(180))
    h = cr(math.tan, theta / f(2))
    vh = f(2) * h
    vw = aspect * vh
    w = norm(sub(frm, at_))
    u = norm(cross(F3((0, 1, 0)), w))
    v = cross(w, u)
    hor = smul(focus * vw, u)
    ver = smul(focus * vh, v)
    llc = sub(sub(sub(frm, sdiv(hor, f(2))), sdiv(ver, f(2))), smul(focus, w))
    return dict(origin=frm, llc=llc, hor=hor, ver=ver, u=u, v=v, w=w, lens=aperture / f(2))


def camera_ray(c, s, t, disk, time):
    rd = smul(c["lens"], disk)
    off = add(smul(rd[0], c["u"]), smul(rd[1], c["v"]))
    direction = sub(sub(add(add(c["llc"], smul(s, c["hor"])), smul(t, c["ver"])), c["origin"]), off)
    return [*add(c["origin"], off), *direction, time]


# ----------------------------------------------------------------------------- perlin / textures
def perlin_tables(rng):
    ranvec = []
    for _ in range(256):
        x = rng.gen_range(-1, 1)
        y = rng.gen_range(-1, 1)
        z = rng.gen_range(-1, 1)
        ranvec.append(norm((x, y, z)))
    perms = []
    for _ in range(3):
        p = list(range(256))
        for i in range(255, 0, -1):
            tgt = rng.gen_range_u64(0, i)
            p[i], p[tgt] = p[tgt], p[i]
        perms.append(p)
    return ranvec, perms


def sat_i32(x):
    if np.isnan(x):
        return 0
    return int(max(-2 ** 31, min(2 ** 31 - 1, math.trunc(float(x)))))


def noise(ranvec, perms, p):
    i, j, k = (sat_i32(np.floor(c)) for c in p)
    c = {}
    for idx in range(8):
        ix, iy, iz = idx // 4, (idx // 2) % 2, idx % 2
        c[(ix, iy, iz)] = ranvec[perms[0][(i + ix) & 255] ^ perms[1][(j + iy) & 255] ^ perms[2][(k + iz) & 255]]
    u, v, w = (q - np.floor(q) for q in p)
    u = u * u * (f(3) - f(2) * u)
    v = v * v * (f(3) - f(2) * v)
    w = w * w * (f(3) - f(2) * w)
    acc = f(0)
    for idx in range(8):
        x, y, z = idx // 4, (idx // 2) % 2, idx % 2
        wt = (u - f(x), v - f(y), w - f(z))
        acc += ((f(x) * u + f(1 - x) * (f(1) - u)) * (f(y) * v + f(1 - y) * (f(1) - v)) *
                (f(z) * w + f(1 - z) * (f(1) - w)) * dot(c[(x, y, z)], wt))
    return acc


def turbulence(ranvec, perms, p, depth=7):
    acc, weight = f(0), f(1)
    for _ in range(depth):
        acc += weight * noise(ranvec, perms, p)
        weight *= f(0.5)
        p = smul(f(2), p)
    return abs(acc)


def checker(p):
    s = cr(math.sin, f(10) * p[0]) * cr(math.sin, f(10) * p[1]) * cr(math.sin, f(10) * p[2])
    return F3((0.2, 0.3, 0.1)) if s < f(0) else F3((0.9, 0.9, 0.9))


def noise_tex(ranvec, perms, scale, p):
    s = f(1) + cr(math.sin, (scale * p[2]) + (f(10) * turbulence(ranvec, perms, smul(scale, p))))
    return smul(s, (f(0.5), f(0.5), f(0.5)))


def image_tex(img, u, v):
    h, w, c = img.shape
    u = f(0) if u < f(0) else (f(1) if u > f(1) else u)
    vc = f(0) if v < f(0) else (f(1) if v > f(1) else v)
    v = f(1) - vc

    def sat_u32(x):
        if np.isnan(x) or x <= 0:
            return 0
        return int(min(2 ** 32 - 1, math.trunc(float(x))))
    i = min(sat_u32(u * f(w)), w - 1)
    j = min(sat_u32(v * f(h)), h - 1)
    s = f(1) / f(255)
    return tuple(s * f(int(img[j, i, ch])) for ch in range(3))


def kat_image():
    y, x = np.mgrid[0:16, 0:32]
    return np.stack([(x * 8) % 256, (y * 16) % 256, (x * y) % 256], -1).astype(np.uint8)


# ----------------------------------------------------------------------------- cases
def main():
    rs = np.random.default_rng(20240611)
    U = lambda lo, hi: f(rs.uniform(lo, hi))  # noqa: E731
    out = {}

    # RNG streams
    rng_cases = []
    for seed, px, smp in [(1, 0, 0), (7, 12345, 499), (0xDEADBEEF, 2073599, 0)]:
        r = Rng(path_key(seed, px, smp))
        u = [r.u32() for _ in range(32)]
        r = Rng(path_key(seed, px, smp))
        g = [bits(r.gen_f32()) for _ in range(32)]
        r = Rng(path_key(seed, px, smp))
        gr = [bits(r.gen_range(-1, 1)) for _ in range(32)]
        rng_cases.append(dict(seed=seed, pixel=px, sample=smp, u32=u, gen_f32=g, gen_range=gr))
    out["rng"] = rng_cases

    # aabb (reference per-axis semantics)
    aabb = []
    inf = f(np.inf)
    for k in range(300):
        mn = F3(rs.uniform(-2, 1, 3))
        mx = add(mn, F3(rs.uniform(0.01, 2, 3)))
        o = F3(rs.uniform(-4, 4, 3))
        d = F3(rs.normal(0, 1, 3))
        if k % 10 == 0:
            d = (f(0.0), d[1], d[2])
        if k % 10 == 1:
            d = (f(-0.0), f(0.0), d[2])
        if k % 10 == 2:
            o = (mn[0], o[1], o[2])
            d = (f(0.0), d[1], d[2])  # 0 * inf = NaN slab
        tmin = f(0.001)
        tmax = inf if k % 3 else U(0.1, 5)
        if k % 37 == 5:
            tmax = f(np.nan)
        aabb.append(dict(mn=[bits(x) for x in mn], mx=[bits(x) for x in mx], o=[bits(x) for x in o],
                         d=[bits(x) for x in d], tmin=bits(tmin), tmax=bits(tmax), hit=aabb_hit(mn, mx, o, d, tmin, tmax)))
    out["aabb"] = aabb

    # primitives
    prims = []
    for k in range(240):
        kind = k % 3
        o = F3(rs.uniform(-5, 5, 3))
        time = U(0, 1)
        tmin = f(0.001) if k % 5 else f(-np.inf)
        tmax = f(np.inf) if k % 4 else U(0.5, 8)
        if kind == 0:
            c, r = F3(rs.uniform(-1, 1, 3)), U(0.2, 2)
            if k % 7 == 0:
                o = add(c, F3((0.1, 0.05, -0.1)))  # inside: far root
            target = add(c, F3(rs.normal(0, float(r), 3)))
            d = sub(target, o)
            p = [*c, r]
            res = sphere_hit(c, r, o, d, tmin, tmax)
        elif kind == 1:
            c0, c1 = F3(rs.uniform(-1, 1, 3)), F3(rs.uniform(-1, 1, 3))
            t0, t1 = (f(0), f(1)) if k % 2 else (U(0, 0.4), U(0.6, 1))
            r = U(0.2, 1.5)
            target = add(moving_center(c0, c1, t0, t1, time), F3(rs.normal(0, float(r), 3)))
            d = sub(target, o)
            p = [*c0, *c1, t0, t1, r]
            res = sphere_hit(moving_center(c0, c1, t0, t1, time), r, o, d, tmin, tmax)
        else:
            plane = int(rs.integers(0, 3))
            a0, b0 = U(-2, 0), U(-2, 0)
            a1, b1 = a0 + U(0.5, 3), b0 + U(0.5, 3)
            kk = U(-1, 1)
            target = F3(rs.uniform(-2.5, 2.5, 3))
            d = sub(target, o)
            p = [f(plane), a0, a1, b0, b1, kk]
            res = rect_hit(plane, a0, a1, b0, b1, kk, o, d, tmin, tmax)
        prims.append(dict(kind=kind, p=[bits(x) for x in p], ray=[bits(x) for x in (*o, *d, time)],
                          tmin=bits(tmin), tmax=bits(tmax), hit=res is not None,
                          rec=[bits(x) for x in res] if res is not None else []))
    out["prims"] = prims

    # math.rs vector helpers
    vec = []
    for k in range(100):
        v = F3(rs.normal(0, 1, 3))
        n = norm(F3(rs.normal(0, 1, 3)))
        uv = norm(v)
        eta = U(0.5, 1.6)
        cos_ = U(0, 1)
        ri = U(1.1, 2.5)
        vec.append(dict(v=[bits(x) for x in v], n=[bits(x) for x in n], eta=bits(eta), cos=bits(cos_), ri=bits(ri),
                        reflect=[bits(x) for x in reflect(v, n)], refract=[bits(x) for x in refract(uv, n, eta)],
                        reflectance=bits(reflectance(cos_, ri)), normalize=[bits(x) for x in uv],
                        near_zero=int(near_zero(smul(f(1e-9 if k % 4 == 0 else 1), v)))))
    out["vec"] = vec

    # cameras (application.rs:132-211 presets) and rays
    cams = []
    for frm, at_, fov, ap, W, H in [((13, 2, 3), (0, 0, 0), 20, 0.1, 1920, 1080), ((13, 2, 3), (0, 0, 0), 20, 0.0, 400, 225),
                                    ((26, 3, 6), (0, 2, 0), 20, 0.0, 640, 360), ((278, 278, -800), (278, 278, 0), 40, 0.0, 2048, 2048),
                                    ((478, 278, -600), (278, 278, 0), 40, 0.0, 800, 800)]:
        c = camera(F3(frm), F3(at_), f(fov), f(ap), f(10), W, H)
        rays = []
        for _ in range(20):
            s, t = U(0, 1), U(0, 1)
            disk = (U(-0.7, 0.7), U(-0.7, 0.7), f(0))
            time = U(0, 1)
            rays.append(dict(s=bits(s), t=bits(t), disk=[bits(x) for x in disk], time=bits(time),
                             ray=[bits(x) for x in camera_ray(c, s, t, disk, time)]))
        fields = [*c["origin"], *c["llc"], *c["hor"], *c["ver"], *c["u"], *c["v"], *c["w"], c["lens"]]
        cams.append(dict(frm=list(frm), at=list(at_), fov=fov, aperture=ap, W=W, H=H, fields=[bits(x) for x in fields], rays=rays))
    out["camera"] = cams

    # perlin tables from the scene stream + noise/turbulence/textures
    ranvec, perms = perlin_tables(scene_rng(1))
    out["perlin_tables_seed1"] = dict(ranvec=[bits(x) for v in ranvec for x in v], perm=[x for p in perms for x in p])
    pn = []
    for k in range(60):
        p = F3(rs.uniform(-20, 20, 3)) if k % 2 else F3(rs.uniform(-300, 300, 3))
        pn.append(dict(p=[bits(x) for x in p], noise=bits(noise(ranvec, perms, p)), turb=bits(turbulence(ranvec, perms, p)),
                       tex4=[bits(x) for x in noise_tex(ranvec, perms, f(4), p)], tex01=[bits(x) for x in noise_tex(ranvec, perms, f(0.1), p)]))
    out["perlin"] = pn
    ch = []
    for k in range(120):
        p = F3(rs.uniform(-50, 50, 3)) if k % 2 else F3(rs.uniform(-1000, 1000, 3))
        ch.append(dict(p=[bits(x) for x in p], value=[bits(x) for x in checker(p)]))
    out["checker"] = ch
    img = kat_image()
    it = []
    for k in range(100):
        u, v = U(-0.2, 1.2), U(-0.2, 1.2)
        if k == 0:
            u = f(np.nan)
        it.append(dict(u=bits(u), v=bits(v), value=[bits(x) for x in image_tex(img, u, v)]))
    out["image"] = dict(shape=list(img.shape), data=img.reshape(-1).tolist(), cases=it)

    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kats.json")
    with open(path, "w") as fh:
        json.dump(out, fh, separators=(",", ":"))
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
