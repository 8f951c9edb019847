"""Pin the CPU oracle (oracle/oracle.cpp) to the independent numpy-float32 restatement of the
reference formulas (tests/golden/make_kats.py -> kats.json), bit for bit, and pin the shared
deterministic transcendentals (include/hrt/hd_math.h) to correctly rounded libm values."""
import ctypes
import json
import math
import os

import numpy as np
import pytest

from oracle import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "kats.json")) as fh:
    K = json.load(fh)


def fa(bits_list):
    return np.array(bits_list, dtype=np.uint32).view(np.float32)


def same(a, b):
    a = np.asarray(a, np.float32).view(np.uint32)
    b = np.asarray(b, np.float32).view(np.uint32)
    # NaN payloads may differ; compare NaN-ness instead
    an = np.isnan(a.view(np.float32))
    bn = np.isnan(b.view(np.float32))
    return bool(np.array_equal(an, bn) and np.array_equal(a[~an], b[~bn]))


def P(a):
    return a.ctypes.data


def test_rng_streams():
    L = O.load()
    for c in K["rng"]:
        for mode, key in ((2, "u32"), (0, "gen_f32"), (1, "gen_range")):
            out = np.zeros(32, np.float32)
            L.oracle_rng(c["seed"], c["pixel"], c["sample"], mode, 32, P(out))
            want = np.array(c[key], np.uint32) if key == "u32" else np.array(c[key], np.uint32)
            assert np.array_equal(out.view(np.uint32), want), (key, c["seed"])


def test_aabb_reference_semantics():
    L = O.load()
    for c in K["aabb"]:
        args = [fa(c[k]) for k in ("mn", "mx", "o", "d")]
        got = L.oracle_aabb_hit(*[P(a) for a in args], float(fa([c["tmin"]])[0]), float(fa([c["tmax"]])[0]))
        assert got == c["hit"], c


def test_primitive_hits():
    L = O.load()
    n_hit = 0
    for c in K["prims"]:
        p = fa(c["p"])
        ray = fa(c["ray"])
        out = np.zeros(10, np.float32)
        h = L.oracle_prim_hit(c["kind"], P(p), P(ray), float(fa([c["tmin"]])[0]), float(fa([c["tmax"]])[0]), P(out))
        assert bool(h) == c["hit"], c
        if h:
            n_hit += 1
            assert same(out, fa(c["rec"])), (c["kind"], out, fa(c["rec"]))
    assert n_hit > 60


def test_vector_helpers():
    L = O.load()
    for c in K["vec"]:
        v, n = fa(c["v"]), fa(c["n"])
        eta, cos_, ri = (float(fa([c[k]])[0]) for k in ("eta", "cos", "ri"))
        out = np.zeros(3, np.float32)
        L.oracle_vec_op(0, P(v), P(n), 0.0, P(out))
        assert same(out, fa(c["reflect"]))
        uv = fa(c["normalize"])
        L.oracle_vec_op(3, P(v), P(n), 0.0, P(out))
        assert same(out, uv)
        L.oracle_vec_op(1, P(uv), P(n), eta, P(out))
        assert same(out, fa(c["refract"]))
        a = np.array([cos_, 0, 0], np.float32)
        L.oracle_vec_op(2, P(a), P(n), ri, P(out))
        assert same(out[:1], fa([c["reflectance"]]))


def test_camera_fields_and_rays():
    L = O.load()
    for c in K["camera"]:
        frm = np.array(c["frm"], np.float32)
        at = np.array(c["at"], np.float32)
        out = np.zeros(24, np.float32)
        L.oracle_camera(P(frm), P(at), c["fov"], c["aperture"], 10.0, 0.0, 1.0, c["W"], c["H"], P(out))
        assert same(out[:22], fa(c["fields"])), c["frm"]
        for r in c["rays"]:
            disk = fa(r["disk"])
            o = np.zeros(7, np.float32)
            L.oracle_camera_ray(P(frm), P(at), c["fov"], c["aperture"], 10.0, c["W"], c["H"],
                                float(fa([r["s"]])[0]), float(fa([r["t"]])[0]), P(disk), float(fa([r["time"]])[0]), P(o))
            assert same(o, fa(r["ray"]))


def test_perlin_tables_noise_and_textures():
    L = O.load()
    rv = np.zeros(768, np.float32)
    pm = np.zeros(768, np.uint32)
    L.oracle_perlin_tables(1, P(rv), P(pm))
    want = K["perlin_tables_seed1"]
    assert np.array_equal(rv.view(np.uint32), np.array(want["ranvec"], np.uint32))
    assert np.array_equal(pm, np.array(want["perm"], np.uint32))
    # each permutation is a single 256-cycle (Sattolo)
    for c in range(3):
        p = pm[256 * c:256 * (c + 1)]
        seen, i, n = set(), 0, 0
        while i not in seen:
            seen.add(i)
            i = int(p[i])
            n += 1
        assert n == 256
    out = np.zeros(3, np.float32)
    for c in K["perlin"]:
        p = fa(c["p"])
        assert same([L.oracle_perlin(P(rv), P(pm), 0, P(p), 0)], fa([c["noise"]]))
        assert same([L.oracle_perlin(P(rv), P(pm), 1, P(p), 7)], fa([c["turb"]]))
        L.oracle_texture(1, P(p), 0.0, 0.0, 4.0, P(rv), P(pm), None, 0, 0, 0, P(out))
        assert same(out, fa(c["tex4"]))
        L.oracle_texture(1, P(p), 0.0, 0.0, 0.1, P(rv), P(pm), None, 0, 0, 0, P(out))
        assert same(out, fa(c["tex01"]))
    for c in K["checker"]:
        p = fa(c["p"])
        L.oracle_texture(0, P(p), 0.0, 0.0, 0.0, None, None, None, 0, 0, 0, P(out))
        assert same(out, fa(c["value"]))
    img = np.array(K["image"]["data"], np.uint8).reshape(K["image"]["shape"])
    h, w, ch = img.shape
    for c in K["image"]["cases"]:
        p = np.zeros(3, np.float32)
        L.oracle_texture(2, P(p), float(fa([c["u"]])[0]), float(fa([c["v"]])[0]), 0.0, None, None, P(img), w, h, ch, P(out))
        assert same(out, fa(c["value"]))


@pytest.mark.parametrize("op,fn,lo,hi", [
    (0, math.sin, -3e4, 3e4), (1, math.cos, -3e4, 3e4), (2, math.acos, -1, 1), (4, math.log, 1e-7, 1),
    (5, lambda x: x ** 5, 0, 1), (6, math.tan, -1.5, 1.5), (3, math.atan2, -10, 10)])
def test_transcendentals_correctly_rounded(op, fn, lo, hi):
    """hd_math's f64-evaluated functions equal the correctly rounded f32 result except in rare
    midpoint cases (<= 1e-4 of inputs) and are never more than 1 ulp away."""
    rs = np.random.default_rng(op)
    x = rs.uniform(lo, hi, 20000).astype(np.float32)
    y = rs.uniform(lo, hi, 20000).astype(np.float32) if op == 3 else None
    got = O.math(op, x, y)
    if op == 3:
        want = np.array([np.float32(fn(float(a), float(b))) for a, b in zip(x, y)], np.float32)
    else:
        want = np.array([np.float32(fn(float(a))) for a in x], np.float32)
    ulps = np.abs(got.view(np.int32).astype(np.int64) - want.view(np.int32).astype(np.int64))
    assert ulps.max() <= 1
    assert np.mean(ulps > 0) <= 1e-4


def test_transcendental_special_values():
    x = np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.nan, 1e-30, 3.0e38], np.float32)
    s = O.math(0, x)
    assert s[0] == 0 and np.signbit(s[1]) and np.isnan(s[4]) and np.isnan(s[6])
    a = O.math(2, np.array([1.0, -1.0, 0.0, 1.0000001, np.nan], np.float32))
    assert a[0] == 0 and a[1] == np.float32(math.pi) and a[2] == np.float32(math.pi / 2) and np.isnan(a[3]) and np.isnan(a[4])
    l = O.math(4, np.array([0.0, 1.0, -1.0, np.inf], np.float32))
    assert l[0] == -np.inf and l[1] == 0 and np.isnan(l[2]) and l[3] == np.inf
    at = O.math(3, np.array([0.0, -0.0, 0.0, 1.0], np.float32), np.array([-0.0, -0.0, 0.0, 0.0], np.float32))
    assert at[0] == np.float32(math.pi) and at[1] == -np.float32(math.pi) and at[2] == 0 and at[3] == np.float32(math.pi / 2)
