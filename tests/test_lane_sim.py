"""The kernels' per-lane code on the host (tests/native/lane_sim.hip over csrc/lane.h) against the oracle.

The GPU kernels schedule lane.h's functions over 64-lane waves. A lane's own sequence of box and
primitive tests and RNG draws never depends on the other lanes, so running each lane alone on the
CPU reproduces what the kernels compute per pixel. On this path, without a GPU, these tests check:
- the resumable walks (render_basic_kernel's basic_step; render_full_kernel's full_step with its
  instance re-derivation and the medium-boundary state machine);
- shading and textures (the sign-only checker);
- the fma-corrected division;
- the sample-chunk summation.

They are held to the oracle at the GPU parity bar. Paths are identical, so world.hit counts must be
equal, and radiance must agree within L-inf 1e-3. Exact culling must equal the verbatim reference
culling bit for bit.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import hrt
from conftest import tool_env
from oracle import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
TOL = 1e-3
CULL_REFERENCE, CULL_SLAB, CULL_EXACT = 0, 1, 2
BASIC_SCENES = {"random", "two_spheres", "random_10k", "motion"}
# sphere scenes with noise / image textures: the sphere kernel's HEAVY instantiation (layout.h F_HEAVY_TEX)
HEAVY_SPHERE_SCENES = {"earth", "two_perlin_spheres", "earth_perlin"}


def _build_sim(tmp_path_factory, extra=()):
    so = str(tmp_path_factory.mktemp("lanesim") / "liblanesim.so")
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    subprocess.run([hipcc, "-O2", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-shared",
                    "--offload-host-only", *extra, *os.environ.get("LANE_SIM_CFLAGS", "").split(),  # scripts/sanitize.sh
                    "-I" + os.path.join(ROOT, "include"),
                    "-I" + os.path.join(ROOT, "hyper-ray-tracer_amd", "csrc"),
                    os.path.join(HERE, "native", "lane_sim.hip"), "-o", so], check=True, env=tool_env())
    L = ctypes.CDLL(so)
    L.lane_sim_render.restype = ctypes.c_int
    L.lane_sim_chunks.restype = ctypes.c_int
    L.lane_sim_chunks.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32]
    return L


@pytest.fixture(scope="module")
def sim(tmp_path_factory):
    return _build_sim(tmp_path_factory)


@pytest.fixture(scope="module")
def sim_submuladd(tmp_path_factory):
    """The lanes with the walk's sub/mul/add box form everywhere (HRT_BOX_FMA=0: the form hybrid general
    streams use, and the one r03's general kernel diverged with)."""
    return _build_sim(tmp_path_factory, ("-DHRT_BOX_FMA=0",))


def sim_render(L, name, w, h, spp, depth, seed, earth, kernel, cull, region=None, sample_offset=0, t_min=0.001,
               options=None, view=False):
    s = hrt.preset(name, 1, earth, options=options)
    cam = hrt.preset_camera(s.info, w, h)
    if view:
        s.set_view(cam)
    blob, info = hrt.scene_blob(s)
    p = hrt.params(w, h, spp, depth, seed, tuple(s.info.background), sample_offset=sample_offset, t_min=t_min)
    x0, y0, rw, rh = region if region is not None else (0, 0, w, h)
    out = np.zeros((rh, rw, 4), np.float32)
    cnt = np.zeros(8, np.uint64)
    rc = L.lane_sim_render(blob, ctypes.byref(info), ctypes.byref(cam), ctypes.byref(p), kernel, cull, x0, y0, rw, rh,
                           out.ctypes.data_as(ctypes.c_void_p), cnt.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0
    return out, {"segments": int(cnt[0]), "samples": int(cnt[1]), "nodes": int(cnt[2]), "prims": int(cnt[3])}


def oracle_render(name, w, h, spp, depth, seed, earth, region=None, sample_offset=0, t_min=0.001):
    return O.OracleScene(hrt.PRESETS[name], 1, earth).render(w, h, spp, depth, seed=seed, region=region, threads=8,
                                                             sample_offset=sample_offset, t_min=t_min)


CASES = [
    ("random", 40, 24, 8, 50),
    ("random", 24, 16, 40, 50),          # three sample chunks
    ("two_spheres", 48, 27, 8, 50),
    ("two_perlin_spheres", 48, 27, 8, 50),
    ("earth", 48, 27, 8, 50),
    ("simple_light", 48, 27, 8, 50),
    ("cornell", 32, 32, 8, 50),
    ("cornell_smoke", 32, 32, 8, 50),
    ("final", 32, 32, 4, 50),
    ("earth_perlin", 48, 27, 8, 50),
    ("random_10k", 32, 18, 2, 50),
    ("features", 48, 27, 8, 50),
    ("motion", 48, 27, 8, 50),           # moving spheres with their own shutter intervals (TRay.tau = time)
    ("cornell", 24, 24, 4, 2),           # depth cap
    ("cornell", 12, 12, 70, 50),         # general scene: three chunks of >= 32 samples (lane.h sample_chunk)
    ("final", 8, 8, 40, 50),             # deep general scene (> 1024 nodes): 40 one-sample chunks
]


@pytest.mark.parametrize("name,w,h,spp,depth", CASES)
def test_general_kernel_lane_matches_oracle(sim, earth, name, w, h, spp, depth):
    img, st = sim_render(sim, name, w, h, spp, depth, 3, earth, kernel=1, cull=CULL_EXACT)
    ref, cnt = oracle_render(name, w, h, spp, depth, 3, earth)
    assert st["segments"] == cnt["segments"]
    assert st["samples"] == w * h * spp
    assert np.isfinite(img).all()
    assert np.abs(img - ref).max() <= TOL


@pytest.mark.parametrize("name,w,h,spp,depth", [c for c in CASES if c[0] in ("cornell_smoke", "final", "features", "random")])
def test_segment_kernel_lane_matches_general_kernel_lane(sim, earth, name, w, h, spp, depth):
    """render_kernel (one segment per wave iteration; media inside instances, HRT_KERNEL=general)."""
    a, sa = sim_render(sim, name, w, h, spp, depth, 3, earth, kernel=2, cull=CULL_EXACT)
    b, sb = sim_render(sim, name, w, h, spp, depth, 3, earth, kernel=1, cull=CULL_EXACT)
    assert sa["segments"] == sb["segments"] and sa["nodes"] == sb["nodes"]
    assert np.array_equal(a, b)


@pytest.mark.parametrize("name,w,h,spp,depth", [c for c in CASES if c[0] in BASIC_SCENES | HEAVY_SPHERE_SCENES])
def test_sphere_kernel_lane_matches_oracle_and_general_kernel(sim, earth, name, w, h, spp, depth):
    img, st = sim_render(sim, name, w, h, spp, depth, 3, earth, kernel=0, cull=CULL_EXACT)
    ref, cnt = oracle_render(name, w, h, spp, depth, 3, earth)
    assert st["segments"] == cnt["segments"]
    assert np.abs(img - ref).max() <= TOL
    full, st_full = sim_render(sim, name, w, h, spp, depth, 3, earth, kernel=1, cull=CULL_EXACT)
    assert np.array_equal(img, full) and st["segments"] == st_full["segments"]


@pytest.mark.parametrize("name,w,h,spp", [("random", 48, 27, 4), ("cornell", 32, 32, 4), ("cornell_smoke", 32, 32, 4),
                                          ("final", 32, 32, 2), ("features", 48, 27, 4), ("random_10k", 32, 18, 2)])
def test_exact_culling_equals_reference_culling_bit_for_bit(sim, earth, name, w, h, spp):
    kernel = 0 if name in BASIC_SCENES else 1
    a, sa = sim_render(sim, name, w, h, spp, 50, 5, earth, kernel=kernel, cull=CULL_EXACT)
    b, sb = sim_render(sim, name, w, h, spp, 50, 5, earth, kernel=kernel, cull=CULL_REFERENCE)
    assert sa["segments"] == sb["segments"]
    assert np.array_equal(a, b)
    assert sa["nodes"] < sb["nodes"]         # exact culling visits fewer nodes


def test_region_of_frame(sim, earth):
    full, _ = sim_render(sim, "final", 32, 32, 2, 50, 9, earth, kernel=1, cull=CULL_EXACT)
    part, _ = sim_render(sim, "final", 32, 32, 2, 50, 9, earth, kernel=1, cull=CULL_EXACT, region=(5, 7, 11, 9))
    assert np.array_equal(part, full[7:16, 5:16])


@pytest.mark.parametrize("kernel,name", [(0, "random"), (1, "cornell_smoke"), (1, "features")])
def test_sample_offset_and_t_min(sim, earth, kernel, name):
    """bench.py --scaling weak gives rank r the samples [r*spp, (r+1)*spp) (sample_offset); t_min is
    application.rs:482's 0.001 by default and a render parameter here."""
    for off, tmin in ((500, 0.001), (0, 0.01), (7, 0.0)):
        img, st = sim_render(sim, name, 32, 18, 4, 50, 11, earth, kernel=kernel, cull=CULL_EXACT,
                             sample_offset=off, t_min=tmin)
        ref, cnt = oracle_render(name, 32, 18, 4, 50, 11, earth, sample_offset=off, t_min=tmin)
        assert st["segments"] == cnt["segments"], (off, tmin)
        assert np.abs(img - ref).max() <= TOL


@pytest.mark.parametrize("depth", [1, 2, 3])
def test_depth_caps(sim, earth, depth):
    for kernel, name in ((0, "random"), (1, "final")):
        img, st = sim_render(sim, name, 24, 16, 4, depth, 2, earth, kernel=kernel, cull=CULL_EXACT)
        ref, cnt = oracle_render(name, 24, 16, 4, depth, 2, earth)
        assert st["segments"] == cnt["segments"]
        assert np.abs(img - ref).max() <= TOL


def test_headline_frame_band_at_500_spp(sim, earth):
    """Two rows through the middle of the BASELINE frame (1920x1080, 500 spp, depth 50: 32 sample
    chunks) on the sphere kernel's lane, against the oracle."""
    region = (0, 539, 1920, 2)
    img, st = sim_render(sim, "random", 1920, 1080, 500, 50, 1, earth, kernel=0, cull=CULL_EXACT, region=region)
    ref, cnt = oracle_render("random", 1920, 1080, 500, 50, 1, earth, region=region)
    assert st["samples"] == 1920 * 2 * 500
    assert st["segments"] == cnt["segments"]
    assert np.abs(img - ref).max() <= TOL


@pytest.mark.parametrize("name", ["random", "random_10k", "two_spheres"])
def test_walk_stream_regrouped_equals_reference_hierarchy(sim, earth, name, monkeypatch):
    """The sphere kernel's walk stream re-groups the inner boxes over the reference's leaf order
    (scene.cpp build_walk): bit-identical to the walk over the reference hierarchy, with fewer node visits."""
    a, sa = sim_render(sim, name, 48, 27, 4, 50, 5, earth, kernel=0, cull=CULL_EXACT)
    b, sb = sim_render(sim, name, 48, 27, 4, 50, 5, earth, kernel=0, cull=CULL_EXACT, options={"walk_tree": 1})
    assert sa["segments"] == sb["segments"] and sa["prims"] == sb["prims"]
    assert np.array_equal(a, b)
    _, info = hrt.scene_blob(hrt.preset(name, 1, earth, options={"walk_tree": 1}))
    assert info.walk_regrouped == 0 and info.walk_bytes > 0
    monkeypatch.setenv("HRT_WALK_TREE", "reference")  # r04's environment knob: no longer read by the library
    _, info = hrt.scene_blob(hrt.preset(name, 1, earth))
    assert info.walk_regrouped == 1
    if name != "two_spheres":  # (two leaves: nothing to re-group)
        assert sa["nodes"] < 0.95 * sb["nodes"], (sa["nodes"], sb["nodes"])
    print(name, "node visits: re-grouped", sa["nodes"], "reference hierarchy", sb["nodes"])


GENERAL_CASES = [c for c in CASES if c[0] not in BASIC_SCENES | HEAVY_SPHERE_SCENES]


@pytest.mark.parametrize("name,w,h,spp,depth", GENERAL_CASES)
def test_general_walk_lane_matches_oracle_and_general_lane(sim, earth, name, w, h, spp, depth):
    """render_gwalk_kernel's lane: the general walk stream (leaf objects of the reference stream under a
    re-grouped hierarchy, layout.h) with each passed leaf's program run from the world ray.  Held to the
    oracle, and bit for bit to render_full_kernel's lane (same tests in the same order, same shading)."""
    img, st = sim_render(sim, name, w, h, spp, depth, 3, earth, kernel=3, cull=CULL_EXACT)
    ref, cnt = oracle_render(name, w, h, spp, depth, 3, earth)
    assert st["segments"] == cnt["segments"]
    assert np.abs(img - ref).max() <= TOL
    full, sf = sim_render(sim, name, w, h, spp, depth, 3, earth, kernel=1, cull=CULL_EXACT)
    assert np.array_equal(img, full) and st["segments"] == sf["segments"]
    print(name, "primitive tests: general walk", st["prims"], "full lane", sf["prims"])


@pytest.mark.parametrize("name", ["cornell", "final", "features", "cornell_smoke", "simple_light"])
def test_general_walk_stream_regrouped_equals_reference_hierarchy(sim, earth, name, monkeypatch):
    a, sa = sim_render(sim, name, 32, 24, 4, 50, 5, earth, kernel=3, cull=CULL_EXACT)
    b, sb = sim_render(sim, name, 32, 24, 4, 50, 5, earth, kernel=3, cull=CULL_EXACT, options={"walk_tree": 1})
    assert sa["segments"] == sb["segments"] and sa["prims"] == sb["prims"]
    assert np.array_equal(a, b)
    print(name, "node visits: re-grouped", sa["nodes"], "reference hierarchy", sb["nodes"])


@pytest.mark.parametrize("name", ["cornell", "final", "features"])
def test_flattened_instance_chains_equal_whole_programs(sim, earth, name, monkeypatch):
    """Instance chains flattened into leaves of their own (each in the innermost frame, after the
    world-frame box test around the chain: layout.h GL_INST) against whole-chain leaf programs
    (HRT_GWALK_FLAT=0): bit-identical, with fewer primitive tests (each flattened leaf is culled by the
    world image of its own geometry)."""
    a, sa = sim_render(sim, name, 32, 24, 4, 50, 6, earth, kernel=3, cull=CULL_EXACT)
    monkeypatch.setenv("HRT_GWALK_FLAT", "0")
    b, sb = sim_render(sim, name, 32, 24, 4, 50, 6, earth, kernel=3, cull=CULL_EXACT)
    assert sa["segments"] == sb["segments"]
    assert np.array_equal(a, b)
    assert sa["prims"] <= sb["prims"]
    print(name, "primitive tests: flattened", sa["prims"], "whole programs", sb["prims"])


def test_group_box_is_tested_once_per_group(sim, earth):
    """A BvhNode leaf holding a chain of instances (a Cornell box: Translation(Rotation(Cuboid))) is
    tested ONCE by the reference, before all six sides; the flattened leaves keep that test's outcome for
    the group (lane.h gwalk_leaf_test gstate).  Re-testing the box before each side with the shrunken
    closest drops sides in rare near-tangent cases: this pixel of BASELINE config 5 (Cornell 2048^2, 1250
    spp) has 12 more world.hit calls that way (found on the GPU: the C5 band was 12 rays off the oracle)."""
    region = (1773, 300, 1, 1)
    img, st = sim_render(sim, "cornell", 2048, 2048, 1250, 50, 1, earth, kernel=3, cull=CULL_EXACT, region=region)
    ref, cnt = oracle_render("cornell", 2048, 2048, 1250, 50, 1, earth, region=region)
    assert st["segments"] == cnt["segments"] == 12578
    assert np.abs(img - ref).max() <= TOL


def _chunks(L, spp, cls, tail=32):
    buf = (ctypes.c_uint32 * 4096)()
    n = L.lane_sim_chunks(spp, cls, tail, buf, 2048)
    return [(buf[2 * k], buf[2 * k + 1]) for k in range(n)]


@pytest.mark.parametrize("spp", [1, 7, 16, 17, 40, 64, 70, 100, 500, 1000, 1250, 2000, 10000])
@pytest.mark.parametrize("cls", [0, 1, 2])
def test_sample_chunks_partition_the_samples(sim, spp, cls):
    """lane.h chunk_plan: head chunks of c samples (the first holds the remainder), then a halving tail
    c/2, c/2, ..., 1, 1; the chunks partition [0, spp) in order, and the first chunk is the only one that
    ends at or before c (the kernels count a pixel once, at its first chunk)."""
    ch = _chunks(sim, spp, cls)
    assert ch[0][0] == 0 and ch[-1][1] == spp
    assert all(a[1] == b[0] for a, b in zip(ch, ch[1:]))
    assert all(s1 > s0 for s0, s1 in ch)
    uni = _chunks(sim, spp, cls, tail=0)
    c = max(s1 - s0 for s0, s1 in uni)
    assert [s1 <= c for _, s1 in ch].count(True) == 1
    sizes = [s1 - s0 for s0, s1 in ch]
    if len(ch) > len(uni):  # a tail: non-increasing sizes after the head, ending in single samples
        tail = sizes[len(ch) - 2 * (c.bit_length() - 1):]
        assert tail == sorted(tail, reverse=True) and tail[-2:] == [1, 1]


def test_sample_chunks_of_the_headline_frame(sim):
    """C2 (500 spp, sphere class): 30 head chunks (6, then 29 of 16) and the tail 8, 8, 4, 4, 2, 2, 1, 1."""
    sizes = [b - a for a, b in _chunks(sim, 500, 0)]
    assert sizes == [6] + [16] * 29 + [8, 8, 4, 4, 2, 2, 1, 1]


def _cull_rays(rng, c, r, n):
    """Rays aimed at grazing points of the sphere (c, r): origins from inside its box to 1e4 radii away,
    targets on the surface jittered by 1e-8 .. 1 radius, directions of any scale, some axis-aligned."""
    u = rng.normal(size=(n, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    w = rng.normal(size=(n, 3))
    w -= (w * u).sum(axis=1, keepdims=True) * u
    w /= np.maximum(np.linalg.norm(w, axis=1, keepdims=True), 1e-30)
    target = c + r * u + (r * 10.0 ** rng.uniform(-8, 0, size=(n, 1))) * w * rng.choice([-1.0, 1.0], size=(n, 1))
    v = rng.normal(size=(n, 3))
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    o = c + v * (r * 10.0 ** rng.uniform(-0.5, 4, size=(n, 1)))
    d = (target - o) * 10.0 ** rng.uniform(-3, 3, size=(n, 1))
    axis = rng.random(n) < 0.1  # zero components: rays that set_dir puts in NaN mode
    d[axis, rng.integers(0, 3, size=int(axis.sum()))] = 0.0
    return np.concatenate([o, d], axis=1).astype(np.float32)


def test_exact_culling_property_on_grazing_rays(sim):
    """the walk's inflated box test never culls a sphere whose reference test accepts a
    root, including grazing false hits outside the sphere's box (G18), tiny spheres far from the origin
    (the CE_FLOOR bound of the fused o*inv form) and rays with zero direction components (NaN mode)."""
    rng = np.random.default_rng(7)
    spheres = []
    for _ in range(60):  # tiny spheres far from the world origin: the floor raises their boxes
        spheres.append((*rng.uniform(-5000, 5000, 3), 10.0 ** rng.uniform(-6, -2)))
    for _ in range(60):  # scene-sized spheres
        spheres.append((*rng.uniform(-50, 50, 3), 10.0 ** rng.uniform(-1, 1)))
    spheres += [(0.0, -1000.0, 0.0, 1000.0), (0.0, 0.0, 0.0, 5000.0), (4.0, 1.0, 0.0, 1.0)]
    fn = sim.lane_sim_cull_property
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_float, ctypes.c_float,
                   ctypes.c_void_p]
    total = np.zeros(6, np.uint64)
    for s in spheres:
        sph = np.array(s, np.float32)
        rays = _cull_rays(rng, sph[:3].astype(np.float64), float(sph[3]), 4000)
        cnt = np.zeros(6, np.uint64)
        assert fn(sph.ctypes.data, 1, rays.ctypes.data, len(rays), 0.001, float("inf"), cnt.ctypes.data) == 0
        assert cnt[2] == 0 and cnt[3] == 0, (s, cnt)
        total += cnt
    accepted, outside, _, _, raised, nan_rays = (int(x) for x in total)
    print("cull property totals", total)
    assert accepted > 100000 and outside > 0  # grazing false hits were produced and none was culled
    assert raised >= 60 and nan_rays > 0


def test_medium_sphere_pair_equals_two_boundary_queries(sim):
    """a medium over one sphere answers constant_medium.rs:37-48's two boundary queries
    (boundary.hit(-inf, inf), then boundary.hit(t1 + 0.0001, inf)) from ONE evaluation of the quadratic
    (lane.h sphere_pair_at, GL_MED leaves and medium_pair).  Held bit for bit to the two sphere tests made
    separately (sphere_root_at) on grazing rays, origins inside, on and outside the sphere, rays starting
    just past the near root, tangent rays, zero and denormal directions and NaN rays."""
    rng = np.random.default_rng(13)
    spheres = [(0.0, 0.0, 0.0, 5000.0), (0.0, 150.0, 145.0, 70.0), (360.0, 150.0, 145.0, 70.0), (4.0, 1.0, 0.0, 1.0),
               (0.0, -1000.0, 0.0, 1000.0)]
    spheres += [(*rng.uniform(-100, 100, 3), 10.0 ** rng.uniform(-2, 2)) for _ in range(20)]
    fn = sim.lane_sim_sphere_pair
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
    total = np.zeros(3, np.int64)
    for s in spheres:
        c, rad = np.array(s[:3], np.float64), float(s[3])
        rays = list(_cull_rays(rng, c, rad, 3000))  # grazing and missing rays around the sphere
        for _ in range(600):  # origins inside, on and near the surface, random directions
            d = rng.normal(size=3)
            d /= np.linalg.norm(d)
            o = c + d * rad * rng.choice([0.0, 0.3, 0.999, 1.0, 1.001, 2.0])
            rays.append(np.r_[o, rng.normal(size=3) * 10.0 ** rng.uniform(-3, 3)])
        o = c + np.array([rad * 2, 0.0, 0.0])
        rays += [np.r_[o, -1.0, 0.0, 0.0], np.r_[o, 0.0, 0.0, 0.0], np.r_[o, 1e-42, 0.0, 0.0],
                 np.r_[c + np.array([-rad * 2, rad, 0.0]), 1.0, 0.0, 0.0],  # tangent
                 np.r_[o, np.nan, 0.0, 1.0], np.r_[np.nan, 0.0, 0.0, 1.0, 0.0, 0.0]]
        rays = np.asarray(rays, np.float32)
        sph = np.array(s, np.float32)
        out = np.zeros((len(rays), 6), np.float32)
        assert fn(sph.ctypes.data, 1, rays.ctypes.data, len(rays), out.ctypes.data) == 0
        pair, two = out[:, :3], out[:, 3:]
        assert np.array_equal(pair.view(np.uint32), two.view(np.uint32)), s  # bit for bit, NaN payloads included
        for k in range(3):
            total[k] += int((pair[:, 0] == k).sum())
    print("sphere pair: rays with 0 / 1 / 2 boundary hits", total)
    assert total.min() > 100  # every outcome was exercised


def sim_render_scene(L, s, w, h, spp, kernel, cull, seed=11):
    """sim_render for a scene built through the ABI's constructors (tests/scenes.py)."""
    import scenes

    blob, info = hrt.scene_blob(s)
    cam = scenes.camera(w, h)
    p = hrt.params(w, h, spp, 50, seed)
    out = np.zeros((h, w, 4), np.float32)
    cnt = np.zeros(8, np.uint64)
    rc = L.lane_sim_render(blob, ctypes.byref(info), ctypes.byref(cam), ctypes.byref(p), kernel, cull, 0, 0, w, h,
                           out.ctypes.data_as(ctypes.c_void_p), cnt.ctypes.data_as(ctypes.c_void_p))
    return rc, out, {"segments": int(cnt[0]), "nodes": int(cnt[2]), "prims": int(cnt[3])}


def test_custom_scenes_exact_lanes_equal_reference_traversal(sim):
    """sphere-only scenes with Lists in BvhNodes walk the GENERAL stream (render_gwalk_kernel's
    lane; the sphere lane refuses it), a List around a nested BvhNode of Lists keeps its group whole, and a
    textured sphere scene beyond the LDS budget walks the sphere stream (HEAVY): each bit for bit equal to
    the verbatim reference traversal of the segment kernel's lane."""
    import scenes

    for make, kernel, (w, h, spp) in ((scenes.sphere_lists, 3, (48, 27, 6)), (scenes.big_textured, 0, (48, 27, 4))):
        s = make()
        rc, a, sa = sim_render_scene(sim, s, w, h, spp, kernel, CULL_EXACT)
        assert rc == 0
        rc, b, sb = sim_render_scene(sim, s, w, h, spp, 2, CULL_REFERENCE)
        assert rc == 0
        assert sa["segments"] == sb["segments"] and np.array_equal(a, b), make.__name__
        assert sa["nodes"] < sb["nodes"]
    rc, _, _ = sim_render_scene(sim, scenes.sphere_lists(), 8, 8, 1, 0, CULL_EXACT)
    assert rc == 1  # no sphere stream: the sphere kernel's lane must not run it


# (x, y, sample) of Cornell 2048^2 (C5) whose paths meet a NaN hit (DESIGN G20: rect.rs divides 0 by 0 for a
# ray that starts on a rect's plane parallel to it, and accepts t = NaN); found by scripts/box_hunt.py on
# C5's 1/8 share at 10000 spp, where the r03 kernels left the oracle's path
NAN_HIT_SAMPLES = [(1644, 1582, 3973), (1574, 232, 8326), (410, 250, 4811)]


@pytest.mark.parametrize("form", ["fused", "submuladd"])
@pytest.mark.parametrize("x,y,sample", NAN_HIT_SAMPLES)
def test_nan_hit_paths_match_oracle(sim, sim_submuladd, earth, x, y, sample, form):
    """After a NaN hit the reference passes every box (aabb.rs: `t_max <= t_min` is false for a NaN t_max) and
    accepts the next hit at any t; the lanes' reference test must keep that (no fminf dropping the NaN), and
    EXACT culling must not cull for a ray that can meet a NaN hit (set_noinv's NaN mode): every lane, both
    culling modes, the oracle's world.hit count; the first sample is the one whose path is all NaN hits."""
    W = H = 2048
    lanes = sim if form == "fused" else sim_submuladd
    ref, cnt = oracle_render("cornell", W, H, 1, 50, 1, earth, region=(x, y, 1, 1), sample_offset=sample)
    for kernel, cull in ((3, CULL_EXACT), (1, CULL_EXACT), (2, CULL_EXACT), (2, CULL_REFERENCE), (1, CULL_REFERENCE)):
        img, st = sim_render(lanes, "cornell", W, H, 1, 50, 1, earth, kernel=kernel, cull=cull, region=(x, y, 1, 1),
                             sample_offset=sample)
        assert st["segments"] == cnt["segments"], (kernel, cull, st["segments"], cnt["segments"])
        assert np.array_equal(img, ref, equal_nan=True) or np.abs(img - ref).max() <= TOL, (kernel, cull, img, ref)


def test_nan_hit_path_is_all_nan(sim, earth):
    """The first sample's path: segment 3 starts on the floor (y = 0) with a direction whose y component is 0
    (a Lambertian scatter whose unit vector rounds to the normal's opposite), so the floor's test gives 0 / 0;
    every later segment starts at a NaN point and meets NaN hits again, up to the depth cap."""
    W = H = 2048
    s = hrt.preset("cornell", 1, earth)
    blob, info = hrt.scene_blob(s)
    cam = hrt.preset_camera(s.info, W, H)
    p = hrt.params(W, H, 1, 50, 1, tuple(s.info.background))
    fn = sim.lane_sim_path
    fn.restype = ctypes.c_int
    out = np.zeros(9 * 64, np.float32)
    for cull in (CULL_EXACT, CULL_REFERENCE):
        n = fn(blob, ctypes.byref(info), ctypes.byref(cam), ctypes.byref(p), cull, 1644, 1582, 3973,
               out.ctypes.data_as(ctypes.c_void_p), 64)
        seg = out[:9 * n].reshape(n, 9)
        assert n == 50
        assert seg[3, 1] == 0.0 and seg[3, 4] == 0.0 and np.isnan(seg[3, 7])  # o.y = 0, d.y = 0, t = NaN
        assert np.isnan(seg[4:, 0]).all()


@pytest.mark.parametrize("name", ["random"])
def test_split_node_parts_equal_interleaved(sim, earth, name, monkeypatch):
    """layout.h WALK_SPLIT_HALF: a sphere stream staged whole in LDS keeps each node part's second 16 B
    16 KB after its first (all 16 bank slots of a ds_read_b128 lane group in use); bit for bit the walk over
    32-B node parts (the default), node for node (opt-in: HRT_WALK_SPLIT=1)."""
    monkeypatch.setenv("HRT_WALK_SPLIT", "1")
    _, info = hrt.scene_blob(hrt.preset(name, 1, earth))
    assert info.walk_half == 16384 and info.walk_hot == 0
    a, sa = sim_render(sim, name, 48, 27, 8, 50, 5, earth, kernel=0, cull=CULL_EXACT)
    monkeypatch.setenv("HRT_WALK_SPLIT", "0")
    _, info0 = hrt.scene_blob(hrt.preset(name, 1, earth))
    assert info0.walk_half == 16
    b, sb = sim_render(sim, name, 48, 27, 8, 50, 5, earth, kernel=0, cull=CULL_EXACT)
    assert sa["segments"] == sb["segments"] and sa["nodes"] == sb["nodes"]
    assert np.array_equal(a, b)


def test_hybrid_split_node_parts_equal_interleaved(sim, earth, monkeypatch):
    """layout.h WALK_SPLIT_HALF_HYB (r06): a hybrid sphere stream (random-10k: 1.6 MB, its
    view-ranked node parts staged) in pages of 512 node parts, first halves then second halves 8 KB later, the
    staged part ending on a page's second halves; the walk over it equals the 32-B layout's bit for bit, and the
    layout's invariants hold (staged set inside the LDS budget, every payload beyond it, every leaf's skip = the
    successor its payload keeps)."""
    s0 = hrt.preset("random_10k", 1, earth)
    s0.set_view(hrt.preset_camera(s0.info, 96, 54))
    _, info0 = hrt.scene_blob(s0)
    monkeypatch.setenv("HRT_WALK_SPLIT", "1")
    s1 = hrt.preset("random_10k", 1, earth)
    s1.set_view(hrt.preset_camera(s1.info, 96, 54))
    blob, info = hrt.scene_blob(s1)
    assert info.walk_half == 8192 and 0 < info.walk_hot <= 77 * 1024 and info.walk_hot > 70 * 1024
    assert info.walk_nodes == info0.walk_nodes and info0.walk_half == 16
    w = np.frombuffer(blob.raw, np.uint8)[info.off_walk:info.off_walk + info.walk_bytes]
    u = w.view(np.uint32)
    off, leaves, seen = 0, 0, set()
    while off < info.walk_bytes:  # pre-order through pass / skip links: every node part once, payloads beyond the staged part
        assert off not in seen and off % 16 == 0 and (off // 8192) % 2 == 0  # a first half, on a page's first half
        seen.add(off)
        skip, pas = int(u[off // 4 + 3]), int(u[(off + 8192) // 4 + 3])
        if pas & (1 << 31):
            q = pas - (1 << 31)
            assert q >= info.walk_hot and int(u[q // 4 + 3]) >> 2 == skip
            leaves += 1
            off = skip
        else:
            off = pas
    assert len(seen) == info.walk_nodes and leaves == (info.walk_nodes + 1) // 2
    monkeypatch.delenv("HRT_WALK_SPLIT")
    a, sa = sim_render(sim, "random_10k", 48, 27, 4, 50, 5, earth, kernel=0, cull=CULL_EXACT, view=True)
    monkeypatch.setenv("HRT_WALK_SPLIT", "1")
    b, sb = sim_render(sim, "random_10k", 48, 27, 4, 50, 5, earth, kernel=0, cull=CULL_EXACT, view=True)
    assert sa == sb
    assert np.array_equal(a, b)


@pytest.mark.parametrize("knob", ["HRT_GWALK_MED=0", "HRT_GWALK_BIG=0"])
def test_final_general_walk_variants(sim, earth, knob, monkeypatch):
    """Final's general walk with a one-sphere medium as a flat program (layout.h GL_MED) and with the 152-KB
    staged set (GWALK_LDS_BIG_BYTES), against the generic program / the 77-KB set: the same frame bit for bit
    and the same work counters (gwalk_medium counts what trace_ray's node loop would)."""
    a, sa = sim_render(sim, "final", 40, 40, 4, 50, 9, earth, kernel=3, cull=CULL_EXACT)
    k, v = knob.split("=")
    monkeypatch.setenv(k, v)
    b, sb = sim_render(sim, "final", 40, 40, 4, 50, 9, earth, kernel=3, cull=CULL_EXACT)
    assert sa == sb
    assert np.array_equal(a, b)


@pytest.fixture(scope="module")
def sim_perlin_select(tmp_path_factory):
    """The lanes with the reference's multiply form of the Perlin corner weights (lane.h HRT_PERLIN_SELECT=0; the
    kernels' default since r06 selects u or 1 - u)."""
    return _build_sim(tmp_path_factory, ("-DHRT_PERLIN_SELECT=0",))


@pytest.mark.parametrize("variant", ["default", "multiply"])
def test_perlin_lane_code_equals_oracle_bit_for_bit(sim, sim_perlin_select, variant):
    """lane.h perlin_noise_t / noise_value_t (the kernels' Perlin) against the oracle's perlin_noise.rs
    restatement on the scene's tables: noise and the noise texture's turbulence term, bit for bit, over points
    of every scale (negative, integer, huge, tiny) -- the corner weights are exact simplifications of the
    reference's x u + (1 - x)(1 - u)."""
    sim = sim if variant == "default" else sim_perlin_select
    L = O.load()
    rv = np.zeros(768, np.float32)
    pm = np.zeros(768, np.uint32)
    L.oracle_perlin_tables(1, rv.ctypes.data_as(ctypes.c_void_p), pm.ctypes.data_as(ctypes.c_void_p))
    sim.lane_sim_perlin.restype = ctypes.c_float
    sim.lane_sim_perlin.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_float]
    rng = np.random.default_rng(5)
    pts = np.concatenate([rng.uniform(-50, 50, (3000, 3)), rng.uniform(-1e5, 1e5, (500, 3)),
                          np.round(rng.uniform(-20, 20, (300, 3))), rng.uniform(-1e-3, 1e-3, (300, 3)),
                          rng.uniform(-1e9, 1e9, (100, 3))]).astype(np.float32)
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    for p in pts:
        p = np.ascontiguousarray(p)
        n_l = sim.lane_sim_perlin(vp(rv), vp(pm), 0, vp(p), 1.0)
        n_o = L.oracle_perlin(vp(rv), vp(pm), 0, vp(p), 0)
        assert np.float32(n_l).view(np.uint32) == np.float32(n_o).view(np.uint32), (p, n_l, n_o)
        for scale in (4.0, 0.1):
            t_l = sim.lane_sim_perlin(vp(rv), vp(pm), 1, vp(p), scale)
            q = (np.float32(scale) * p).astype(np.float32)
            t_o = L.oracle_perlin(vp(rv), vp(pm), 1, vp(q), 7)
            # noise_value_t = 1 + sin_f(scale p.z + 10 |turb|): compare the turbulence through it
            assert np.isfinite(t_l) or not np.isfinite(t_o)
            want = 1.0 + float(np.float32(np.sin(np.float64(np.float32(np.float32(scale) * p[2]) + np.float32(10.0 * abs(np.float32(t_o)))))))
            assert abs(t_l - want) <= 2e-6 * max(1.0, abs(want)), (p, scale, t_l, want)


def test_foggy_scene_media_shapes(sim, monkeypatch):
    """tests/scenes.py foggy: every medium shape the general walk stream distinguishes (flat GL_MED programs over
    a sphere and a moving sphere, a box-less List member, a Cuboid boundary, a fog around everything).  The
    general walk lane under EXACT equals the verbatim reference traversal of the segment lane bit for bit, and
    equals itself with the media as generic programs (HRT_GWALK_MED=0)."""
    import scenes

    s = scenes.foggy()
    blob, info = hrt.scene_blob(s)
    flags = [f for _, _, f, _ in scenes.general_stream_leaves(blob, info)]
    assert sum(1 for f in flags if f & scenes.GL_MED) == 3  # the sphere, the moving sphere, the fog
    rc, a, sa = sim_render_scene(sim, s, 40, 24, 6, 3, CULL_EXACT)
    assert rc == 0
    rc, b, sb = sim_render_scene(sim, s, 40, 24, 6, 2, CULL_REFERENCE)
    assert rc == 0
    assert sa["segments"] == sb["segments"] and np.array_equal(a, b)
    monkeypatch.setenv("HRT_GWALK_MED", "0")
    s2 = scenes.foggy()
    rc, c, sc = sim_render_scene(sim, s2, 40, 24, 6, 3, CULL_EXACT)
    assert rc == 0
    assert sa == sc and np.array_equal(a, c)


def _c16_boxes(blob, info):
    """The 16-B walk stream's node boxes as [lo, hi] in the tree's pre-order (layout.h WALK_C16)."""
    words = np.frombuffer(bytes(blob), np.uint32)[info.off_walk // 4:(info.off_walk + info.walk_bytes) // 4]
    parts = words[:info.walk_nodes * 4].reshape(-1, 4)
    halves = parts[:, :3].copy().view(np.float16).astype(np.float64).reshape(-1, 6)  # Cx Cy Cz Ex Ey Ez
    C, E = halves[:, :3], halves[:, 3:]
    out = []

    def walk(j):
        out.append((C[j] - E[j], C[j] + E[j]))
        p = int(parts[j, 3]) >> 16
        if p & 0x8000:
            return
        walk(p)
        walk(int(parts[p, 3]) & 0xFFFF)

    walk(0)
    return out


def _b32_boxes(blob, info):
    """The 32-B walk stream's node boxes [C - E, C + E] in the tree's pre-order (layout.h)."""
    base = info.off_walk
    raw = bytes(blob)[base:base + info.walk_bytes]
    out = []

    def part(off):
        return np.frombuffer(raw[off:off + 32], np.float32), np.frombuffer(raw[off:off + 32], np.uint32)

    def walk(off):
        f, u = part(off)
        C, E = f[:3].astype(np.float64), f[4:7].astype(np.float64)
        out.append((C - E, C + E))
        if u[7] & 0x80000000:
            return
        walk(int(u[7]))
        walk(int(part(int(u[7]))[1][3]))

    walk(0)
    return out


def test_c16_stream_boxes_hold_the_32b_boxes_and_nest(monkeypatch):
    """layout.h WALK_C16 (opt-in, HRT_WALK_C16=1; the hybrid sphere stream of random_10k, BASELINE config 4): every 16-B node part's
    binary16 box holds the 32-B part's box of the same node (so the node's geometry: all the inflated test
    needs), and every inner node's encoded box holds its children's encoded boxes (monotone inclusion, as in the
    32-B stream); the tree, the links and twice the staged node parts in the same LDS bytes."""
    import sys

    sys.setrecursionlimit(10000)
    monkeypatch.setenv("HRT_WALK_C16", "1")  # opt-in (layout.h WALK_C16)
    s16 = hrt.preset("random_10k", 1, None)
    b16, i16 = hrt.scene_blob(s16)
    monkeypatch.delenv("HRT_WALK_C16")
    b32, i32 = hrt.scene_blob(hrt.preset("random_10k", 1, None))
    assert i16.walk_c16 == 1 and i32.walk_c16 == 0 and i16.walk_nodes == i32.walk_nodes
    assert i16.walk_hot == i32.walk_hot and i16.walk_hot // 16 == 2 * (i32.walk_hot // 32)
    bx16, bx32 = _c16_boxes(b16, i16), _b32_boxes(b32, i32)
    assert len(bx16) == len(bx32) == i16.walk_nodes
    for (l16, h16), (l32, h32) in zip(bx16, bx32):
        assert (l16 <= l32).all() and (h16 >= h32).all()
    # nesting: parent boxes hold children's, checked along the pre-order with the parsed structure
    words = np.frombuffer(bytes(b16), np.uint32)[i16.off_walk // 4:(i16.off_walk + i16.walk_bytes) // 4]
    parts = words[:i16.walk_nodes * 4].reshape(-1, 4)
    halves = parts[:, :3].copy().view(np.float16).astype(np.float64).reshape(-1, 6)
    lo, hi = halves[:, :3] - halves[:, 3:], halves[:, :3] + halves[:, 3:]
    inner = np.nonzero((parts[:, 3] >> 16) & 0x8000 == 0)[0]
    c0 = parts[inner, 3] >> 16
    c1 = parts[c0, 3] & 0xFFFF
    for c in (c0, c1):
        assert (lo[inner] <= lo[c]).all() and (hi[inner] >= hi[c]).all()


def test_c16_stream_renders_like_the_32b_stream(sim, earth, monkeypatch):
    """The sphere lane over the 16-B stream (random_10k) against the 32-B stream: the same closest hits and
    winners, so bit-identical pixels and equal ray counts; and against the oracle at the parity bar."""
    region = (1600, 900, 32, 8)
    monkeypatch.setenv("HRT_WALK_C16", "1")  # opt-in (layout.h WALK_C16)
    a, sa = sim_render(sim, "random_10k", 3840, 2160, 6, 50, 3, earth, kernel=0, cull=CULL_EXACT, region=region)
    monkeypatch.delenv("HRT_WALK_C16")
    b, sb = sim_render(sim, "random_10k", 3840, 2160, 6, 50, 3, earth, kernel=0, cull=CULL_EXACT, region=region)
    assert sa["segments"] == sb["segments"] and np.array_equal(a, b)
    ref, cnt = oracle_render("random_10k", 3840, 2160, 6, 50, 3, earth, region=region)
    assert sa["segments"] == cnt["segments"] and np.abs(a - ref).max() <= TOL
    print("node visits: 16-B parts", sa["nodes"], "32-B parts", sb["nodes"])


@pytest.mark.parametrize("name,kernel,region", [("random_10k", 0, (1600, 900, 32, 8)), ("final", 3, (300, 420, 24, 8)),
                                                ("random", 0, (700, 500, 48, 8))])
def test_view_placement_renders_the_same_frame(sim, earth, name, kernel, region):
    """hrt_scene_set_view (DESIGN.md sections 4-5): the re-grouping DP weighs the view's camera rays (Random,
    random_10k: another hierarchy over the same leaf order, fewer node visits) and a walk stream beyond LDS
    (random_10k's sphere stream, BASELINE config 4; Final's general stream) stages the node parts those rays
    visit most.  The stream's bytes differ, its size and staged bytes do not, and the lane renders the same
    pixels bit for bit with the same rays and primitive tests (and, where only the placement moved, the same
    node visits)."""
    W, H, spp = {"random_10k": (3840, 2160, 4), "final": (800, 800, 4), "random": (1920, 1080, 8)}[name]
    s0 = hrt.preset(name, 1, earth)
    b0, i0 = hrt.scene_blob(s0)
    s1 = hrt.preset(name, 1, earth)
    s1.set_view(hrt.preset_camera(s1.info, W, H))
    b1, i1 = hrt.scene_blob(s1)
    assert (i0.walk_hot > 0) == (name != "random") and (i0.walk_hot, i0.walk_bytes) == (i1.walk_hot, i1.walk_bytes)
    w0 = bytes(b0)[i0.off_walk:i0.off_walk + i0.walk_bytes]
    w1 = bytes(b1)[i1.off_walk:i1.off_walk + i1.walk_bytes]
    assert w0 != w1
    a, sa = sim_render(sim, name, W, H, spp, 50, 3, earth, kernel=kernel, cull=CULL_EXACT, region=region)
    b, sb = sim_render(sim, name, W, H, spp, 50, 3, earth, kernel=kernel, cull=CULL_EXACT, region=region, view=True)
    assert (sa["segments"], sa["prims"]) == (sb["segments"], sb["prims"])
    if name == "final":  # its general stream keeps its hierarchy (a leaf without a box turns the view DP off)
        assert sa["nodes"] == sb["nodes"]
    else:
        assert sb["nodes"] < sa["nodes"], (sa["nodes"], sb["nodes"])
    assert np.array_equal(a, b)
    print(name, "node visits", sa["nodes"], "->", sb["nodes"])


@pytest.mark.parametrize("name", ["random", "random_10k", "final", "cornell", "cornell_smoke", "motion", "features"])
def test_leaf_skip_is_its_payload_successor(earth, name):
    """layout.h: a leaf's skip link equals the pre-order successor its payload keeps, in every stream (sphere and
    general, with and without a view).  The hybrid walk kernels continue a parked lane at the skip kept from the
    leaf's step instead of reading the successor from the payload (lane.h walk_box, HRT_KEEP_SKIP)."""
    for view in (False, True):
        s = hrt.preset(name, 1, earth)
        if view:
            s.set_view(hrt.preset_camera(s.info, 800, 600))
        b, i = hrt.scene_blob(s)
        assert i.walk_bytes > 0 and not i.walk_c16
        u = np.frombuffer(bytes(b)[i.off_walk:i.off_walk + i.walk_bytes], np.uint32)
        leaves, stack = 0, [0]
        while stack:
            off = stack.pop()
            skip, pas = int(u[off // 4 + 3]), int(u[off // 4 + 7])
            if pas & 0x80000000:
                leaves += 1
                assert int(u[(pas & 0x7FFFFFFF) // 4 + 3]) >> 2 == skip, (name, off)
            else:
                stack += [int(u[pas // 4 + 3]), pas]
        assert leaves > 0


def test_rotation_forms_bit_identical(sim):
    """lane.h rotate_any's run-time-axis form and rotate_axis<AX> (what a wave turning about one axis runs on the
    device, HRT_ROT_SPECIAL) give the same bits, on ordinary, huge, tiny, zero and signed-zero components."""
    rng = np.random.default_rng(7)
    n = 200_000
    axis = rng.integers(0, 3, n).astype(np.uint32)
    ang = rng.uniform(-np.pi, np.pi, n)
    sc = np.stack([np.sin(ang), np.cos(ang)], 1).astype(np.float32)
    od = (rng.standard_normal((n, 6)) * 10.0 ** rng.integers(-30, 30, (n, 6))).astype(np.float32)
    od[rng.random((n, 6)) < 0.05] = 0.0
    od[rng.random((n, 6)) < 0.05] = -0.0
    out = np.zeros((n, 12), np.float32)
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    sim.lane_sim_rotate(ctypes.c_uint32(n), vp(axis), vp(sc), vp(od), vp(out))
    assert np.array_equal(out[:, :6].view(np.uint32), out[:, 6:].view(np.uint32))
    assert not np.array_equal(out[:, :6], od)  # the rays did turn
