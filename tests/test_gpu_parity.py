"""GPU parity: the HIP megakernel (through the C ABI) against the CPU oracle at a fixed seed.

Bar (north star): per-pixel L-infinity <= 1e-3 on RGB.  The two sides share every branch-deciding
operation (hd_math.h, -ffp-contract=off), so the paths are identical: the device's segment count
(world.hit calls) must equal the oracle's exactly, and the only RGB difference left is the order in
which each path's radiance is accumulated (front-to-back on the GPU, recursive in the reference).
"""
import numpy as np
import pytest

import hrt
from oracle import oracle as O

TOL = 1e-3

# (preset, width, height, spp, depth): every scene feature of the reference
CASES = [
    ("random", 64, 36, 16, 50),
    ("two_spheres", 48, 27, 16, 50),
    ("two_perlin_spheres", 48, 27, 16, 50),
    ("earth", 48, 27, 16, 50),
    ("simple_light", 48, 27, 16, 50),
    ("cornell", 40, 40, 16, 50),
    ("cornell_smoke", 40, 40, 16, 50),
    ("final", 40, 40, 8, 50),
    ("earth_perlin", 48, 27, 16, 50),
    ("random_10k", 48, 27, 4, 50),
    ("features", 64, 36, 16, 50),
]


def _gpu_render(name, w, h, spp, depth, seed, earth, region=None, sample_offset=0):
    s = hrt.preset(name, 1, earth)
    s.commit()
    cam = hrt.preset_camera(s.info, w, h)
    p = hrt.params(w, h, spp, depth, seed, tuple(s.info.background), sample_offset=sample_offset)
    img, st = hrt.render(s, cam, p, region=region, stats=True)
    return img, st, s


@pytest.mark.gpu
@pytest.mark.parametrize("name,w,h,spp,depth", CASES)
def test_preset_parity(name, w, h, spp, depth, earth):
    img, st, s = _gpu_render(name, w, h, spp, depth, 7, earth)
    o = O.OracleScene(hrt.PRESETS[name], 1, earth)
    ref, cnt = o.render(w, h, spp, depth, seed=7)
    assert st.pixels == w * h and st.samples == w * h * spp
    assert np.isfinite(img).all()
    assert st.segments == cnt["segments"], (st.segments, cnt["segments"])
    linf = float(np.abs(img - ref).max())
    assert linf <= TOL, f"{name}: L-inf {linf}"


@pytest.mark.gpu
def test_region_and_depth_cap(earth):
    """A sub-region renders the same pixels as the full frame; depth caps (incl. 1) match."""
    full, _, _ = _gpu_render("random", 64, 36, 8, 3, 11, earth)
    part, _, _ = _gpu_render("random", 64, 36, 8, 3, 11, earth, region=(10, 5, 20, 17))
    assert np.array_equal(full[5:22, 10:30], part)
    o = O.OracleScene(0, 1, earth)
    for depth in (1, 2):
        img, st, _ = _gpu_render("random", 32, 18, 8, depth, 3, earth)
        ref, cnt = o.render(32, 18, 8, depth, seed=3)
        assert st.segments == cnt["segments"]
        assert np.abs(img - ref).max() <= TOL


@pytest.mark.gpu
def test_device_math_bit_identical():
    """hd_math transcendentals give the same bits on gfx950 as on the host."""
    rng = np.random.default_rng(0)
    xs = {
        0: rng.uniform(-2e4, 2e4, 200000).astype(np.float32),
        1: rng.uniform(-2e4, 2e4, 200000).astype(np.float32),
        2: rng.uniform(-1, 1, 200000).astype(np.float32),
        3: rng.uniform(-5, 5, 200000).astype(np.float32),
        4: rng.uniform(0, 1, 200000).astype(np.float32),
        5: rng.uniform(0, 1, 200000).astype(np.float32),
        6: rng.uniform(-1.5, 1.5, 200000).astype(np.float32),
    }
    ys = rng.uniform(-5, 5, 200000).astype(np.float32)
    for op, x in xs.items():
        y = ys if op == 3 else None
        d = hrt.device_math(op, x, y)
        h = O.math(op, x, y)
        assert np.array_equal(d.view(np.uint32), h.view(np.uint32)), f"op {op}: {np.sum(d != h)} differ"
