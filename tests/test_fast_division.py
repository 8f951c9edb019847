"""The walk's division by dot(d, d) (render.hip div_rn: per-ray RN(1/a) + one fma correction) is
bit-identical to IEEE division wherever its fast path is taken (Markstein's theorem).  The reference
divides in sphere.rs:47,49 / moving_sphere.rs:71,73; the oracle keeps the plain division."""
import os
import subprocess

import numpy as np
import pytest
from conftest import tool_env

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("divrn") / "div_rn_check")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", exe, os.path.join(HERE, "native", "div_rn_check.c"), "-lm"],
                   check=True, env=tool_env())
    return exe


@pytest.mark.parametrize("seed,emin,emax", [(1, -30, 30), (2, -100, 100), (3, -3, 3)])
def test_fma_corrected_division_is_correctly_rounded(checker, seed, emin, emax):
    out = subprocess.run([checker, "20000000", str(seed), str(emin), str(emax)], check=True, capture_output=True,
                         text=True).stdout.split()
    fast, bad = int(out[0]), int(out[1])
    assert fast > 5_000_000
    assert bad == 0


def test_camera_divisions_exact_on_the_whole_parameter_range(checker):
    """start_sample's u = x / (W - 1), v = y / (H - 1) use div_rn's bare core with host reciprocals and no
    IEEE fallback (lane.h): every divisor W - 1 in [1, 65534] (the accepted 2 <= W <= 65535), x = px + a
    gen_f32 draw at its edges (0, 2^-24, 0.5, 1 - 2^-24) and random, px in [0, W - 1]."""
    out = subprocess.run([checker, "camera", "5"], check=True, capture_output=True, text=True).stdout.split()
    cases, bad = int(out[0]), int(out[1])
    assert cases == 65534 * 64
    assert bad == 0


def _pairs(n, rng):
    a = (rng.random(n, dtype=np.float32) * 8).astype(np.float32) * np.float32(2.0) ** rng.integers(-40, 40, n).astype(np.float32)
    x = (rng.standard_normal(n).astype(np.float32)) * np.float32(2.0) ** rng.integers(-40, 40, n).astype(np.float32)
    # structured: all-ones significands, exact quotients, zeros of both signs, extremes, NaN/inf
    ones = np.float32(1.9999999)
    extra_a = np.array([ones, 1.0, 3.0, 2.0**-100, 2.0**100, 2.0**-120, 1e30, 0.0, np.inf, 7.0], np.float32)
    extra_x = np.array([ones, -0.0, 0.0, 1.0, -1.0, 2.0**-110, 3e38, 1.0, 1.0, np.nan], np.float32)
    return np.concatenate([x, extra_x]), np.concatenate([np.abs(a), extra_a])


@pytest.mark.gpu
def test_device_division_matches_ieee():
    import hrt

    rng = np.random.default_rng(7)
    x, a = _pairs(4_000_000, rng)
    got = hrt.device_math(7, x, a)
    with np.errstate(all="ignore"):
        ref = (x / a).astype(np.float32)
    same = (got.view(np.uint32) == ref.view(np.uint32)) | (np.isnan(got) & np.isnan(ref))
    assert same.all(), (x[~same][:5], a[~same][:5], got[~same][:5], ref[~same][:5])
