"""The walk's inflated box test (CULL_EXACT's culling half, csrc/lane.h box_ce) on the device against the same
code compiled for the host, bit for bit, in both forms (the general kernel's earlier
sub/mul/add form diverged from the oracle on the GPU only; tests/test_lane_sim.py proves the culling
property with the HOST compilation, so this pins the device's decisions to the host's).

Pairs: grazing rays aimed at spheres of every scale (test_lane_sim._cull_rays: tiny spheres far from the
origin, scene-sized ones, axis-aligned rays with zero direction components) against the spheres' boxes as
the stream builder encodes them (walk_box.h ce_floored), and every node box of the Random and Cornell walk
streams against rays of random origins and directions, some with zero or denormal components."""
import numpy as np
import pytest

import hrt
from test_lane_sim import _cull_rays


def _ce_floored(mn, mx):
    """csrc/walk_box.h ce_of + ce_floored (centre / half-extent, E rounded up, the 2^-12 floor)."""
    C, E = np.zeros(3, np.float32), np.zeros(3, np.float32)
    for k in range(3):
        lo, hi = float(mn[k]), float(mx[k])
        c = np.float32((lo + hi) * 0.5)
        e = max(float(c) - lo, hi - float(c))
        e += e * 2.0 ** -50
        ef = np.float32(e)
        if float(ef) < e:
            ef = np.nextafter(ef, np.float32(np.inf))
        C[k], E[k] = c, ef
    f = np.float32(np.ldexp(np.abs(C).max(), -12))
    if E.max() < f:
        E = np.maximum(E, f)
    return C, E


def _sphere_cases(seed=7):
    rng = np.random.default_rng(seed)
    spheres = [(*rng.uniform(-5000, 5000, 3), 10.0 ** rng.uniform(-6, -2)) for _ in range(20)]
    spheres += [(*rng.uniform(-50, 50, 3), 10.0 ** rng.uniform(-1, 1)) for _ in range(20)]
    spheres += [(0.0, -1000.0, 0.0, 1000.0), (4.0, 1.0, 0.0, 1.0)]
    for s in spheres:
        c = np.array(s[:3], np.float32)
        r = np.float32(s[3])
        C, E = _ce_floored(c - r, c + r)
        box = np.concatenate([C, [0], E, [0]]).astype(np.float32)[None]
        yield box, _cull_rays(rng, c.astype(np.float64), float(r), 3000)


def _stream_boxes(name):
    s = hrt.preset(name, 1, None)
    blob, info = hrt.scene_blob(s)
    raw = np.frombuffer(bytes(blob), np.uint8)
    base, end = int(info.off_walk), int(info.walk_bytes)
    boxes, o = [], 0
    half = int(info.walk_half)  # a node part's second 16 B (layout.h WALK_SPLIT_HALF or 16)
    while o < end:  # pre-order over the node parts (tests/scenes.py general_stream_leaves)
        a = raw[base + o:base + o + 16]
        b = raw[base + o + half:base + o + half + 16]
        boxes.append(np.concatenate([a.view(np.float32)[:3], [0], b.view(np.float32)[:3], [0]]))
        o = int(a.view(np.uint32)[3]) if b.view(np.uint32)[3] & (1 << 31) else int(b.view(np.uint32)[3])
    return np.array(boxes, np.float32)


def _random_rays(n, seed=3):
    rng = np.random.default_rng(seed)
    o = rng.uniform(-600, 600, (n, 3))
    d = rng.normal(size=(n, 3)) * 10.0 ** rng.uniform(-2, 2, (n, 1))
    z = rng.random(n) < 0.05
    d[z, rng.integers(0, 3, int(z.sum()))] = 0.0
    dn = rng.random(n) < 0.02
    d[dn, rng.integers(0, 3, int(dn.sum()))] = 1e-40  # denormal component: 1/d overflows
    return np.concatenate([o, d], axis=1).astype(np.float32)


def test_host_box_test_runs():
    """The host compilation (on_device = 0) is usable without a GPU: an infinite box always passes."""
    inf = np.float32(np.inf)
    box = np.array([[0, 0, 0, 0, inf, inf, inf, 0]], np.float32)
    rays = _random_rays(64)
    for form in (0, 1):
        assert hrt.box_test(form, box, rays, 0.001, float("inf"), on_device=False).all()


@pytest.mark.gpu
def test_device_box_test_equals_host_bit_for_bit():
    n_pairs = 0
    for box, rays in _sphere_cases():
        for form in (0, 1):
            dev = hrt.box_test(form, box, rays, 0.001, float("inf"))
            host = hrt.box_test(form, box, rays, 0.001, float("inf"), on_device=False)
            assert np.array_equal(dev, host), (form, box, np.nonzero(dev != host))
            n_pairs += dev.size
    rays = _random_rays(20000)
    for name in ("random", "cornell"):
        boxes = _stream_boxes(name)
        for form in (0, 1):
            for tmax in (float("inf"), 50.0):
                dev = hrt.box_test(form, boxes, rays, 0.001, tmax)
                host = hrt.box_test(form, boxes, rays, 0.001, tmax, on_device=False)
                assert np.array_equal(dev, host), (name, form, tmax, int((dev != host).sum()))
                n_pairs += dev.size
    print("box-test pairs compared device vs host:", n_pairs)
