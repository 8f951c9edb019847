"""The C-ABI boundary without a GPU: libhrt.so loads, exports every entry point include/hrt/hrt.h
declares, and its host half (scene graph, BvhNode::new, bounding boxes, counts, camera, tile grid,
error codes) behaves like the reference's trait surface (restated by the oracle)."""
import ctypes
import os
import re

import numpy as np
import pytest

import hrt
from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "hrt", "hrt.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(hrt_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    L = hrt.load()
    declared = header_functions()
    assert len(declared) >= 30
    assert sorted(declared) == sorted(hrt.EXPORTS)
    for name in declared:
        assert hasattr(L, name), name
    assert b"gfx950" in L.hrt_version()


def test_library_is_hip_code_object_for_gfx950():
    data = open(hrt.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    assert b"render_kernel" in data


def test_presets_match_oracle_structure(earth):
    for name, pid in hrt.PRESETS.items():
        s = hrt.preset(name, 1, earth)
        o = O.OracleScene(pid, 1, earth)
        assert s.count(s.info.root) == o.count(), name
        bb = s.bounding_box(s.info.root)
        assert np.array_equal(np.array(bb[0] + bb[1], np.float32), o.bbox()), name
        assert np.array_equal(np.array(s.info.look_from, np.float32), o.look_from)
        assert np.array_equal(np.array(s.info.look_at, np.float32), o.look_at)
        assert (s.info.fov, s.info.aperture, s.info.focus_dist) == (o.fov, o.aperture, o.focus_dist)
        assert np.array_equal(np.array(s.info.background, np.float32), o.background)


def test_preset_counts_follow_reference_semantics(earth):
    s = hrt.preset("random", 1, earth)
    assert 480 <= s.count(s.info.root) <= 490          # ~485 over seeds
    assert hrt.preset("cornell", 1, earth).count(hrt.preset("cornell", 1, earth).info.root) == 8  # Rotation::count == 1
    f = hrt.preset("final", 1, earth)
    assert f.count(f.info.root) == 2410                 # 400 cuboids * 6 + 10 (rotated sphere box counts 1)


def test_scene_seed_changes_random_scene(earth):
    a = hrt.preset("random", 1, earth)
    b = hrt.preset("random", 2, earth)
    assert a.bounding_box(a.info.root) != b.bounding_box(b.info.root) or a.count(a.info.root) != b.count(b.info.root)


def test_camera_matches_oracle_bit_for_bit():
    for frm, at, fov, ap, W, H in [((13, 2, 3), (0, 0, 0), 20, 0.1, 1920, 1080), ((278, 278, -800), (278, 278, 0), 40, 0.0, 2048, 2048),
                                   ((26, 3, 6), (0, 2, 0), 20, 0.0, 400, 225)]:
        c = hrt.camera(frm, at, fov, ap, 10.0, 0.0, 1.0, W, H)
        mine = np.array([*c.origin, *c.lower_left_corner, *c.horizontal, *c.vertical, *c.u, *c.v, *c.w, c.lens_radius], np.float32)
        ref = np.zeros(24, np.float32)
        L = O.load()
        f32_from, f32_at = np.array(frm, np.float32), np.array(at, np.float32)
        L.oracle_camera(f32_from.ctypes.data, f32_at.ctypes.data, fov, ap, 10.0, 0.0, 1.0, W, H, ref.ctypes.data)
        assert np.array_equal(mine.view(np.uint32), ref[:22].view(np.uint32))


def test_camera_rejects_empty_shutter():
    with pytest.raises(hrt.HrtError) as e:
        hrt.camera((0, 0, 1), (0, 0, 0), 40, 0, 10, 1.0, 1.0, 10, 10)
    assert e.value.status == hrt.ERR_INVALID_ARG


@pytest.mark.parametrize("W,H,n,last", [(1920, 1080, 24 * 14, (1840, 1040, 80, 40)), (400, 225, 5 * 3, (320, 160, 80, 65)),
                                        (3840, 2160, 48 * 27, (3760, 2080, 80, 80)), (2048, 2048, 26 * 26, (2000, 2000, 48, 48)),
                                        (100, 7, 2, (80, 0, 20, 7))])
def test_tile_grid_matches_reference_layout(W, H, n, last):
    tiles = hrt.tile_grid(W, H, 80)
    assert len(tiles) == n and tiles[-1] == last
    cov = np.zeros((H, W), np.int32)
    for x, y, w, h in tiles:
        cov[y:y + h, x:x + w] += 1
    assert (cov == 1).all()


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_tile_grid_rank_split_is_a_partition(world):
    W, H = 1920, 1080
    allt = hrt.tile_grid(W, H, 80)
    parts = [hrt.tile_grid(W, H, 80, r, world) for r in range(world)]
    assert sorted(t for p in parts for t in p) == sorted(allt)
    sizes = [len(p) for p in parts]
    assert max(sizes) - min(sizes) <= 1


def test_error_codes_and_messages():
    s = hrt.Scene()
    t = s.solid(0.5, 0.5, 0.5)
    m = s.lambertian(t)
    with pytest.raises(hrt.HrtError) as e:
        s.bvh([])
    assert e.value.status == hrt.ERR_EMPTY and "no elements" in str(e.value)
    a = s.sphere((0, 0, 0), 1, m)
    b = s.sphere((1, 0, 0), 1, m)
    lst = s.list([a, b])
    with pytest.raises(hrt.HrtError) as e:   # Box<dyn Hittable> ownership: a child has one parent
        s.list([a])
    assert e.value.status == hrt.ERR_INVALID_ARG
    with pytest.raises(hrt.HrtError):
        s.lambertian(999)
    with pytest.raises(hrt.HrtError):
        s.sphere((0, 0, 0), 1, 999)
    with pytest.raises(hrt.HrtError):
        s.rect(7, 0, 1, 0, 1, 0, m)
    n = s.sphere((0, 0, 0), float("nan"), m)
    with pytest.raises(hrt.HrtError) as e:
        s.bvh([n, s.sphere((0, 0, 0), 1, m)])
    assert e.value.status == hrt.ERR_NAN
    empty = s.list([])
    with pytest.raises(hrt.HrtError) as e:      # a List with no objects has no bounding box
        s.bvh([empty, s.sphere((0, 0, 0), 1, m)])
    assert e.value.status == hrt.ERR_NO_BBOX
    with pytest.raises(hrt.HrtError) as e:
        s.commit()                               # no root yet
    assert e.value.status == hrt.ERR_STATE
    s.set_root(lst)
    assert s.count(lst) == 2


def test_bounding_boxes_follow_reference():
    s = hrt.Scene()
    m = s.lambertian(s.solid(1, 1, 1))
    # rect.rs:97-102: the ZX box spans x in [a0,a1], z in [b0,b1] although the hit test reads a as z
    r = s.rect(hrt.PLANE_ZX, 213, 343, 227, 332, 554, m)
    (mn, mx) = s.bounding_box(r)
    assert mn == (213.0, np.float32(554 - 0.0001), 227.0) and mx == (343.0, np.float32(554 + 0.0001), 332.0)
    ms = s.moving_sphere((0, 0, 0), (1, 2, 3), 0, 1, 0.5, m)
    (mn, mx) = s.bounding_box(ms, 0, 1)
    assert mn == (-0.5, -0.5, -0.5) and mx == (1.5, 2.5, 3.5)
    c = s.cuboid((0, 0, 0), (165, 330, 165), m)
    rot = s.rotate(hrt.AXIS_Y, c, 15.0)
    tr = s.translate(rot, (265, 0, 295))
    assert s.count(tr) == 1                       # rotation.rs:140-142
    (mn, mx) = s.bounding_box(tr)
    assert mn[1] == 0.0 and mx[1] == 330.0 and mn[0] == 265.0 and mx[0] > 265 + 165  # +15 deg about Y widens x
    med = s.constant_medium(s.sphere((0, 0, 0), 2, m), 0.5, s.solid(1, 1, 1))
    assert s.bounding_box(med) == ((-2.0, -2.0, -2.0), (2.0, 2.0, 2.0))


def test_render_without_commit_is_a_state_error():
    s = hrt.preset("two_spheres", 1)
    cam = hrt.preset_camera(s.info, 8, 8)
    with pytest.raises(hrt.HrtError) as e:
        hrt.render(s, cam, hrt.params(8, 8, 1))
    assert e.value.status == hrt.ERR_STATE


def test_device_info_needs_commit():
    s = hrt.preset("random", 1)
    with pytest.raises(hrt.HrtError) as e:
        s.scene_info()
    assert e.value.status == hrt.ERR_STATE


def test_commit_without_a_device_fails_loudly():
    """No CPU fallback: on a host without a GPU the device upload (and so every render) is an error."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    s = hrt.preset("two_spheres", 1)
    with pytest.raises(hrt.HrtError) as e:
        s.commit(0)
    assert e.value.status == hrt.ERR_HIP


def test_progressive_render_argument_errors():
    s = hrt.preset("two_spheres", 1)
    cam = hrt.preset_camera(s.info, 16, 16)
    p = hrt.params(16, 16, 1)
    with pytest.raises(hrt.HrtError) as e:       # not committed
        hrt.render_progressive(s, cam, p, lambda t: None, tile_size=8)
    assert e.value.status == hrt.ERR_STATE
    for kw in ({"tile_size": 0}, {"batch": 0}, {"rank": 2, "world": 2}):
        with pytest.raises(hrt.HrtError) as e:
            hrt.render_progressive(s, cam, p, lambda t: None, **{"tile_size": 8, **kw})
        assert e.value.status == hrt.ERR_INVALID_ARG
