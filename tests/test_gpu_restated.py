"""The GPU against the independent Python restatement of the path (tests/test_path_restated.py), directly.

The device is held to the CPU oracle everywhere else; the restatement is held to the oracle bit for bit on the CPU.
This closes the triangle on the device itself: pixels of Random, Cornell and Final rendered by the default HIP
kernels (one launch over each pixel, its samples in the frame's chunks) against the restatement's colours, with
the north star's bar (per-pixel L-inf <= 1e-3; the device sums radiance front to back, the reference recursively)
and equal world.hit counts."""
import numpy as np
import pytest

import hrt

import test_path_restated as T

K = T.K
f = np.float32
TOL = 1e-3


def _gpu_pixel(name, W, H, spp, seed, x, y, earth):
    s = hrt.preset(name, 1, earth)
    s.commit()
    cam = hrt.preset_camera(s.info, W, H)
    img, st = hrt.render(s, cam, hrt.params(W, H, spp, 50, seed, tuple(s.info.background)), region=(x, y, 1, 1),
                         stats=True)
    return img[0, 0, :3], int(st.segments), s.info


def _restated(world, info, W, H, spp, seed, x, y, color_fn):
    cam = K.camera(K.F3(info.look_from), K.F3(info.look_at), f(info.fov), f(info.aperture), f(info.focus_dist), W, H)
    bg = K.F3(info.background)
    count = [0]
    total = (f(0), f(0), f(0))
    for s in range(spp):
        T.PATH[0], T.PATH[1] = K.path_key(seed, y * W + x, s), 0
        rng = K.Rng(T.PATH[0])
        u = (f(x) + rng.gen_f32()) / (f(W) - f(1))
        v = (f(y) + rng.gen_f32()) / (f(H) - f(1))
        r = K.camera_ray(cam, u, v, T.random_in_unit_disk(rng), rng.gen_range(float(info.time0), float(info.time1)))
        total = K.add(total, color_fn(world, tuple(r[0:3]), tuple(r[3:6]), r[6], bg, 50, rng, count))
    return np.array([np.sqrt(c * (f(1) / f(spp))) for c in total], np.float32), count[0]


@pytest.mark.gpu
@pytest.mark.parametrize("name,W,H,spp,seed,x,y", [
    ("random", 64, 36, 40, 3, 33, 17),   # 40 spp: two sample chunks of the sphere kernel's schedule
    ("random", 64, 36, 16, 3, 45, 22),
    ("cornell", 40, 40, 24, 5, 20, 10),
    ("final", 40, 40, 4, 7, 3, 15),      # the Earth
    ("final", 40, 40, 4, 7, 18, 18),     # the Perlin sphere
    ("final", 40, 40, 4, 7, 24, 15),     # the blue medium
])
def test_gpu_pixel_equals_independent_restatement(name, W, H, spp, seed, x, y, earth):
    got, segs, info = _gpu_pixel(name, W, H, spp, seed, x, y, earth)
    if name == "random":
        world, fn = T.Bvh(T.SB.random_scene(K.scene_rng(1))), T.ray_color
    elif name == "cornell":
        world, fn = T.cornell_world(), T.ray_color_full
    else:
        world, fn = T.final_world(np.ascontiguousarray(earth, np.uint8)), T.ray_color_final
    want, count = _restated(world, info, W, H, spp, seed, x, y, fn)
    assert segs == count, (segs, count)
    assert float(np.abs(got - want).max()) <= TOL, (got, want)
