"""the walk stream's hierarchy built on the device (hyper-ray-tracer_amd/csrc/build_walk.hip).

The sphere kernel walks a hierarchy re-grouped over the reference's leaf order (scene.cpp walk_regroup,
DESIGN.md section 4).  build_walk.hip makes the same cuts on the GPU (f64 costs in the host's operation
order, the host's tie rule); the host then places and writes the records.  Bar: the walk stream is
byte-identical to the host build's, so the frames are too.  Large scenes (>= 32768 leaves) use the device
build by default (HRT_WALK_BUILD = host | device | auto)."""
import hashlib

import numpy as np
import pytest

import hrt


def _walk_bytes(s):
    buf, info = hrt.scene_blob(s)
    return bytes(buf.raw[info.off_walk:info.off_walk + info.walk_bytes]), info


def _committed(build, monkeypatch, make):
    monkeypatch.setenv("HRT_WALK_BUILD", build)
    monkeypatch.setenv("HRT_WALK_DP", "0")  # the host's greedy split, which the device build mirrors
    s = make()
    s.commit()
    monkeypatch.delenv("HRT_WALK_BUILD")
    return s


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["random", "random_10k"])
def test_device_build_equals_host_build(name, earth, monkeypatch):
    host = _committed("host", monkeypatch, lambda: hrt.preset(name, 1, earth))
    dev = _committed("device", monkeypatch, lambda: hrt.preset(name, 1, earth))
    assert dev.scene_info().walk_device_built == 1 and host.scene_info().walk_device_built == 0
    (a, ia), (b, ib) = _walk_bytes(host), _walk_bytes(dev)
    assert ia.walk_regrouped == ib.walk_regrouped == 1 and ia.walk_hot == ib.walk_hot
    assert ia.walk_c16 == ib.walk_c16 and len(a) == len(b)
    assert hashlib.sha256(a).digest() == hashlib.sha256(b).digest()  # (a bytes diff of a 1 MB stream takes minutes)


def _big_scene(n, seed=5):
    """n spheres of the reference's Random family (static, Lambertian / Metal) scattered over a square,
    under one BvhNode::new, plus the ground sphere: a scene for which the device build is the default."""
    rng = np.random.default_rng(seed)
    s = hrt.Scene()
    ground = s.lambertian(s.checker(s.solid(0.2, 0.3, 0.1), s.solid(0.9, 0.9, 0.9)))
    objs = [s.sphere((0.0, -1000.0, 0.0), 1000.0, ground)]
    side = float(np.sqrt(n)) * 1.2
    xs, zs = rng.uniform(-side / 2, side / 2, n), rng.uniform(-side / 2, side / 2, n)
    rs = rng.uniform(0.1, 0.4, n)
    mats = [s.lambertian(s.solid(*rng.uniform(0, 1, 3))) for _ in range(16)] + \
           [s.metal(rng.uniform(0.5, 1, 3), float(rng.uniform(0, 0.5))) for _ in range(4)] + [s.dielectric(1.5)]
    for i in range(n):
        objs.append(s.sphere((float(xs[i]), float(rs[i]), float(zs[i])), float(rs[i]), mats[i % len(mats)]))
    s.set_root(s.bvh(objs, 0.0, 1.0))
    return s


@pytest.mark.gpu
def test_device_build_large_scene(monkeypatch):
    """100k spheres: the default (device) build equals the host build byte for byte, renders the same
    frame, and the two build times are reported (hrt_scene_info.walk_build_us)."""
    import torch

    n = 100_000
    host = _committed("host", monkeypatch, lambda: _big_scene(n))
    dev = _big_scene(n)
    dev.commit()  # default: >= 32768 leaves -> the device build
    ih, idv = host.scene_info(), dev.scene_info()
    assert idv.walk_device_built == 1 and ih.walk_device_built == 0 and ih.walk_regrouped == 1
    (a, ia), (b, ib) = _walk_bytes(host), _walk_bytes(dev)
    assert hashlib.sha256(a).digest() == hashlib.sha256(b).digest() and ia.walk_hot == ib.walk_hot > 0
    print(f"walk hierarchy of {n + 1} leaves: host build {ih.walk_build_us / 1e3:.1f} ms, "
          f"device build {idv.walk_build_us / 1e3:.1f} ms; stream {ia.walk_bytes / 1e6:.1f} MB, {ia.walk_hot} B in LDS")
    W, H = 96, 54
    cam = hrt.camera((0.0, 40.0, 120.0), (0.0, 0.0, 0.0), 30.0, 0.0, 10.0, 0.0, 1.0, W, H)
    p = hrt.params(W, H, 4, 50, 3)
    imgs = []
    for s in (host, dev):
        d = torch.empty(W * H * 4, dtype=torch.float32, device="cuda")
        st = hrt.render_tiles_device(s, cam, p, [(0, 0, W, H)], d.data_ptr(), 0, want_stats=True)
        imgs.append((d.cpu().numpy(), int(st.segments)))
    assert imgs[0][1] == imgs[1][1] and np.array_equal(imgs[0][0], imgs[1][0])
