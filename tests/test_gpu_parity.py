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

# (preset, width, height, spp, depth): every scene feature of the reference; spp > 16 on sphere scenes
# and spp > 32 on general ones exercises the sample-chunk split (chunk sums reduced in a fixed order).
# earth_perlin, random_10k, features and motion are BUILD-DEFINED scenes (no reference builder): the oracle
# builds them with the same generator as the library, so their cases check the kernels against the
# restatement of the reference's per-object code, and no reference fixture covers them (parity unpinned,
# like every scene here: the reference has no fixtures at all).  The per-sphere shutter
# path of `motion` (the ray's time in TRay.tau) is also held to the uniform-motion path of the reference
# scenes indirectly: Random's moving spheres run the scene-wide factor, `motion` the per-sphere one.
CASES = [
    ("random", 40, 24, 100, 50),
    ("cornell", 24, 24, 70, 50),
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
    ("motion", 64, 36, 16, 50),          # per-sphere shutter intervals: no scene-wide motion factor
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
    full, st_full, _ = _gpu_render("random", 64, 36, 8, 3, 11, earth)
    part, st_part, _ = _gpu_render("random", 64, 36, 8, 3, 11, earth, region=(10, 5, 20, 17))
    assert st_full.pixels == 64 * 36 and st_part.pixels == 20 * 17, (st_full.pixels, st_part.pixels)
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


def _rust_cast(x, signed):
    """Rust's saturating `x as i32` / `x as u32` (truncation toward zero, NaN -> 0, clamped), in float64."""
    lo, hi = (-2.0 ** 31, 2.0 ** 31 - 1) if signed else (0.0, 2.0 ** 32 - 1)
    t = np.trunc(np.nan_to_num(x.astype(np.float64), nan=0.0, posinf=hi, neginf=lo))
    return np.clip(t, lo, hi).astype(np.int64).astype(np.int32 if signed else np.uint32)


@pytest.mark.gpu
def test_device_float_to_int_casts():
    """hd_math sat_f2i32 / sat_f2u32 on the device (v_cvt_i32_f32 / v_cvt_u32_f32, HRT_HW_CVT) equal Rust's
    saturating casts on every edge: NaNs of both signs and payloads, infinities, the limits of the range and
    their neighbours, signed zeros, values just below and above integers, denormals, and random values of
    every exponent (the Perlin lattice `floor(p) as i32`, perlin_noise.rs:86-88; the image texel
    `(u * w) as u32`, image_texture.rs)."""
    rng = np.random.default_rng(5)
    edge = np.array([0.0, -0.0, 0.5, -0.5, 0.9999999, -0.9999999, 1.0, -1.0, 1.5, -1.5, 2.5, -2.5, 255.99998,
                     2.0 ** 31, -2.0 ** 31, 2.0 ** 32, -2.0 ** 32, 3e38, -3e38, np.inf, -np.inf, np.nan, -np.nan,
                     1e-45, -1e-45, 1.17e-38, 16777217.0, 8388607.5], np.float32)
    near = np.array([2.0 ** 31, 2.0 ** 32, 2.0 ** 24, 1.0], np.float32)
    neigh = np.concatenate([np.nextafter(near, np.float32(np.inf)), np.nextafter(near, np.float32(-np.inf))])
    nans = np.array([0x7fc00000, 0xffc00000, 0x7f800001, 0xff812345, 0x7fffffff], np.uint32).view(np.float32)
    rand = (rng.uniform(-1, 1, 300000) * 2.0 ** rng.uniform(-30, 40, 300000)).astype(np.float32)
    bits = rng.integers(0, 2 ** 32, 100000, dtype=np.uint64).astype(np.uint32).view(np.float32)
    x = np.concatenate([edge, neigh, -neigh, nans, rand, bits])
    with np.errstate(invalid="ignore"):
        for op, signed in ((8, True), (9, False)):
            d = hrt.device_math(op, x).view(np.int32 if signed else np.uint32)
            want = _rust_cast(x, signed)
            bad = np.flatnonzero(d != want)
            assert bad.size == 0, (op, x[bad[:5]], d[bad[:5]], want[bad[:5]])


@pytest.mark.gpu
def test_repeated_calls_on_two_streams(earth):
    """Many back-to-back tile renders on two HIP streams (scratch-slot reuse) all match a single
    full-frame render: the per-pixel RNG keys make tiles independent of call order and stream."""
    import torch

    s = hrt.preset("random", 1, earth)
    s.commit()
    W, H = 96, 54
    cam = hrt.preset_camera(s.info, W, H)
    p = hrt.params(W, H, 4, 8, 5, tuple(s.info.background))
    full = hrt.render(s, cam, p)
    tiles = hrt.tile_grid(W, H, 16)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = []
    for rep in range(3):
        for i, t in enumerate(tiles):
            d = torch.full((t[3], t[2], 4), -7.0, device="cuda")
            st = streams[(i + rep) % 2]
            st.wait_stream(torch.cuda.current_stream())
            hrt.render_tiles_device(s, cam, p, [t], d.data_ptr(), st.cuda_stream)
            outs.append((t, d, st))
    torch.cuda.synchronize()
    for t, d, _ in outs:
        x, y, w, h = t
        assert np.array_equal(d.cpu().numpy(), full[y:y + h, x:x + w]), t


@pytest.mark.gpu
def test_multi_tile_call_matches_full_frame(earth):
    """One call over a rank's interleaved tile subset (the multi-GPU split) packs tiles back to back
    and reproduces the full-frame pixels bit for bit, for every rank of a 3-way split."""
    import torch

    s = hrt.preset("random", 1, earth)
    s.commit()
    W, H = 200, 90
    cam = hrt.preset_camera(s.info, W, H)
    p = hrt.params(W, H, 4, 8, 9, tuple(s.info.background))
    full = hrt.render(s, cam, p)
    covered = np.zeros((H, W), bool)
    for rank in range(3):
        tiles = hrt.tile_grid(W, H, 80, rank, 3)
        n = sum(t[2] * t[3] for t in tiles)
        d = torch.zeros(n * 4, device="cuda")
        st = hrt.render_tiles_device(s, cam, p, tiles, d.data_ptr(), 0, want_stats=True)
        assert st.pixels == n
        flat = d.cpu().numpy()
        off = 0
        for x, y, w, h in tiles:
            blk = flat[off * 4:(off + w * h) * 4].reshape(h, w, 4)
            assert np.array_equal(blk, full[y:y + h, x:x + w])
            covered[y:y + h, x:x + w] = True
            off += w * h
    assert covered.all()


# The verbatim reference traversal (HRT_RENDER_REFERENCE_CULL: aabb.rs's per-axis test alone) is
# checked against the oracle above; the default EXACT culling must give the same bits as it at sizes
# the oracle cannot reach.
EXACT_CASES = [
    ("random", 320, 180, 16), ("two_spheres", 320, 180, 16), ("two_perlin_spheres", 320, 180, 16),
    ("earth", 320, 180, 16), ("simple_light", 320, 180, 16), ("cornell", 256, 256, 16),
    ("cornell_smoke", 256, 256, 16), ("final", 200, 200, 8), ("earth_perlin", 320, 180, 16),
    ("random_10k", 320, 180, 8), ("features", 320, 180, 16),
]


@pytest.mark.gpu
@pytest.mark.parametrize("name,w,h,spp", EXACT_CASES)
def test_exact_culling_bit_identical_to_reference_traversal(name, w, h, spp, earth):
    s = hrt.preset(name, 1, earth)
    s.commit()
    cam = hrt.preset_camera(s.info, w, h)
    bg = tuple(s.info.background)
    ref, st_ref = hrt.render(s, cam, hrt.params(w, h, spp, 50, 13, bg, flags=hrt.RENDER_REFERENCE_CULL), stats=True)
    ex, st_ex = hrt.render(s, cam, hrt.params(w, h, spp, 50, 13, bg), stats=True)
    assert st_ex.segments == st_ref.segments
    assert np.array_equal(ex, ref)


@pytest.mark.gpu
def test_headline_frame_exact_equals_reference_traversal(earth):
    """BASELINE config 2 at full size: 1920x1080, 500 spp, depth 50 (2.9 G rays): the default path is
    bit-identical to the verbatim reference traversal; properties: finite, alpha 1, deterministic."""
    s = hrt.preset("random", 1, earth)
    s.commit()
    W, H = 1920, 1080
    cam = hrt.preset_camera(s.info, W, H)
    bg = tuple(s.info.background)
    ex, st = hrt.render(s, cam, hrt.params(W, H, 500, 50, 1, bg), stats=True)
    ref, st_ref = hrt.render(s, cam, hrt.params(W, H, 500, 50, 1, bg, flags=hrt.RENDER_REFERENCE_CULL), stats=True)
    assert st.samples == W * H * 500 and st.pixels == W * H
    assert st.segments == st_ref.segments
    assert np.array_equal(ex, ref)
    assert np.isfinite(ex).all() and (ex[..., 3] == 1).all()
    again = hrt.render(s, cam, hrt.params(W, H, 500, 50, 1, bg))
    assert np.array_equal(again, ex)


def _has_gpu():
    import torch

    return torch.cuda.is_available()


@pytest.mark.gpu
@pytest.mark.skipif(not _has_gpu(), reason="needs a GPU")
@pytest.mark.parametrize("name,w,h,spp", [("cornell", 40, 40, 16), ("cornell_smoke", 40, 40, 16), ("final", 40, 40, 8),
                                          ("features", 64, 36, 16), ("earth_perlin", 48, 27, 16), ("simple_light", 48, 27, 16)])
def test_general_kernels_are_bit_identical(earth, monkeypatch, name, w, h, spp):
    """The default general-scene kernel, render_gwalk_kernel (the general walk stream: persistent walks,
    batched leaf programs), against the segment-at-a-time kernel (HRT_KERNEL=segment) and render_full_kernel
    (HRT_KERNEL=persistent): the per-lane code is shared (csrc/lane.h, host-checked by
    tests/test_lane_sim.py), so the images must be identical bit for bit.  The default is the walk-stream
    kernel: only it and the sphere kernel run batched leaf blocks (prim_slots > 0)."""
    s = hrt.preset(name, 1, earth)
    s.commit()
    cam = hrt.preset_camera(s.info, w, h)
    p = hrt.params(w, h, spp, 50, 7, tuple(s.info.background))
    a, sa = hrt.render(s, cam, p, stats=True)
    pc = hrt.params(w, h, spp, 50, 7, tuple(s.info.background), flags=hrt.RENDER_COUNT_WORK)
    c, sc = hrt.render(s, cam, pc, stats=True)
    packet = "PACKET = true" in hrt.last_launch()["kernel"]
    assert packet or name not in ("cornell_smoke", "earth_perlin"), hrt.last_launch()["kernel"]
    assert (sc.prim_slots > 0 or packet) and np.array_equal(a, c)
    if packet:  # the per-lane walk of the same kernel (A/B knobs): the same frame
        for k in ("HRT_GWALK_PACKET", "HRT_SPHERE_PACKET"):
            monkeypatch.setenv(k, "0")
        d, sd = hrt.render(s, cam, p, stats=True)
        assert "PACKET = false" in hrt.last_launch()["kernel"]
        assert sd.segments == sa.segments and np.array_equal(a, d)
        for k in ("HRT_GWALK_PACKET", "HRT_SPHERE_PACKET"):
            monkeypatch.delenv(k)
    for kernel in ("segment", "persistent"):
        monkeypatch.setenv("HRT_KERNEL", kernel)
        b, sb = hrt.render(s, cam, p, stats=True)
        assert sa.segments == sb.segments, kernel
        assert np.array_equal(a, b), kernel
        monkeypatch.delenv("HRT_KERNEL")


@pytest.mark.gpu
@pytest.mark.parametrize("name,W,H,spp", [("cornell", 96, 80, 70), ("final", 64, 48, 40)])
def test_general_walk_kernel_tiles_and_chunks(earth, monkeypatch, name, W, H, spp):
    """render_gwalk_kernel on a multi-tile call (ragged 16-px tiles of a 3-way split, packed back to back)
    and with sample chunks (spp > 32: several chunk sums per pixel): every share equals the whole frame's
    pixels, and the frame equals the segment kernel's."""
    import torch

    from hrt import tiling

    s = hrt.preset(name, 1, earth)
    s.commit()
    cam = hrt.preset_camera(s.info, W, H)
    p = hrt.params(W, H, spp, 50, 5, tuple(s.info.background))
    full, st = hrt.render(s, cam, p, stats=True)
    frame = np.full((H, W, 4), np.nan, np.float32)
    segs = 0
    for r in range(3):
        t = tiling.split_tiles(W, H, 3, r)
        d = torch.empty(tiling.share_pixels(t) * 4, dtype=torch.float32, device="cuda")
        sr = hrt.render_tiles_device(s, cam, p, t, d.data_ptr(), 0, want_stats=True)
        segs += int(sr.segments)
        tiling.place_tiles(frame, t, d.cpu().numpy())
    assert segs == st.segments and np.array_equal(frame, full)
    monkeypatch.setenv("HRT_KERNEL", "segment")
    seg, ss = hrt.render(s, cam, p, stats=True)
    assert ss.segments == st.segments and np.array_equal(seg, full)


@pytest.mark.gpu
def test_general_walk_watchdog(earth):
    """Corrupt skip links in the general walk stream (every inner record's fail link -> the root) make walks
    loop; render_gwalk_kernel's watchdog stops them and the frame is reported HRT_ERR_STATE."""
    s = hrt.preset("final", 1, earth)
    s.commit()
    W, H = 48, 32
    cam = hrt.preset_camera(s.info, W, H)
    p = hrt.params(W, H, 2, 50, 3, tuple(s.info.background))
    hrt.render(s, cam, p)  # intact scene first
    buf, info = hrt.scene_blob(s)
    assert info.walk_bytes > 0
    ws = np.frombuffer(buf.raw, np.uint32, count=info.walk_bytes // 4, offset=info.off_walk).copy()
    off, inner = 0, 0
    while off < info.walk_bytes:  # pre-order over the node parts by their links (records may be placed apart)
        link, skip = int(ws[off // 4 + 7]), int(ws[off // 4 + 3])
        if link & 0x80000000:  # a leaf: its pass link is its payload; the walk goes on at its skip link
            off = skip
        else:
            ws[off // 4 + 3] = 0
            inner += 1
            off = link
    assert inner > 100
    s.poke_blob(info.off_walk, ws.tobytes())
    with pytest.raises(hrt.HrtError) as e:
        hrt.render(s, cam, p)
    assert e.value.status == hrt.ERR_STATE


@pytest.mark.gpu
@pytest.mark.skipif(not _has_gpu(), reason="needs a GPU")
@pytest.mark.parametrize("batch,world", [(1, 1), (5, 1), (64, 1), (3, 2)])
def test_progressive_tiles_assemble_the_frame(earth, batch, world):
    """hrt_render_progressive: every tile of the grid arrives once, in grid order, with
    the pixels hrt_render gives for the whole frame."""
    W, H, T = 200, 130, 40
    s = hrt.preset("random", 1, earth)
    s.commit()
    cam = hrt.preset_camera(s.info, W, H)
    p = hrt.params(W, H, 8, 50, 3, tuple(s.info.background))
    full = hrt.render(s, cam, p)
    frame = np.full((H, W, 4), np.nan, np.float32)
    seen = []
    for rank in range(world):
        def on_tile(t):
            seen.append((t.x, t.y))
            x0, y0 = t.x * T, t.y * T
            assert np.isnan(frame[y0:y0 + t.height, x0:x0 + t.width]).all()
            frame[y0:y0 + t.height, x0:x0 + t.width] = t.pixels
        st = hrt.render_progressive(s, cam, p, on_tile, tile_size=T, rank=rank, world=world, batch=batch, stats=True)
        assert st.samples == sum(t[2] * t[3] for t in hrt.tile_grid(W, H, T, rank, world)) * 8
    assert len(seen) == len(set(seen)) == len(hrt.tile_grid(W, H, T))
    assert np.array_equal(frame, full)


@pytest.mark.gpu
def test_watchdog_reports_a_killed_frame_without_stats(earth):
    """Corrupt skip links (box nodes' fail links pointing back to the root) make walks loop; the
    watchdog stops them, and the frame is reported HRT_ERR_STATE although the launch asked for no stats:
    by hrt_scene_synchronize, and by the call that next reuses the launch's scratch slot."""
    import torch

    s = hrt.preset("random", 1, earth)
    s.commit()
    W, H = 64, 36
    cam = hrt.preset_camera(s.info, W, H)
    p = hrt.params(W, H, 2, 50, 3, tuple(s.info.background))
    ok, st = hrt.render(s, cam, p, stats=True)  # intact scene first
    assert st.pixels == W * H
    # every box node's fail link (dword 3) -> node 0: a ray that fails any box below the root walks
    # back to the root and repeats the same walk for ever (a single corrupt link is not enough: the
    # root's children contain the ground sphere's huge box, which nearly every ray passes)
    buf, info = hrt.scene_blob(s)
    nodes = np.frombuffer(buf.raw, np.uint32, count=8 * info.n_nodes, offset=info.off_nodes).reshape(-1, 8).copy()
    boxed = ((nodes[:, 7] >> 24) & 0x7F) <= 1  # K_BOX, K_BOX_PRIM (layout.h)
    assert boxed.sum() > 100
    nodes[boxed, 3] = 0
    s.poke_blob(info.off_nodes, nodes.tobytes())
    # the sphere kernel's walk stream (layout.h): every inner record's skip link -> offset 0 (the root)
    assert info.walk_bytes > 0
    ws = np.frombuffer(buf.raw, np.uint32, count=info.walk_bytes // 4, offset=info.off_walk).copy()
    off, inner = 0, 0
    while off < info.walk_bytes:
        leaf = (ws[off // 4 + 7] & 0x80000000) != 0  # pass link with WALK_PEND: a leaf, its payload follows
        if not leaf:
            ws[off // 4 + 3] = 0
            inner += 1
        off += 128 if leaf else 32  # layout.h WALK_NODE_BYTES (+ WALK_PAYLOAD_BYTES)
    assert inner > 100
    s.poke_blob(info.off_walk, ws.tobytes())
    d = torch.zeros(W * H * 4, device="cuda")
    hrt.render_tiles_device(s, cam, p, [(0, 0, W, H)], d.data_ptr(), 0)  # no stats: returns at once
    with pytest.raises(hrt.HrtError) as e:
        s.synchronize()
    assert e.value.status == hrt.ERR_STATE and "did not terminate" in str(e.value)
    s.synchronize()  # reported once
    for _ in range(4):  # fill the slots; the 5th call reuses the first slot and finds its error
        try:
            hrt.render_tiles_device(s, cam, p, [(0, 0, W, H)], d.data_ptr(), 0)
        except hrt.HrtError as err:
            assert err.status == hrt.ERR_STATE
            break
    else:
        with pytest.raises(hrt.HrtError) as e:
            hrt.render_tiles_device(s, cam, p, [(0, 0, W, H)], d.data_ptr(), 0)
        assert e.value.status == hrt.ERR_STATE
    with pytest.raises(hrt.HrtError) as e:  # a synchronous call reports its own launch
        hrt.render(s, cam, p)
    assert e.value.status == hrt.ERR_STATE


@pytest.mark.gpu
def test_image_size_range_is_enforced(earth):
    """2 <= width, height <= 65535 (the camera divisions' proven domain, lane.h start_sample)."""
    s = hrt.preset("random", 1, earth)
    s.commit()
    for W, H in [(1, 8), (8, 1), (65536, 8), (8, 65536)]:
        cam = hrt.preset_camera(s.info, max(W, 2), max(H, 2))
        with pytest.raises(hrt.HrtError) as e:
            hrt.render(s, cam, hrt.params(W, H, 1, 4, 1), region=(0, 0, 1, 1))
        assert e.value.status == hrt.ERR_INVALID_ARG
        with pytest.raises(hrt.HrtError) as e:
            hrt.trace_path(s, cam, hrt.params(W, H, 1, 4, 1), 0, 0, 0)
        assert e.value.status == hrt.ERR_INVALID_ARG
    cam = hrt.preset_camera(s.info, 2, 2)
    img = hrt.render(s, cam, hrt.params(2, 2, 2, 4, 1, tuple(s.info.background)))
    ref, _ = O.OracleScene(0, 1, earth).render(2, 2, 2, 4, seed=1)
    assert np.abs(img - ref).max() <= TOL
    cam = hrt.preset_camera(s.info, 65535, 2)
    img = hrt.render(s, cam, hrt.params(65535, 2, 1, 4, 1, tuple(s.info.background)), region=(65000, 0, 16, 2))
    ref, _ = O.OracleScene(0, 1, earth).render(65535, 2, 1, 4, seed=1, region=(65000, 0, 16, 2))
    assert np.abs(img - ref).max() <= TOL


@pytest.mark.gpu
def test_hrt_render_tile_by_tile(earth):
    """INTEGRATION.md section 3's simple loop: one synchronous hrt_render per 80x80 tile (its device
    output buffer comes from the scene's pool, not a hipMalloc per call) reassembles the whole-frame
    render bit for bit, buffers of different sizes included."""
    s = hrt.preset("random", 1, earth)
    s.commit()
    W, H = 400, 225
    cam = hrt.preset_camera(s.info, W, H)
    p = hrt.params(W, H, 4, 50, 2, tuple(s.info.background))
    full = hrt.render(s, cam, p)
    frame = np.full((H, W, 4), np.nan, np.float32)
    for x, y, w, h in hrt.tile_grid(W, H, 80):
        frame[y:y + h, x:x + w] = hrt.render(s, cam, p, region=(x, y, w, h))
    assert np.array_equal(frame, full)


@pytest.mark.gpu
def test_split_node_parts_render_the_same_frame(earth, monkeypatch):
    """layout.h WALK_SPLIT_HALF (opt-in HRT_WALK_SPLIT=1): the sphere kernel's SPLIT instantiation reads each node
    part's halves 16 KB apart; the frame and ray count equal the default 32-B parts' bit for bit."""
    a, sa, s0 = _gpu_render("random", 160, 90, 16, 50, 3, earth)
    assert hrt.scene_blob(s0)[1].walk_half == 16
    monkeypatch.setenv("HRT_WALK_SPLIT", "1")
    b, sb, s1 = _gpu_render("random", 160, 90, 16, 50, 3, earth)
    assert hrt.scene_blob(s1)[1].walk_half == 16384
    assert sa.segments == sb.segments and np.array_equal(a, b)


@pytest.mark.gpu
def test_hybrid_split_node_parts_render_the_same_frame(earth, monkeypatch):
    """layout.h WALK_SPLIT_HALF_HYB (opt-in HRT_WALK_SPLIT=1): the hybrid sphere walk (random-10k) over node parts in
    8-KB-split pages, LDS and buffer reads alike, renders the default 32-B layout's frame and rays bit for bit."""
    def render():
        import torch

        s = hrt.preset("random_10k", 1, earth)
        cam = hrt.preset_camera(s.info, 384, 216)
        s.set_view(cam)
        s.commit()
        p = hrt.params(384, 216, 16, 50, 3, tuple(s.info.background))
        d = torch.empty(384 * 216 * 4, dtype=torch.float32, device="cuda")
        st = hrt.render_tiles_device(s, cam, p, [(0, 0, 384, 216)], d.data_ptr(), 0, want_stats=True)
        return d.cpu().numpy(), st, hrt.scene_blob(s)[1], hrt.last_launch()["kernel"]
    a, sa, ia, ka = render()
    monkeypatch.setenv("HRT_WALK_SPLIT", "1")
    b, sb, ib, kb = render()
    assert ia.walk_half == 16 and ib.walk_half == 8192 and ib.walk_hot > 0
    assert "HYB = true" in kb and "SPLIT = true" in kb, kb
    assert sa.segments == sb.segments and np.array_equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("knob", ["HRT_GWALK_MED=0", "HRT_GWALK_BIG=0", "HRT_GWALK_TRIMP=0"])
def test_final_walk_variants_are_bit_identical(earth, monkeypatch, knob):
    """Final through the general walk kernel's r04 variants against the default (flat one-sphere media
    GL_MED, the 152-KB staged set of one 1024-thread workgroup, the TRIM_PROGRAMS instantiation): each knob
    switches one back (the scene is committed under it: placement knobs act at commit), and the frame and
    its ray count stay bit for bit the default's."""
    w, h, spp = 96, 64, 24
    s = hrt.preset("final", 1, earth)
    s.commit()
    cam = hrt.preset_camera(s.info, w, h)
    p = hrt.params(w, h, spp, 50, 5, tuple(s.info.background))
    a, sa = hrt.render(s, cam, p, stats=True)
    k0 = hrt.last_launch()["kernel"]
    assert "BIG = true" in k0 and "TRIM = 4" in k0, k0
    k, v = knob.split("=")
    monkeypatch.setenv(k, v)
    s2 = hrt.preset("final", 1, earth)
    s2.commit()
    b, sb = hrt.render(s2, cam, p, stats=True)
    assert sa.segments == sb.segments and np.array_equal(a, b), knob
    # the launch reports the A/B knob, as read at the launch and at the scene's commit
    assert hrt.last_launch()["knobs"].split(";") == [knob, "commit:" + knob], hrt.last_launch()["knobs"]


@pytest.mark.gpu
def test_commit_knob_is_reported_after_it_is_unset(earth, monkeypatch):
    """a placement knob set while the scene is committed and unset before the launch still shows in
    the launch's record (hrt_launch_info.knobs, "commit:NAME=value"), so bench.py refuses such a line."""
    w, h, spp = 48, 32, 4
    monkeypatch.setenv("HRT_GWALK_BIG", "0")
    s = hrt.preset("final", 1, earth)
    s.commit()
    monkeypatch.delenv("HRT_GWALK_BIG")
    cam = hrt.preset_camera(s.info, w, h)
    hrt.render(s, cam, hrt.params(w, h, spp, 50, 5, tuple(s.info.background)))
    assert hrt.last_launch()["knobs"] == "commit:HRT_GWALK_BIG=0"
    s2 = hrt.preset("final", 1, earth)
    s2.commit()
    hrt.render(s2, cam, hrt.params(w, h, spp, 50, 5, tuple(s2.info.background)))
    assert hrt.last_launch()["knobs"] == ""


@pytest.mark.gpu
@pytest.mark.parametrize("spp", [24, 1, 65])
def test_final_one_sample_chunks_equal_the_chunk_loop(earth, monkeypatch, spp):
    """render_gwalk_kernel's ONE instantiation (every chunk one sample: Final up to 64 spp; no work item or
    running sum kept across the walk and shading) against the general chunk loop on the same schedule
    (HRT_GWALK_ONE=0): the same pixels bit for bit, the same ray, sample and pixel counts.  spp 1 writes the
    frame directly (one chunk); at 65 spp the schedule has 2-sample chunks and ONE is not chosen."""
    w, h = 80, 48
    s = hrt.preset("final", 1, earth)
    s.commit()
    cam = hrt.preset_camera(s.info, w, h)
    p = hrt.params(w, h, spp, 50, 3, tuple(s.info.background))
    a, sa = hrt.render(s, cam, p, stats=True)
    ka = hrt.last_launch()["kernel"]
    assert ("ONE = true" in ka) == (spp <= 64), ka
    monkeypatch.setenv("HRT_GWALK_ONE", "0")
    b, sb = hrt.render(s, cam, p, stats=True)
    kb = hrt.last_launch()["kernel"]
    assert "ONE = false" in kb, kb
    assert (sa.segments, sa.samples, sa.pixels) == (sb.segments, sb.samples, sb.pixels)
    assert sa.pixels == w * h and sa.samples == w * h * spp
    assert np.array_equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("name,w,h,spp", [("random", 64, 36, 100), ("cornell", 48, 48, 150)])
def test_env_chunk_knobs_do_not_change_frame(earth, monkeypatch, name, w, h, spp):
    """the r04 environment knobs that regrouped each pixel's sum (HRT_CHUNK_MIN / DIV /
    TAIL) are no longer read: with them set the default ABI renders the same bits and reports no knob.  The
    explicit option (hrt_scene_options.chunk_min) does regroup the sums: same rays, a different summation
    order (within the parity bar of the oracle, not bit-identical)."""
    s = hrt.preset(name, 1, earth)
    s.commit()
    cam = hrt.preset_camera(s.info, w, h)
    p = hrt.params(w, h, spp, 50, 9, tuple(s.info.background))
    a, sa = hrt.render(s, cam, p, stats=True)
    for k, v in (("HRT_CHUNK_MIN", "1"), ("HRT_CHUNK_DIV", "512"), ("HRT_CHUNK_TAIL", "0")):
        monkeypatch.setenv(k, v)
    b, sb = hrt.render(s, cam, p, stats=True)
    assert sa.segments == sb.segments and np.array_equal(a, b)
    assert hrt.last_launch()["knobs"] == ""
    s2 = hrt.preset(name, 1, earth, options={"chunk_min": 1, "chunk_max": 512, "chunk_uniform": 1})
    assert hrt.sample_chunks(s2, p) != hrt.sample_chunks(s, p)
    s2.commit()
    c, sc = hrt.render(s2, cam, p, stats=True)
    assert sc.segments == sa.segments and float(np.abs(c - a).max()) <= 1e-5
