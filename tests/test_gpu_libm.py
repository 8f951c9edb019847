"""The GPU frame against the oracle running on the reference platform's arithmetic (glibc's f32
transcendentals, oracle_set_libm): BASELINE config 1 at full size.  See tests/test_libm.py for the
per-function measurement; this is the end-to-end number the north star's bar is on."""
import numpy as np
import pytest

import hrt
from oracle import oracle as O


@pytest.mark.gpu
def test_gpu_config1_vs_glibc_oracle(earth):
    W, H, spp = 400, 225, 50
    s = hrt.preset("random", 1, earth)
    s.commit()
    cam = hrt.preset_camera(s.info, W, H)
    img, st = hrt.render(s, cam, hrt.params(W, H, spp, 50, 1, tuple(s.info.background)), stats=True)
    with O.libm_arithmetic():
        ref, cnt = O.OracleScene(0, 1, earth).render(W, H, spp, 50, seed=1, threads=16)
    d = np.abs(img - ref).max(axis=2)
    print(f"GPU vs glibc-arithmetic oracle, 400x225x50: L-inf {d.max():.3e}, pixels > 1e-3: {(d > 1e-3).sum()}, "
          f"rays {st.segments} vs {cnt['segments']}")
    assert st.segments == cnt["segments"]
    assert d.max() <= 1e-3


@pytest.mark.gpu
@pytest.mark.parametrize("name,W,H,spp", [("earth", 200, 112, 16), ("final", 100, 100, 8)])
def test_gpu_texture_medium_scenes_vs_glibc_oracle(name, W, H, spp, earth):
    """Scenes whose (u, v) / ln arguments do differ by an ulp under glibc: at most the recorded flips."""
    s = hrt.preset(name, 1, earth)
    s.commit()
    cam = hrt.preset_camera(s.info, W, H)
    img, st = hrt.render(s, cam, hrt.params(W, H, spp, 50, 1, tuple(s.info.background)), stats=True)
    with O.libm_arithmetic():
        ref, cnt = O.OracleScene(hrt.PRESETS[name], 1, earth).render(W, H, spp, 50, seed=1, threads=16)
    d = np.abs(img - ref).max(axis=2)
    print(f"{name}: L-inf {d.max():.3e}, pixels > 1e-3: {(d > 1e-3).sum()}, rays {st.segments} vs {cnt['segments']}")
    assert (d > 1e-3).sum() <= 1
    assert abs(int(st.segments) - cnt["segments"]) <= 10


@pytest.mark.gpu
@pytest.mark.parametrize("name,W,H,spp,rows,x0,w", [
    ("earth", 200, 112, 1000, list(range(112)), 0, None),             # the 16-spp frame with the recorded texel flip
    ("earth_perlin", 1920, 1080, 1000, [420, 540, 660], 0, None),     # BASELINE config 3 at its own spp
])
def test_gpu_texture_scenes_full_spp_vs_glibc_oracle(name, W, H, spp, rows, x0, w, earth):
    """At the configs' sample counts a 1-ulp glibc difference in acosf / atan2f (sphere uv) or sinf
    (turbulence) moves one sample's texel or noise value, 1/spp of a pixel: every pixel stays within the
    north star's 1e-3 of the reference platform's arithmetic, with equal ray counts (textures draw no
    random numbers and decide no branch)."""
    import torch

    s = hrt.preset(name, 1, earth)
    s.commit()
    cam = hrt.preset_camera(s.info, W, H)
    ww = W - x0 if w is None else w
    p = hrt.params(W, H, spp, 50, 1, tuple(s.info.background))
    d = torch.empty(len(rows) * ww * 4, dtype=torch.float32, device="cuda")
    st = hrt.render_tiles_device(s, cam, p, [(x0, y, ww, 1) for y in rows], d.data_ptr(), 0, want_stats=True)
    img = d.view(len(rows), ww, 4).cpu().numpy()
    with O.libm_arithmetic():
        ref, cnt = O.OracleScene(hrt.PRESETS[name], 1, earth).render_rows(W, H, spp, rows, 50, seed=1, threads=16,
                                                                         x0=x0, w=ww, task_w=8)
    dd = np.abs(img - ref).max(axis=2)
    print(f"{name} {W}x{H} {spp} spp, {len(rows)} rows vs glibc oracle: L-inf {dd.max():.3e}, "
          f"pixels differing {(dd > 0).sum()}, rays {st.segments} vs {cnt['segments']}")
    assert st.segments == cnt["segments"]
    assert dd.max() <= 1e-3
