"""Measure how far hd_math (the kernel's and the oracle's transcendentals) is from the reference
platform's arithmetic: the reference's f32::{sin, cos, tan, acos, atan2, ln, powf} are glibc's sinf /
cosf / tanf / acosf / atan2f / logf / powf on Linux (this image: glibc 2.35, x86-64).

  python tests/golden/make_libm_report.py      -> tests/golden/libm_report.json

1. Arguments: every transcendental call of single-threaded oracle renders of all scenes is recorded
   (oracle_record_math), so the inputs are the distributions the scenes actually produce.
2. Per function: how many of those calls give different f32 bits in hd_math and glibc, the largest
   difference in ulps, and which of the two is the correctly rounded RN32(float64 libm) value.
3. Frames: the oracle rendered with hd_math vs the same oracle with glibc's functions
   (oracle_set_libm), per scene: L-inf, pixels over 1e-3, ray counts (branch flips change them).
The GPU frame equals the hd_math oracle (tests/test_gpu_parity.py); tests/test_gpu_libm.py compares
it with the glibc oracle on the GPU box, tests/test_libm.py re-measures this report on the CPU.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "hyper-ray-tracer_amd"), ROOT]

import hrt  # noqa: E402
from oracle import oracle as O  # noqa: E402

NAMES = ["sinf", "cosf", "acosf", "atan2f", "logf", "powf(x,5)", "tanf"]
SCENES = ["random", "two_spheres", "two_perlin_spheres", "earth", "simple_light", "cornell", "cornell_smoke", "final",
          "earth_perlin", "random_10k", "features"]
# (scene, W, H, spp): frame comparisons; random 400x225x50 is BASELINE config 1
FRAMES = [("random", 400, 225, 50), ("earth", 200, 112, 16), ("earth_perlin", 200, 112, 16),
          ("two_perlin_spheres", 200, 112, 16), ("simple_light", 200, 112, 16), ("cornell", 100, 100, 16),
          ("cornell_smoke", 100, 100, 16), ("final", 100, 100, 8), ("features", 160, 90, 16)]


def earth():
    return hrt.load_image(os.path.join(ROOT, "tests", "golden", "earthmap_rgb8.png"))


def correctly_rounded(op, x, y):
    xd = x.astype(np.float64)
    with np.errstate(all="ignore"):
        v = {0: np.sin, 1: np.cos, 2: np.arccos, 4: np.log, 6: np.tan}.get(op)
        r = v(xd) if v else (np.arctan2(xd, y.astype(np.float64)) if op == 3 else xd ** 5)
    return r.astype(np.float32)


def function_report(img):
    agg = {k: [] for k in range(O.N_OPS)}
    for name in SCENES:
        rec = O.record_math(lambda: O.OracleScene(hrt.PRESETS[name], 1, img).render(48, 27, 8, 50, seed=1, threads=1),
                            cap=1 << 20)
        for k, (n, a) in rec.items():
            if n:
                agg[k].append(a)
    out = {}
    for k in range(O.N_OPS):
        if not agg[k]:
            continue
        a = np.concatenate(agg[k])
        x, y = a[:, 0].copy(), (a[:, 1].copy() if k == 3 else None)
        h, g, cr = O.math(k, x, y), O.math_libm(k, x, y), correctly_rounded(k, x, y)
        both_nan = np.isnan(h) & np.isnan(g)
        diff = (h.view(np.int32) != g.view(np.int32)) & ~both_nan
        ulp = np.abs(h.view(np.int32).astype(np.int64) - g.view(np.int32).astype(np.int64))
        ok = ~np.isnan(cr)
        out[NAMES[k]] = {"calls": int(x.size), "mismatches": int(diff.sum()), "rate": float(diff.mean()),
                         "max_ulp": int(ulp[diff].max()) if diff.any() else 0,
                         "hd_not_correctly_rounded": int(((h != cr) & ok).sum()),
                         "glibc_not_correctly_rounded": int(((g != cr) & ok).sum())}
    return out


def frame_report(img):
    out = []
    for name, W, H, spp in FRAMES:
        a, ca = O.OracleScene(hrt.PRESETS[name], 1, img).render(W, H, spp, 50, seed=1, threads=8)
        with O.libm_arithmetic():
            b, cb = O.OracleScene(hrt.PRESETS[name], 1, img).render(W, H, spp, 50, seed=1, threads=8)
        d = np.abs(a - b).max(axis=2)
        out.append({"scene": name, "size": [W, H, spp], "linf": float(d.max()), "pixels_over_1e-3": int((d > 1e-3).sum()),
                    "pixels_differing": int((d > 0).sum()), "rays_hd": ca["segments"], "rays_glibc": cb["segments"]})
    return out


def main():
    img = earth()
    rep = {"libm": "glibc 2.35 (Ubuntu 22.04 image), x86-64",
           "functions": function_report(img), "frames": frame_report(img)}
    path = os.path.join(ROOT, "tests", "golden", "libm_report.json")
    with open(path, "w") as fh:
        json.dump(rep, fh, indent=1)
    print(json.dumps(rep, indent=1))


if __name__ == "__main__":
    main()
