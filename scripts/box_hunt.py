"""Find the (pixel, sample) where a library's ray count leaves the oracle's on given tiles (bit-identity hunts;
VERDICT r03 item 1: the general kernel's sub/mul/add box form diverged on three C5 share tiles on the GPU only).

  HRT_LIB=<lib.so> python scripts/box_hunt.py <tag> <preset> <W> <H> <spp> <x,y,w,h> [<x,y,w,h> ...]

For each region: the GPU's and the oracle's ray counts; for a region that differs, per pixel; for a pixel
that differs, per sample (sample_offset = s, one sample).  Results go to gpurun_out/<tag>.json."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hyper-ray-tracer_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import hrt  # noqa: E402
from oracle import oracle as O  # noqa: E402

OUT = os.path.join(ROOT, "gpurun_out")
EARTH = os.path.join(ROOT, "tests", "golden", "earthmap_rgb8.png")


def main():
    tag, preset = sys.argv[1], sys.argv[2]
    W, H, spp = (int(v) for v in sys.argv[3:6])
    regions = [tuple(int(v) for v in a.split(",")) for a in sys.argv[6:]]
    earth = hrt.load_image(EARTH)
    s = hrt.preset(preset, 1, earth)
    s.commit(0)
    cam = hrt.preset_camera(s.info, W, H)
    orc = O.OracleScene(hrt.PRESETS[preset], 1, earth)
    bg = tuple(s.info.background)
    d = torch.empty(max(r[2] * r[3] for r in regions) * 4, dtype=torch.float32, device="cuda")

    def gpu(region, n, off=0):
        p = hrt.params(W, H, n, 50, 1, bg, sample_offset=off)
        return int(hrt.render_tiles_device(s, cam, p, [region], d.data_ptr(), 0, want_stats=True).segments)

    def cpu(region, n, off=0):
        _, cnt = orc.render(W, H, n, 50, seed=1, region=region, threads=16, sample_offset=off)
        return int(cnt["segments"])

    res = {"lib": hrt.LIB_PATH, "preset": preset, "W": W, "H": H, "spp": spp, "regions": []}
    t0 = time.time()
    for reg in regions:
        g, c = gpu(reg, spp), cpu(reg, spp)
        ent = {"region": reg, "gpu": g, "oracle": c, "pixels": []}
        print(tag, "region", reg, "gpu", g, "oracle", c, "diff", g - c, f"{time.time() - t0:.1f}s", flush=True)
        if g != c:
            x0, y0, w, h = reg
            for y in range(y0, y0 + h):
                for x in range(x0, x0 + w):
                    gp, cp = gpu((x, y, 1, 1), spp), cpu((x, y, 1, 1), spp)
                    if gp == cp:
                        continue
                    pix = {"x": x, "y": y, "gpu": gp, "oracle": cp, "samples": []}
                    print(tag, " pixel", (x, y), "gpu", gp, "oracle", cp, flush=True)
                    # bisect the sample range (counts are sums over samples)
                    todo = [(0, spp)]
                    while todo:
                        a, b = todo.pop()
                        if gpu((x, y, 1, 1), b - a, a) == cpu((x, y, 1, 1), b - a, a):
                            continue
                        if b - a == 1:
                            pix["samples"].append({"sample": a, "gpu": gpu((x, y, 1, 1), 1, a),
                                                   "oracle": cpu((x, y, 1, 1), 1, a)})
                            print(tag, "   sample", pix["samples"][-1], flush=True)
                            continue
                        m = (a + b) // 2
                        todo += [(m, b), (a, m)]
                    ent["pixels"].append(pix)
        res["regions"].append(ent)
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, tag + ".json"), "w") as f:
        json.dump(res, f, indent=1)
    print(tag, "done", f"{time.time() - t0:.1f}s", flush=True)


if __name__ == "__main__":
    main()
