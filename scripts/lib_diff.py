"""Render one preset (optionally rank 0's N-way tile share) with the library HRT_LIB points at and save the
image + ray count under gpurun_out/<tag>.npz; `compare <tagA> <tagB>` lists the pixels that differ.
  HRT_LIB=ab/libhrt_x.so python scripts/lib_diff.py render <tag> <preset> <W> <H> <spp> [share]
  python scripts/lib_diff.py compare <tagA> <tagB>"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hyper-ray-tracer_amd"), ROOT]
import numpy as np  # noqa: E402

OUT = os.path.join(ROOT, "gpurun_out")
if sys.argv[1] == "compare":
    a, b = (np.load(os.path.join(OUT, t + ".npz")) for t in sys.argv[2:4])
    print("rays", int(a["rays"]), int(b["rays"]), "diff", int(a["rays"]) - int(b["rays"]))
    d = np.abs(a["img"] - b["img"]).max(axis=-1)
    ys, xs = np.nonzero(d > 0)
    px = a["px"]
    print(f"{len(ys)} pixels differ, max {float(d.max()) if d.size else 0:.3g}")
    for y, x in list(zip(ys, xs))[:40]:
        print("  pixel", tuple(int(v) for v in px[y, x]), "diff", float(d[y, x]), a["img"][y, x, :3], b["img"][y, x, :3])
    sys.exit(0)
import torch  # noqa: E402
import hrt  # noqa: E402
from hrt import tiling  # noqa: E402

tag, preset, W, H, spp = sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5]), int(sys.argv[6])
share = int(sys.argv[7]) if len(sys.argv) > 7 else 1
s = hrt.preset(preset, 1, None)
s.commit(0)
cam = hrt.preset_camera(s.info, W, H)
p = hrt.params(W, H, spp, 50, 1, tuple(s.info.background))
tiles = [(0, 0, W, H)] if share == 1 else [tuple(t) for t in tiling.split_tiles(W, H, share, 0)]
n = sum(t[2] * t[3] for t in tiles)
out = torch.empty((n, 4), dtype=torch.float32, device="cuda")
import time  # noqa: E402
torch.cuda.synchronize()
t0 = time.perf_counter()
st = hrt.render_tiles_device(s, cam, p, tiles, out.data_ptr(), 0, want_stats=True)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
img = out.cpu().numpy()
px = np.concatenate([np.stack(np.meshgrid(np.arange(x, x + w), np.arange(y, y + h)), -1).reshape(-1, 2) for x, y, w, h in tiles])
os.makedirs(OUT, exist_ok=True)
np.savez(os.path.join(OUT, tag + ".npz"), img=img[None], px=px[None], rays=np.array(st.segments))
print(tag, "rays", st.segments, f"{dt * 1e3:.1f} ms {st.segments / dt / 1e6:.1f} Mrays/s", flush=True)
