"""Locate where two libraries' ray counts differ on rank 0's N-way share of a frame (bit-identity hunts):
  HRT_LIB=A python scripts/ray_bisect.py groups <tag> <preset> <W> <H> <spp> <share> <g>   per-group counts
  python scripts/ray_bisect.py compare <tagA> <tagB> [<out.txt>]       differing entries (their indices to out)
  HRT_LIB=A python scripts/ray_bisect.py tiles <tag> <preset> <W> <H> <spp> <share> <g> <groups.txt>
                                                                          single tiles of the listed groups
Counts go to gpurun_out/<tag>.npz (tiles rendered together in groups of g tiles, in share order)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hyper-ray-tracer_amd"), ROOT]
import numpy as np  # noqa: E402

OUT = os.path.join(ROOT, "gpurun_out")
if sys.argv[1] == "compare":
    a, b = (np.load(os.path.join(OUT, t + ".npz")) for t in sys.argv[2:4])
    d = a["rays"].astype(np.int64) - b["rays"].astype(np.int64)
    idx = np.nonzero(d)[0]
    print("totals", int(a["rays"].sum()), int(b["rays"].sum()), "entries differing", len(idx), flush=True)
    for i in idx[:64]:
        print("  entry", int(a["ids"][i]), "tiles", [tuple(int(v) for v in t) for t in a["tiles"][i] if t[2] > 0][:2],
              "rays", int(a["rays"][i]), int(b["rays"][i]), "diff", int(d[i]), flush=True)
    if len(sys.argv) > 4:
        np.savetxt(sys.argv[4], a["ids"][idx], fmt="%d")
    sys.exit(0)
import torch  # noqa: E402
import hrt  # noqa: E402
from hrt import tiling  # noqa: E402

mode, tag, preset = sys.argv[1], sys.argv[2], sys.argv[3]
W, H, spp, share, g = (int(v) for v in sys.argv[4:9])
s = hrt.preset(preset, 1, None)
s.commit(0)
cam = hrt.preset_camera(s.info, W, H)
p = hrt.params(W, H, spp, 50, 1, tuple(s.info.background))
tiles = [(0, 0, W, H)] if share == 1 else [tuple(t) for t in tiling.split_tiles(W, H, share, 0)]
groups = [tiles[i:i + g] for i in range(0, len(tiles), g)]
if mode == "groups":
    jobs = [(i, grp) for i, grp in enumerate(groups)]
else:
    sel = np.atleast_1d(np.loadtxt(sys.argv[9], dtype=np.int64))
    jobs = [(int(k) * g + j, [t]) for k in sel for j, t in enumerate(groups[int(k)])]
out = torch.empty((sum(t[2] * t[3] for t in max((j[1] for j in jobs), key=len)), 4), dtype=torch.float32, device="cuda")
rays = np.zeros(len(jobs), np.uint64)
tl = np.zeros((len(jobs), g, 4), np.int64)
for n, (i, grp) in enumerate(jobs):
    st = hrt.render_tiles_device(s, cam, p, grp, out.data_ptr(), 0, want_stats=True)
    rays[n] = st.segments
    tl[n, :len(grp)] = grp
    if n % 32 == 0:
        print(tag, mode, n, "of", len(jobs), flush=True)
os.makedirs(OUT, exist_ok=True)
np.savez(os.path.join(OUT, tag + ".npz"), rays=rays, ids=np.array([j[0] for j in jobs]), tiles=tl)
print(tag, "total rays", int(rays.sum()), flush=True)
