"""Compare traversal modes on one frame: exact reference (flags 8), slab on the reference tree (4),
SAH streams (0).  Prints ray counts and the pixels that differ, and checks a few of them against the
CPU oracle (which implements the exact reference)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hyper-ray-tracer_amd"), ROOT]
import numpy as np, torch, hrt
from oracle import oracle as O
preset = sys.argv[1] if len(sys.argv) > 1 else "random"
W, H, spp = 1920, 1080, int(sys.argv[2]) if len(sys.argv) > 2 else 32
modes = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [8, 4, 0]
check_oracle = len(sys.argv) > 4
s = hrt.preset(preset, 1); s.commit(0)
cam = hrt.preset_camera(s.info, W, H)
imgs, segs = {}, {}
import time
for fl in modes:
    p = hrt.params(W, H, spp, 50, 1, tuple(s.info.background), flags=fl)
    t0 = time.perf_counter()
    img, st = hrt.render(s, cam, p, stats=True)
    dt = time.perf_counter() - t0
    imgs[fl], segs[fl] = img, st.segments
    print("flags", fl, "segments", st.segments, f"{dt:.2f}s {st.segments/dt/1e6:.0f} Mrays/s", flush=True)
o = O.OracleScene(hrt.PRESETS[preset], 1)
for fl in modes[1:]:
    d = np.abs(imgs[fl] - imgs[modes[0]]).max(axis=2)
    ys, xs = np.nonzero(d > 0)
    print(f"flags {fl} vs exact: {len(ys)} pixels differ, max {d.max():.3g}", flush=True)
    print("   first pixels (x,y,diff):", [(int(x), int(y), float(d[y, x])) for y, x in list(zip(ys, xs))[:8]], flush=True)
    for y, x in (list(zip(ys, xs))[:4] if check_oracle else []):
        ref, cnt = o.render(W, H, spp, 50, seed=1, region=(int(x), int(y), 1, 1), threads=1)
        print(f"   pixel ({x},{y}): exact {imgs[modes[0]][y,x,:3]} mode {imgs[fl][y,x,:3]} oracle {ref[0,0,:3]}", flush=True)
