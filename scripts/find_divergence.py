"""Locate the sample whose path differs between two traversal modes at one pixel and print both
paths segment by segment (device traces)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hyper-ray-tracer_amd"), ROOT]
import numpy as np, hrt
preset, x, y, spp = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
fa, fb = int(sys.argv[5]), int(sys.argv[6])
W, H = 1920, 1080
if len(sys.argv) > 7:
    W, H = int(sys.argv[7]), int(sys.argv[8])
s = hrt.preset(preset, 1); s.commit(0)
cam = hrt.preset_camera(s.info, W, H)
pa = hrt.params(W, H, spp, 50, 1, tuple(s.info.background), flags=fa)
pb = hrt.params(W, H, spp, 50, 1, tuple(s.info.background), flags=fb)
for k in range(spp):
    A, ra = hrt.trace_path(s, cam, pa, x, y, k)
    B, rb = hrt.trace_path(s, cam, pb, x, y, k)
    if len(A) != len(B) or not np.array_equal(ra, rb):
        print(f"sample {k}: {len(A)} vs {len(B)} segments, radiance {ra} vs {rb}")
        for i in range(max(len(A), len(B))):
            sa = A[i] if i < len(A) else None
            sb = B[i] if i < len(B) else None
            fmt = lambda t: "-" if t is None else f"o={np.array2string(t[0], precision=9)} d={np.array2string(t[1], precision=9)} t={t[3]!r} w={t[4]}"
            print(f"  seg {i}: A {fmt(sa)}")
            print(f"          B {fmt(sb)}")
        break
