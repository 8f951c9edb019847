"""Price a 4-wide walk on the host before building it: the lane simulator
(tests/native/lane_sim.hip lane_sim_wide_price) walks every segment of a region both over the sphere walk
stream's binary hierarchy (what render_basic_kernel walks) and over that hierarchy collapsed to 4-wide records,
checks the two give the same closest hit and winner, and counts the work.

  python scripts/price_wide.py [--preset random] [--width 1920 --height 1080] [--spp 16] [--rows 6]

Output: per segment, binary node steps vs wide dependent loads (records + climbs) and box tests; per lockstep
group (the 64 lanes of an 8x8 block at one sample and one segment index), the sum of the slowest lane's steps
(what a wave would spend if its lanes walked together)."""
import argparse
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hyper-ray-tracer_amd"), ROOT]
import hrt  # noqa: E402


def build(out="/tmp/hrt_price/liblanesim.so"):
    os.makedirs(os.path.dirname(out), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-shared",
                    "--offload-host-only", "-I" + os.path.join(ROOT, "include"),
                    "-I" + os.path.join(ROOT, "hyper-ray-tracer_amd", "csrc"),
                    os.path.join(ROOT, "tests", "native", "lane_sim.hip"), "-o", out], check=True)
    return ctypes.CDLL(out)


def price(L, preset, W, H, spp, rows, x0=0, w=None, seed=1, arity=4):
    earth = hrt.load_image(os.path.join(ROOT, "tests", "golden", "earthmap_rgb8.png"))
    s = hrt.preset(preset, 1, earth)
    blob, info = hrt.scene_blob(s)
    cam = hrt.preset_camera(s.info, W, H)
    p = hrt.params(W, H, spp, 50, seed, tuple(s.info.background))
    w = W - x0 if w is None else w
    tot = np.zeros(16, np.uint64)
    for y in rows:  # 8-row bands: whole 8x8 blocks, the lockstep groups of the kernels' waves
        out = np.zeros((8, w, 4), np.float32)
        cnt = np.zeros(8, np.uint64)
        o = np.zeros(16, np.uint64)
        rc = L.lane_sim_wide_price(blob, ctypes.byref(info), ctypes.byref(cam), ctypes.byref(p), x0, y, w, 8,
                                   out.ctypes.data_as(ctypes.c_void_p), cnt.ctypes.data_as(ctypes.c_void_p),
                                   o.ctypes.data_as(ctypes.c_void_p), arity)
        assert rc == 0, rc
        tot[:8] += o[:8]
        tot[8] = max(tot[8], o[8])
        tot[9:] += o[9:]
    seg = int(tot[0])
    r = {k: int(v) for k, v in zip(["segments", "bin_steps", "bin_leaf", "wide_records", "wide_climbs", "wide_tests",
                                     "wide_leaf", "mismatch", "depth_max", "groups", "bin_lock", "wide_lock",
                                     "lock_steps", "lock_cold_77k32", "lock_cold_77k16", "lock_cold_152k32"], tot)}
    per = {k: round(r[k] / seg, 3) for k in ("bin_steps", "bin_leaf", "wide_records", "wide_climbs", "wide_tests", "wide_leaf")}
    per["wide_dependent"] = round((r["wide_records"] + r["wide_climbs"]) / seg, 3)
    per["bin_lane_util"] = round(r["bin_steps"] / max(1, r["bin_lock"]), 3)
    per["wide_lane_util"] = round((r["wide_records"] + r["wide_climbs"]) / max(1, r["wide_lock"]), 3)
    per["lock_ratio_wide_over_bin"] = round(r["wide_lock"] / max(1, r["bin_lock"]), 3)
    # VALU under lockstep: a binary iteration ~28 VALU (23 for the node step + loop control); a wide iteration
    # runs the record visit (4 box tests ~76 + mask / trail ~10; arity 2: 2 tests ~38 + 6) and the climb (~8)
    # for every lane of the wave
    for k in ("lock_cold_77k32", "lock_cold_77k16", "lock_cold_152k32"):  # lockstep steps a wave waits on global memory
        per[k + "_share"] = round(r[k] / max(1, r["lock_steps"]), 4)
    per["valu_lock_ratio_wide_over_bin"] = round(r["wide_lock"] * (94 if arity == 4 else 52) / max(1, r["bin_lock"] * 28), 3)
    return r, per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="random")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=16)
    ap.add_argument("--rows", type=int, default=6)
    ap.add_argument("--x0", type=int, default=0)
    ap.add_argument("--w", type=int, default=None)
    ap.add_argument("--arity", type=int, default=4)
    a = ap.parse_args()
    L = build()
    rows = [int((k + 0.5) * a.height / a.rows) // 8 * 8 for k in range(a.rows)]
    r, per = price(L, a.preset, a.width, a.height, a.spp, rows, a.x0, a.w, arity=a.arity)
    print(a.preset, a.width, a.height, a.spp, "rows", rows)
    print(r)
    print(per)


if __name__ == "__main__":
    main()
