"""Quick device probe: time the megakernel on one preset (segments/s), no oracle involved."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "hyper-ray-tracer_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import hrt  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--preset", default="random")
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--spp", type=int, default=16)
ap.add_argument("--depth", type=int, default=50)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--ab", default="", help="comma list of flag values to alternate (A/B in one process)")
ap.add_argument("--env", default="", help="/-list of NAME=VALUE[,NAME=VALUE] env settings to alternate (A/B)")
ap.add_argument("--commit-env", default="", help="/-list of NAME=VALUE[,...] env settings applied while the scene is "
                "committed (walk-stream placement knobs): one scene per setting, alternated (A/B)")
ap.add_argument("--count", action="store_true", help="also run one instrumented pass per variant")
ap.add_argument("--options", default="", help="/-list of NAME=VALUE[,...] hrt_scene_options (chunk_min, chunk_max, "
                "chunk_uniform, walk_tree, bvh_ties): one scene per setting, alternated (A/B)")
ap.add_argument("--view", action="store_true", help="commit with hrt_scene_set_view(the camera), as bench.py does")
ap.add_argument("--share", type=int, default=1, help="render rank 0's share of an N-way tile split (hrt/tiling.py)")
a = ap.parse_args()

_earth = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "earthmap_rgb8.png")


def set_env(e):
    for kv in filter(None, e.split(",")):
        k, v = kv.split("=", 1)
        os.environ[k] = v


def clear_env(e):
    for kv in filter(None, e.split(",")):
        os.environ.pop(kv.split("=", 1)[0], None)


scenes = {}
variants = [("env", ce) for ce in (a.commit_env.split("/") if a.commit_env else [""])]
if a.options:
    variants = [("opt", o) for o in a.options.split("/")]
for kind, ce in variants:
    opts = {kv.split("=")[0]: int(kv.split("=")[1]) for kv in filter(None, ce.split(","))} if kind == "opt" else None
    if kind == "env":
        set_env(ce)
    sc = hrt.preset(a.preset, 1, hrt.load_image(_earth) if os.path.exists(_earth) else None, options=opts)
    if a.view and hasattr(hrt.load(), "hrt_scene_set_view"):  # bench.py's default placement hint
        sc.set_view(hrt.preset_camera(sc.info, a.width, a.height))
    sc.commit(0)
    if kind == "env":
        clear_env(ce)
    scenes[ce] = sc
    si = sc.scene_info()
    print(f"scene {a.preset} [{ce}]: nodes {si.nodes} prims {si.prims} features {si.feature_mask:#x} cull {si.cull_mode} blob {si.blob_bytes} B", flush=True)
s = scenes[next(iter(scenes))]
cam = hrt.preset_camera(s.info, a.width, a.height)
flag_sets = [int(x) for x in a.ab.split(",")] if a.ab else [0]
env_sets = a.env.split("/") if a.env else [""]
flag_sets = [(f, e, c) for f in flag_sets for e in env_sets for c in scenes]
out = torch.empty((a.height, a.width, 4), dtype=torch.float32, device="cuda")
tiles = [(0, 0, a.width, a.height)]
if a.share > 1:
    from hrt import tiling
    tiles = [tuple(t) for t in tiling.split_tiles(a.width, a.height, a.share, 0)]
    print(f"share 0 of {a.share}: {len(tiles)} tiles, {tiling.share_pixels(tiles)} pixels", flush=True)
res = {k: [] for k in flag_sets}
imgs = {}
for r in range(a.reps):
    for key in flag_sets:
        fl, env, ce = key
        set_env(env)
        p = hrt.params(a.width, a.height, a.spp, a.depth, 1, tuple(s.info.background), flags=fl)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st = hrt.render_tiles_device(scenes[ce], cam, p, tiles, out.data_ptr(), 0, want_stats=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        res[key].append(st.segments / dt / 1e6)
        imgs[key] = out.clone()
        clear_env(env)
        print(f"rep {r} {key}: {dt*1e3:.1f} ms  segments {st.segments}  seg/sample {st.segments/st.samples:.3f}  "
              f"{st.segments/dt/1e6:.1f} Mrays/s  {st.samples/dt/1e6:.1f} Msamples/s", flush=True)
for key in flag_sets:
    print(f"{key}: median {sorted(res[key])[len(res[key])//2]:.1f} Mrays/s  identical-to-first {bool(torch.equal(imgs[key], imgs[flag_sets[0]]))}")
    if a.count:
        fl, env, ce = key
        set_env(env)
        p = hrt.params(a.width, a.height, a.spp, a.depth, 1, tuple(s.info.background), flags=fl | hrt.RENDER_COUNT_WORK)
        st = hrt.render_tiles_device(scenes[ce], cam, p, tiles, out.data_ptr(), 0, want_stats=True)
        clear_env(env)
        print(f"   count: nodes/ray {st.node_visits/st.segments:.2f} prims/ray {st.prim_tests/st.segments:.3f} "
              f"walk-lane-util {(getattr(st, 'walk_steps', 0) or st.node_visits)/max(1, st.walk_slots):.3f} walk-iters/ray {st.walk_slots/st.segments:.1f} "
              f"shade-passes/ray {st.shade_slots/st.segments:.3f} prim-blocks/ray {st.prim_slots/st.segments:.2f} (x64 lanes)", flush=True)
        pcs = list(st.phase_cycles)
        if sum(pcs):
            print("   phase cycles: claim+start {:.1%}  walk {:.1%}  shade {:.1%}".format(*[c / sum(pcs) for c in pcs]),
                  f" (leaf tests {st.leaf_cycles / sum(pcs):.1%} of all, inside walk)", flush=True)
        if st.walk_slots:
            ws = st.walk_slots
            steps = getattr(st, "walk_steps", 0) or st.node_visits  # node_visits also counts leaf-program nodes
            print(f"   walk slots: stepping {steps/ws:.1%}  parked on a leaf {st.park_slots/ws:.1%}  "
                  f"done, waiting to shade {st.wait_slots/ws:.1%}  no walk {1 - (steps + st.park_slots + st.wait_slots)/ws:.1%}",
                  flush=True)
img = out.cpu().numpy()
print("mean rgb", img[..., :3].mean(axis=(0, 1)), "finite", bool(np.isfinite(img).all()))
