"""bench.py — Mrays/s of the MI355X path-tracing megakernel on the RTIOW random-spheres scene.

Workload (BASELINE.json configs[1]): Scene::Random (src/application.rs:497-565, scene seed 1),
1920x1080, 500 spp, max_depth 50, camera :133-139.  One STEP = one full frame rendered into HBM
(inputs resident: the scene is committed once before timing).  1 ray = 1 world.hit call
(application.rs:482), counted exactly on the device.

  python bench.py                      # N=1, 3 timed frames after 1 warm-up
  python -m torch.distributed.run --nproc-per-node N bench.py --gpus N

Multi-GPU: one process per GPU, no RCCL (control-plane barrier/max over gloo only).
  --scaling weak   (default) every rank renders its own full 1920x1080x500 frame: the same image
                   with the next 500 samples per pixel (sample_offset = rank*500) -- per-GPU work fixed.
  --scaling strong the reference's 80x80 tiles of ONE frame dealt round-robin to the ranks
                   (hrt_tile_grid), each rank rendering its tile set in one launch.
Prints ONE JSON line on rank 0 (contract in the task statement).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "hyper-ray-tracer_amd"))

import torch  # noqa: E402  (first: libhrt binds to torch's HIP runtime)

import hrt  # noqa: E402

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
EARTHMAP = os.path.join(ROOT, "tests", "golden", "earthmap_rgb8.png")  # the reference's assets/earthmap.jpg, decoded


def earth_image():
    """The texture of the Earth scenes (earth, earth_perlin, final): the reference's own asset."""
    return hrt.load_image(EARTHMAP) if os.path.exists(EARTHMAP) else hrt.synthetic_earth()


# algorithmic bytes of one traversal/shading step of THIS kernel (layout.h):
NODE_B, PRIM_B, MAT_B, TEX_B, PIXEL_B = 32, 48, 32, 32, 16


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=500)
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--preset", default="random")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="budget of the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true", help="skip the oracle parity band (profiling runs)")
    ap.add_argument("--save", default="", help="write rank 0's last timed frame here (.pfm exact / .ppm 8-bit)")
    return ap.parse_args()


def host_cpu():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


SCENE_LABEL = {  # BASELINE.json configs
    "random": "RTIOW random spheres",
    "earth_perlin": "Earth-mapped sphere over a Perlin-noise ground",
    "random_10k": "10k random spheres, deep BVH",
    "cornell": "Next-Week Cornell box",
    "final": "Next-Week final scene",
}
SCENE_DATA = {
    "random": "synthetic (seeded Scene::Random builder; no external assets)",
    "earth_perlin": "seeded builder; the reference's assets/earthmap.jpg (tests/golden/earthmap_rgb8.png)",
    "final": "seeded builder; the reference's assets/earthmap.jpg (tests/golden/earthmap_rgb8.png)",
}


def log(msg):
    """Progress on stderr (stdout carries only the JSON line)."""
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"[bench] {msg}", file=sys.stderr, flush=True)


def cpu_baseline(args, rank_segments_per_sample):
    """The CPU restatement of the reference path (oracle/, 'port'), 80x80 tiles on a thread pool,
    timed on this host on a bounded band of the same frame (rows through the middle of the image),
    plus a one-thread rate on a short band."""
    sys.path.insert(0, ROOT)
    from oracle import oracle as O

    threads = min(16, os.cpu_count() or 1)
    o = O.OracleScene(hrt.PRESETS[args.preset], 1, earth_image())
    W, H = args.width, args.height
    # calibrate on one row at a few spp, then size a band to ~cpu_seconds
    t0 = time.perf_counter()
    _, c = o.render(W, H, 8, args.depth, seed=args.seed, region=(0, H // 2, W, 1), threads=threads)
    rate = c["segments"] / max(1e-6, time.perf_counter() - t0)
    seg_per_row = c["segments"] / 8 * args.spp
    rows = max(1, min(H // 2, int(args.cpu_seconds * rate / max(1.0, seg_per_row))))
    y0 = H // 2 - rows // 2
    t0 = time.perf_counter()
    _, c = o.render(W, H, args.spp, args.depth, seed=args.seed, region=(0, y0, W, rows), threads=threads)
    dt = time.perf_counter() - t0
    # one thread, a short stretch of the middle row (~2 s)
    px1 = max(8, min(W, int(2.0 * rate / threads / max(1.0, seg_per_row / W))))
    t1 = time.perf_counter()
    _, c1 = o.render(W, H, args.spp, args.depth, seed=args.seed, region=(0, H // 2, px1, 1), threads=1)
    dt1 = time.perf_counter() - t1
    return {
        "value": round(c["segments"] / dt / 1e6, 4),
        "unit": "Mrays/s",
        "cores": threads,
        "kind": "port",
        "label": "CPU restatement of the reference path (oracle/, not the reference binary)",
        "sample": f"rows {y0}..{y0 + rows - 1} of the {W}x{H} frame at {args.spp} spp "
                  f"({c['samples']} samples, {c['segments']} rays, {dt:.1f} s); reference aabb.rs culling",
        "segments_per_sample": round(c["segments"] / c["samples"], 4),
        "one_core_value": round(c1["segments"] / dt1 / 1e6, 4),
        "one_core_sample": f"{px1} pixels of row {H // 2} at {args.spp} spp ({c1['segments']} rays, {dt1:.1f} s)",
        "host_cpu": host_cpu(),
        "nproc": os.cpu_count(),
    }


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("gloo")  # control plane only: barrier + max of the timings
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    scene = hrt.preset(args.preset, 1, earth_image())
    scene.commit(local)
    si = scene.scene_info()
    W, H = args.width, args.height
    cam = hrt.preset_camera(scene.info, W, H)
    bg = tuple(scene.info.background)
    if args.scaling == "weak" or world == 1:
        tiles = [(0, 0, W, H)]
        p = hrt.params(W, H, args.spp, args.depth, args.seed, bg, sample_offset=rank * args.spp)
    else:
        tiles = hrt.tile_grid(W, H, 80, rank, world)
        p = hrt.params(W, H, args.spp, args.depth, args.seed, bg)
    n_px = sum(t[2] * t[3] for t in tiles)
    out = torch.empty(n_px * 4, dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev)

    # exact work of one step: segments are deterministic for a fixed seed and sample range
    tw = time.perf_counter()
    st = hrt.render_tiles_device(scene, cam, p, tiles, out.data_ptr(), stream.cuda_stream, want_stats=True)
    seg_step, samples_step = int(st.segments), int(st.samples)
    warm_s = time.perf_counter() - tw
    progress = warm_s > 20.0  # long frames: a progress line per timed frame
    log(f"warm-up frame: {seg_step} rays in {warm_s:.1f} s")
    for _ in range(max(0, args.warmup - 1)):
        hrt.render_tiles_device(scene, cam, p, tiles, out.data_ptr(), stream.cuda_stream)

    def barrier():
        if world > 1:
            torch.distributed.barrier()

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record(stream)
        hrt.render_tiles_device(scene, cam, p, tiles, out.data_ptr(), stream.cuda_stream)
        ev[k][1].record(stream)
        if progress and k + 1 < args.steps:
            ev[k][1].synchronize()  # progress line per frame (long configs); the clock keeps running
            log(f"timed frame {k + 1}/{args.steps}")
    torch.cuda.synchronize(dev)
    barrier()
    dt = time.perf_counter() - t0
    launch_ms = sum(a.elapsed_time(b) for a, b in ev) / max(1, args.steps)
    if world > 1:
        import torch.distributed as dist

        t = torch.tensor([dt, float(seg_step), float(samples_step)], dtype=torch.float64)
        tmax = t.clone()
        dist.all_reduce(tmax[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        dt, seg_all, samples_all = float(tmax[0]), float(t[1]), float(t[2])
    else:
        seg_all, samples_all = float(seg_step), float(samples_step)

    value = seg_all * args.steps / dt / 1e6

    # algorithmic bytes of one launch (instrumented pass, rank 0, outside the timed region)
    roofline = None
    if rank == 0:
        pc = hrt.params(W, H, args.spp, args.depth, args.seed, bg, sample_offset=p.sample_offset, flags=hrt.RENDER_COUNT_WORK)
        sc = hrt.render_tiles_device(scene, cam, pc, tiles, out.data_ptr(), stream.cuda_stream, want_stats=True)
        shades = int(sc.segments)  # upper bound: one material fetch per segment that hit (misses fetch none)
        alg_bytes = (int(sc.node_visits) * NODE_B + int(sc.prim_tests) * PRIM_B + shades * MAT_B
                     + int(sc.tex_evals) * TEX_B + n_px * PIXEL_B)
        achieved = alg_bytes / (launch_ms * 1e-3) / 1e9
        roofline = {
            "bound": "hbm",
            "achieved": round(achieved, 2),
            "peak": PEAK_HBM_GBS,
            "unit": "GB/s",
            "frac": round(achieved / PEAK_HBM_GBS, 5),
            "traffic": None,
            "bytes_per_launch": alg_bytes,
            "bytes_per_ray": round(alg_bytes / max(1, seg_step), 1),
            "node_visits_per_ray": round(int(sc.node_visits) / max(1, seg_step), 2),
            "prim_tests_per_ray": round(int(sc.prim_tests) / max(1, seg_step), 3),
            "launch_ms": round(launch_ms, 3),
        }
        prof = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(prof):
            try:
                with open(prof) as fh:
                    pm = json.load(fh)
                key = f"{args.preset}_{W}x{H}_{args.spp}"
                if key in pm:
                    roofline["traffic"] = pm[key]["hbm_bytes_per_launch"]
                    roofline["traffic_source"] = pm[key]["source"]
            except (OSError, ValueError, KeyError):
                pass

    if rank == 0 and args.save:
        if tiles == [(0, 0, W, H)]:
            hrt.write_image(args.save, out.view(H, W, 4).cpu().numpy())
        else:
            print("--save: rank 0 holds a tile set, not the frame; nothing written", file=sys.stderr)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, seg_step / max(1, samples_step))

    if rank == 0:
        line = {
            "metric": "Mrays/sec at 1920x1080, 500 spp, RTIOW final scene; per-pixel Linf vs CPU ref",
            "value": round(value, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 2),
            "higher_is_better": True,
            "scaling": "weak" if world == 1 or args.scaling == "weak" else "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": SCENE_DATA.get(args.preset, "synthetic (seeded scene builder)"),
            "config": {
                "workload": f"Scene::{args.preset} ({SCENE_LABEL.get(args.preset, args.preset)}) {W}x{H}, {args.spp} spp, max_depth {args.depth}",
                "width": W, "height": H, "spp": args.spp, "max_depth": args.depth,
                "rays_per_step": int(seg_all), "samples_per_step": int(samples_all),
                "rays_per_sample": round(seg_all / max(1.0, samples_all), 4),
                "msamples_per_s": round(samples_all * args.steps / dt / 1e6, 2),
                "parallelism": f"{world} GPU(s), {args.scaling} split, no collectives",
                "cull_mode": {0: "reference", 1: "slab (approximate)", 2: "exact (reference test + provably safe culling)"}[si.cull_mode],
            },
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
