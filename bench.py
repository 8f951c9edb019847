"""bench.py — Mrays/s of the MI355X path-tracing megakernel on the RTIOW random-spheres scene.

Workload (BASELINE.json configs[1]): Scene::Random (src/application.rs:497-565, scene seed 1),
1920x1080, 500 spp, max_depth 50, camera :133-139.  One STEP = one full frame rendered into HBM
(inputs resident: the scene is committed once before timing).  1 ray = 1 world.hit call
(application.rs:482), counted exactly on the device.

  python bench.py                      # N=1, 3 timed frames after 1 warm-up
  python bench.py --gpus N             # N ranks, started by bench.py itself (hrt/launcher.py)
  python -m torch.distributed.run --nproc-per-node N bench.py --gpus N

Multi-GPU (north star: the image tiled across the GPUs of one node, host gather, no RCCL): one process
per GPU; gloo carries only the control plane (barrier, max of the timings) and the host gather.  Without
torchrun, `--gpus N` (N > 1, no WORLD_SIZE in the environment) makes this process a supervisor that starts
N fresh ranks before anything touches the GPU, forwards rank 0's line and exits non-zero if any rank fails.
  --scaling tiles  (default) the frame's tile grid dealt to the ranks (hrt/tiling.py: 16-px tiles,
                   diagonal interleave); each rank renders its share in one launch per step; after the
                   timed steps the shares are gathered to rank 0 and the frame is checked bit for bit
                   against a 1-GPU render of the whole frame.  Total work fixed: "scaling": "strong".
  --scaling weak   replicas: every rank renders the whole frame with its own next spp samples per pixel.
Rank 0 prints ONE JSON line (contract in the task statement), with
  parity       per-pixel L-inf of the timed frame against the CPU oracle on a band of rows spread over
               the frame (one GPU's share, --share N: on 16-px tiles spread over the share), at the frame's
               full spp, plus equality of the ray counts (the metric's own "per-pixel Linf vs CPU ref");
  roofline     the kernel's real bound, VALU instruction issue (PMC counts of this build from
               profiles/roofline_pmc.json over the live launch time), with the LDS / HBM figures beside it;
  cpu_baseline the CPU restatement of the reference path (oracle/) on the same rows, timed on this
               host's usable cores.
"""
import argparse
import hashlib
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "hyper-ray-tracer_amd"))

if __name__ == "__main__":
    # `--gpus N` without a launcher: start the N ranks here, before torch or the HIP library is loaded
    from hrt import launcher

    _pre = argparse.ArgumentParser(add_help=False)
    _pre.add_argument("--gpus", type=int, default=1)
    _gpus = _pre.parse_known_args()[0].gpus
    if launcher.needs_spawn(_gpus):
        sys.exit(launcher.run_ranks([sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:], _gpus))

import torch  # noqa: E402  (first: libhrt binds to torch's HIP runtime)

import hrt  # noqa: E402
from hrt import tiling  # noqa: E402

PEAK_HBM_GBS = 8000.0     # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
PEAK_LDS_GBS = 150000.0   # ds_read_b64/b128 aggregate with every CU streaming (MI355X_MICROARCH.md, LDS)
SIMDS, MAX_CLOCK_HZ = 1024, 2.4e9
VALU_CYC = 2.0            # a wave64 VALU instruction issues over 2 cycles on a SIMD32 (MI355X_MICROARCH.md)
EARTHMAP = os.path.join(ROOT, "tests", "golden", "earthmap_rgb8.png")  # the reference's assets/earthmap.jpg, decoded
TOL = 1e-3                # north star: per-pixel L-inf <= 1e-3 vs the CPU reference


def earth_image():
    """The texture of the Earth scenes (earth, earth_perlin, final): the reference's own asset."""
    return hrt.load_image(EARTHMAP) if os.path.exists(EARTHMAP) else hrt.synthetic_earth()


# SURVEY 8(d) algorithmic bytes of one traversal / shading step (the reference model, this kernel's counts)
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
    ap.add_argument("--scaling", choices=["tiles", "weak"], default="tiles")
    ap.add_argument("--tile", type=int, default=tiling.TILE, help="tile pitch of the multi-GPU split")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="budget of the CPU-baseline / parity sample")
    ap.add_argument("--no-cpu-baseline", action="store_true", help="skip the CPU leg (and with it the parity band)")
    ap.add_argument("--no-parity", action="store_true", help="skip the oracle parity band (profiling runs)")
    ap.add_argument("--no-frame-check", action="store_true", help="N>1: skip the 1-GPU bit-identity check")
    ap.add_argument("--save", default="", help="write rank 0's last timed frame here (.pfm exact / .ppm 8-bit)")
    ap.add_argument("--one-device", action="store_true",
                    help="every rank on GPU 0 (rehearsal of the N > 1 path on a one-GPU box; not a scaling figure)")
    ap.add_argument("--rehearsal", choices=["turns", "concurrent"], default="turns",
                    help="--one-device timing: ranks launch their shares in turns (each launch alone on the GPU, "
                         "as on separate GPUs), or all at once (the ranks' persistent grids then contend for the "
                         "one GPU, DESIGN.md section 9)")
    ap.add_argument("--streams", default="auto",
                    help="timed steps round-robin over this many HIP streams (their own output buffers and library "
                         "slots): a step's persistent grid then starts on the CUs the previous step's last waves free.  "
                         "'auto' = 2 for a short launch of a tile share (stream_count), else 1")
    ap.add_argument("--allow-knobs", action="store_true",
                    help="print the line even when A/B environment knobs of the library are set (never for a headline)")
    ap.add_argument("--chunks", default="frame",
                    help="sample-chunk schedule (hrt_scene_options): 'frame' (default) = the library's schedule for the "
                         "frame, the same at every GPU count; an integer k = chunks of at least k samples (A/B lines "
                         "only: the image then differs from the default frame in its low bits)")
    ap.add_argument("--view", choices=["camera", "none"], default="camera",
                    help="hrt_scene_set_view before commit: 'camera' = the rendered camera (a walk stream beyond LDS "
                         "stages the node parts its rays visit most: C4, Final), 'none' = the largest-box ranking.  "
                         "Same image bit for bit either way")
    ap.add_argument("--share", type=int, default=1,
                    help="one process: render rank 0's share of an N-way tile split (one GPU's part of an N-GPU frame)")
    ap.add_argument("--launch-record", default="",
                    help="write the timed launch's record (hrt_last_launch: kernel, grid, occupancy, VGPRs, scratch) here")
    ap.add_argument("--no-delivery", action="store_true",
                    help="skip the per-frame delivery phase (frame_ms: launch + D2H + host placement, pipelined)")
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


def usable_cpus():
    """CPUs this process may actually use: its affinity set, capped by the cgroup CPU quota (the GPU
    box exposes 256 host threads but grants one job a 16-CPU quota)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    return max(1, min(n, int(math.floor(quota)) if quota else n)), quota


def rank_devices(dev, rank, local, world):
    """Every rank's GPU: its PCI address (domain:bus:device) and UUID, gathered to all ranks over gloo, so the
    line shows how many distinct devices the N ranks really ran on."""
    pr = torch.cuda.get_device_properties(dev)
    me = {"rank": rank, "local_rank": local, "device": dev.index, "name": pr.name,
          "pci": f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}", "uuid": str(pr.uuid)}
    if world == 1:
        return [me]
    import torch.distributed as dist

    allv = [None] * world
    dist.all_gather_object(allv, me)
    return allv


def distinct_devices(devices):
    return len({(d["pci"], d["uuid"]) for d in devices})


OVERLAP_LAUNCH_SAMPLES = 600e6  # stream_count: C2's halves (518 M samples) still gain from overlapping steps


def chunk_options(args):
    """hrt_scene_options for the run's sample chunks (--chunks).  'frame' (the default, every headline and every
    N > 1 line): None, the library's schedule, a function of the frame alone (spp, scene class, full image size),
    so the image is the same bits at every GPU count.  An integer k: chunks of at least k samples
    (at most 64 of them), an A/B line only; its frame_check then compares with the default frame and reports
    the difference instead of bit identity.  (r05 switched C2's shares at 4 and 8 GPUs to 8-sample chunks, which
    made the 4- and 8-GPU images differ in their low bits from the 1-GPU image: VERDICT r05, missing 2.)"""
    if args.chunks == "frame":
        return None
    return {"chunk_min": int(args.chunks), "chunk_max": 64}


def stream_count(args, share):
    """--streams: how many HIP streams the timed steps alternate over.  Two for a GPU's share of a tile split in a
    short launch (under OVERLAP_LAUNCH_SAMPLES: C2's shares), so the next step's grid fills the CUs the end of the
    previous one frees (profiles/r05_stream_overlap_ab.jsonl: C2's 1/8 share +5.5%, 1/4 +1%, 1/2 +1.6%); one for a
    whole frame (within noise, and once 3.5% slower) and for long launches (C4's 1/8 share: 3.3% slower)."""
    if args.streams != "auto":
        return max(1, int(args.streams))
    return 2 if share >= 2 and args.width * args.height * args.spp / share < OVERLAP_LAUNCH_SAMPLES else 1


def knob_report(launch):
    """The library's A/B environment knobs in effect (hrt_last_launch.knobs: every HRT_* variable the library
    read that is set), as a list of NAME=value."""
    k = (launch or {}).get("knobs") or ""
    return [x for x in k.split(";") if x]


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


def log(msg, all_ranks=False):
    """Progress on stderr (stdout carries only the JSON line)."""
    rank = int(os.environ.get("RANK", "0"))
    if rank == 0 or all_ranks:
        print(f"[bench r{rank}] {msg}", file=sys.stderr, flush=True)


def band_rows(H, n):
    """n full-width rows spread evenly over the frame (the CPU sample and the parity band)."""
    n = max(1, min(H, n))
    return sorted({min(H - 1, int((k + 0.5) * H / n)) for k in range(n)})


def cpu_leg(args, frame_rays_per_sample):
    """The CPU restatement of the reference path (oracle/, 'port') on rows spread over the frame at the
    frame's full spp, on this host's usable cores, plus a one-thread rate on a short
    stretch.  Returns (cpu_baseline dict, rows, oracle image of the rows, oracle counters)."""
    sys.path.insert(0, ROOT)
    from oracle import oracle as O

    threads, quota = usable_cpus()
    o = O.OracleScene(hrt.PRESETS[args.preset], 1, earth_image())
    W, H = args.width, args.height
    # calibrate on a few rows at a few spp, then size the band to ~cpu_seconds
    probe = band_rows(H, 4)
    t0 = time.perf_counter()
    _, c = o.render_rows(W, H, 4, probe, args.depth, seed=args.seed, threads=threads)
    rate = c["segments"] / max(1e-6, time.perf_counter() - t0)
    rays_per_row = c["segments"] / (4 * len(probe)) * args.spp
    n_rows = max(2, min(H, int(args.cpu_seconds * rate / max(1.0, rays_per_row))))
    rows = band_rows(H, n_rows)
    t0 = time.perf_counter()
    img, c = o.render_rows(W, H, args.spp, rows, args.depth, seed=args.seed, threads=threads)
    dt = time.perf_counter() - t0
    # one thread, a stretch of the middle row (~2 s)
    px1 = max(8, min(W, int(2.0 * rate / threads / max(1.0, rays_per_row / W))))
    t1 = time.perf_counter()
    _, c1 = o.render(W, H, args.spp, args.depth, seed=args.seed, region=(0, H // 2, px1, 1), threads=1)
    dt1 = time.perf_counter() - t1
    seg_per_sample = c["segments"] / max(1, c["samples"])
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    cb = {
        "value": round(c["segments"] / dt / 1e6, 4),
        "unit": "Mrays/s",
        "cores": threads,
        "kind": "port",
        "label": "CPU restatement of the reference path (oracle/, not the reference binary)",
        "sample": f"{len(rows)} full-width rows spread evenly over the {W}x{H} frame at {args.spp} spp "
                  f"({c['samples']} samples, {c['segments']} rays, {dt:.1f} s); reference aabb.rs culling",
        "segments_per_sample": round(seg_per_sample, 4),
        "frame_segments_per_sample": round(frame_rays_per_sample, 4),
        "sample_vs_frame": round(seg_per_sample / max(1e-9, frame_rays_per_sample), 4),
        "one_core_value": round(c1["segments"] / dt1 / 1e6, 4),
        "one_core_sample": f"{px1} pixels of row {H // 2} at {args.spp} spp ({c1['segments']} rays, {dt1:.1f} s)",
        "host_cpu": host_cpu(),
        "nproc": os.cpu_count(),
        "cpu_quota": quota,
        "threads_note": f"{threads} worker threads = the CPUs this job may use (affinity {aff}, "
                        f"cgroup cpu.max quota {quota if quota else 'none'})",
    }
    return cb, rows, img, c


def rows_parity(args, frame, band_render, frame_rays_per_sample):
    """The metric's own figure on a whole delivered frame (1 GPU, or rank 0's gathered N-GPU frame): the oracle
    (cpu_leg) on full-width rows spread over the frame at full spp, and the per-pixel L-inf of the frame's rows
    against it.  `frame` is the (H, W, 4) frame (numpy or a tensor); band_render(rows) renders those rows again
    on this process's GPU and returns (pixels (len(rows), W, 4), world.hit count), so the GPU's ray count of the
    rows is compared with the oracle's and the band with the frame's rows (the delivered frame is what was
    checked).  Returns (cpu_baseline, parity)."""
    import numpy as np

    cpu, rows, ref_rows, cnt = cpu_leg(args, frame_rays_per_sample)
    if args.no_parity:
        return cpu, None
    got = frame[torch.tensor(rows, device=frame.device)].cpu().numpy() if torch.is_tensor(frame) else np.asarray(frame)[rows]
    band_px, band_segs = band_render(rows)
    band_same = bool((np.asarray(band_px) == got).all())
    linf = float(abs(got - ref_rows).max())
    rays_equal = int(band_segs) == cnt["segments"]
    parity = {"linf": linf, "tol": TOL, "pass": bool(linf <= TOL and rays_equal and band_same), "rays_equal": rays_equal,
              "gpu_rays": int(band_segs), "cpu_rays": cnt["segments"], "rows": len(rows),
              "pixels": len(rows) * args.width, "spp": args.spp, "band_render_equals_frame_rows": band_same,
              "reference": "oracle/ CPU restatement of the reference path, same seed and samples"}
    return cpu, parity


def parity_plan(world, rank, share, tiled, args):
    """Which CPU leg rank 0 runs after the timed steps (the other ranks wait at a barrier, no GPU work):
    'tiles' for one GPU's share of a split (--share N, the C4 / C5 config lines), 'rows' for a whole frame:
    one GPU's, the frame gathered from N ranks' tile shares, or rank 0's replica (--scaling weak: sample
    offset 0, the same frame); None on other ranks or without the CPU leg.  Every N prints both."""
    if rank != 0 or args.no_cpu_baseline:
        return None
    if world == 1 and share > 1:
        return "tiles"
    return "rows"


def spread_tiles(tiles, n, W, H):
    """Indices of n of a share's tiles spread over the frame in two dimensions: for each point of a
    Hammersley set (x = (k + 1/2) / n, y = the golden-ratio sequence) the share tile nearest to it, not yet
    picked.  (Evenly spaced list indices land in one tile column under the diagonal deal: C5's 1/8 share
    then sampled only the frame's left edge, where every camera ray misses the box.)"""
    phi = (5 ** 0.5 - 1) / 2
    centre = [(x + w / 2, y + h / 2) for x, y, w, h in tiles]
    picked = set()
    for k in range(min(n, len(tiles))):
        px, py = (k + 0.5) / n * W, ((0.5 + k * phi) % 1.0) * H
        best = min((i for i in range(len(tiles)) if i not in picked),
                   key=lambda i: (centre[i][0] - px) ** 2 + (centre[i][1] - py) ** 2)
        picked.add(best)
    return sorted(picked)


def cpu_leg_tiles(args, tiles, frame_rays_per_sample):
    """cpu_leg for one GPU's share of a tile split (the C4 / C5 config lines): the oracle on 16-px tiles of the
    share spread over the frame (spread_tiles) at the frame's full spp (each tile's rows in 8-px tasks on the usable cores), as many
    as the CPU budget allows (at least one).  Returns (cpu_baseline dict, picked tile indices, the oracle's
    pixels of those tiles packed as the share is, oracle counters)."""
    import numpy as np

    sys.path.insert(0, ROOT)
    from oracle import oracle as O

    threads, quota = usable_cpus()
    o = O.OracleScene(hrt.PRESETS[args.preset], 1, earth_image())
    W, H = args.width, args.height

    def tile_render(t, spp):
        x, y, w, h = t
        img, c = o.render_rows(W, H, spp, list(range(y, y + h)), args.depth, seed=args.seed, threads=threads, x0=x, w=w,
                               task_w=8)
        return img, c

    probes = spread_tiles(tiles, 4, W, H)  # the cost of a tile varies across the frame: price four
    t0 = time.perf_counter()
    seg = sum(tile_render(tiles[i], 4)[1]["segments"] for i in probes)
    rate = seg / max(1e-6, time.perf_counter() - t0)
    per_tile = seg / len(probes) / 4 * args.spp
    n = max(1, min(len(tiles), int(args.cpu_seconds * rate / max(1.0, per_tile))))
    picks = spread_tiles(tiles, n, W, H)
    t0 = time.perf_counter()
    imgs, tot = [], {}
    for i in picks:
        img, c = tile_render(tiles[i], args.spp)
        imgs.append(img.reshape(-1))
        for k, v in c.items():
            tot[k] = tot.get(k, 0) + v
    dt = time.perf_counter() - t0
    seg_per_sample = tot["segments"] / max(1, tot["samples"])
    cb = {
        "value": round(tot["segments"] / dt / 1e6, 4),
        "unit": "Mrays/s",
        "cores": threads,
        "kind": "port",
        "label": "CPU restatement of the reference path (oracle/, not the reference binary)",
        "sample": f"{len(picks)} of the share's {len(tiles)} 16-px tiles, spread over the frame, at {args.spp} spp "
                  f"({tot['samples']} samples, {tot['segments']} rays, {dt:.1f} s); reference aabb.rs culling",
        "segments_per_sample": round(seg_per_sample, 4),
        "frame_segments_per_sample": round(frame_rays_per_sample, 4),
        "sample_vs_frame": round(seg_per_sample / max(1e-9, frame_rays_per_sample), 4),
        "host_cpu": host_cpu(),
        "nproc": os.cpu_count(),
        "cpu_quota": quota,
        "threads_note": f"{threads} worker threads = the CPUs this job may use (cgroup cpu.max quota {quota if quota else 'none'})",
    }
    return cb, picks, np.concatenate(imgs), tot


def pmc_key(args, share):
    """profiles/roofline_pmc.json key of the launch this run times: the preset, the frame and spp, and for a
    tile split the share (rank 0's of `share` ranks), whose counters are those of that share's launch."""
    return f"{args.preset}_{args.width}x{args.height}_{args.spp}" + (f"_share{share}" if share > 1 else "")


def load_pmc(key):
    try:
        return json.load(open(os.path.join(ROOT, "profiles", "roofline_pmc.json"))).get(key)
    except (OSError, ValueError):
        return None


def apply_pmc(ro, key, pm, launch_s, seg_step):
    """Fill the roofline object's counter fields from the PMC record of this launch's workload (`key`);
    counters that would put the launch above peak belong to another workload and are rejected."""
    ro["pmc_key"] = key
    if pm and pm.get("rejected"):
        ro["pmc_rejected"] = pm["rejected"]
    elif pm and pm.get("valu_insts"):
        sha = hashlib.sha256(open(hrt.LIB_PATH, "rb").read()).hexdigest()[:16]
        ach = pm["valu_insts"] / launch_s / 1e9
        ro.update(achieved=round(ach, 1), frac=round(ach / ro["peak"], 4), traffic=pm.get("hbm_bytes"),
                  pmc_source=pm["source"], pmc_build_match=(pm.get("lib_sha16") == sha), lib_sha16=sha,
                  valu_insts_per_launch=pm["valu_insts"], valu_insts_per_ray=round(pm["valu_insts"] / max(1, seg_step), 2))
        if pm.get("clock_hz"):
            ro["clock_ghz_profiled"] = round(pm["clock_hz"] / 1e9, 3)
            ro["frac_at_profiled_clock"] = round(pm["valu_insts"] * VALU_CYC / (SIMDS * pm["clock_hz"] * launch_s), 4)
        if pm.get("hbm_bytes"):
            ro["hbm_counter_GBs"] = round(pm["hbm_bytes"] / launch_s / 1e9, 2)
            ro["hbm_frac"] = round(pm["hbm_bytes"] / launch_s / 1e9 / PEAK_HBM_GBS, 5)
        if pm.get("sq_lds_idx_active"):
            ro["lds_bank_conflict_share"] = round(pm["sq_lds_bank_conflict"] / pm["sq_lds_idx_active"], 4)
        if ro["frac"] > 1.0:
            # counters of another workload (or build) than this launch: never report above peak
            ro.update(achieved=None, frac=None, frac_at_profiled_clock=None,
                      pmc_rejected=f"counters of {key} give {ach:.0f} > peak over this launch's time")


def roofline_obj(args, scene, cam, bg, tiles, p, out_ptr, stream, launch_ms, seg_step, n_px, share=1):
    """The kernel's bound and where it sits (rank 0, instrumented pass outside the timed region)."""
    pc = hrt.params(args.width, args.height, args.spp, args.depth, args.seed, bg, sample_offset=p.sample_offset,
                    flags=hrt.RENDER_COUNT_WORK)
    sc = hrt.render_tiles_device(scene, cam, pc, tiles, out_ptr, stream, want_stats=True)
    launch_s = launch_ms * 1e-3
    alg_bytes = (int(sc.node_visits) * NODE_B + int(sc.prim_tests) * PRIM_B + int(sc.segments) * MAT_B
                 + int(sc.tex_evals) * TEX_B + n_px * PIXEL_B)
    ro = {
        "bound": "valu_issue",
        "achieved": None, "peak": round(SIMDS * MAX_CLOCK_HZ / VALU_CYC / 1e9, 1), "unit": "Gwave-inst/s",
        "frac": None, "traffic": None,
        "walk_lane_util": round(int(sc.walk_steps or sc.node_visits) / max(1, int(sc.walk_slots)), 4) if sc.walk_slots else None,
        "alg_bytes_per_launch": alg_bytes,
        "alg_bytes_per_ray": round(alg_bytes / max(1, seg_step), 1),
        "lds_frac": round(alg_bytes / launch_s / 1e9 / PEAK_LDS_GBS, 4),
        "node_visits_per_ray": round(int(sc.node_visits) / max(1, seg_step), 2),
        "prim_tests_per_ray": round(int(sc.prim_tests) / max(1, seg_step), 3),
        "launch_ms": round(launch_ms, 3),
        "note": "achieved = SQ_INSTS_VALU of one launch of this build (rocprofv3 PMC, profiles/) / the live "
                "HIP-event launch time; peak = 1024 SIMDs x 2.4 GHz / 2 cycles per wave64 VALU instruction",
    }
    key = pmc_key(args, share)
    apply_pmc(ro, key, load_pmc(key), launch_s, seg_step)
    return ro


def delivery_phase(args, scene, cam, p, tiles, n_px, dev, stream, world, rank, barrier, W, H, ms_per_step):
    """K more steps, each launch followed by its frame's delivery to the host (hrt/delivery.py): D2H copy
    of the share into pinned memory on a second stream, placement into a node-wide shared-memory frame
    by a worker thread, rank 0 handing the completed frame over; double-buffered, so frame k is copied
    and placed while frame k + 1 renders.  Returns (delivery dict for rank 0's line, rank 0's last
    delivered frame or None)."""
    from hrt import delivery

    outs = [torch.empty(n_px * 4, dtype=torch.float32, device=dev) for _ in range(2)]
    K = args.steps
    last = {}

    def keep(k, f):
        if k == K:  # the last timed frame (step 0 is the untimed warm-up through the pipeline)
            last["frame"] = f.copy()

    log("delivery phase: set-up", all_ranks=True)
    fd = delivery.FrameDelivery(W, H, world, rank, tiles, on_frame=keep, device=dev)
    log("delivery phase: running", all_ranks=True)
    try:
        for k in range(K + 1):
            if k == 1:  # step 0 warmed the pipeline (pinned pages, placement index, shared frame)
                fd.flush(1)
                barrier()
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
            fd.before_launch(k, stream)
            hrt.render_tiles_device(scene, cam, p, tiles, outs[k % 2].data_ptr(), stream.cuda_stream)
            fd.submit(k, outs[k % 2], stream)
        fd.flush(K + 1)
        log(f"delivery phase: {K + 1} frames delivered", all_ranks=True)
        barrier()
        dt = time.perf_counter() - t0
        if world > 1:
            import torch.distributed as dist

            t = torch.tensor([dt], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t[0])
        scene.synchronize()
    except BaseException:
        fd.close(failed=True)  # no collective on the error path: the other ranks' waits end on the shared flag
        raise
    barrier()
    fd.close()
    frame_ms = dt / K * 1e3
    d = {"frame_ms": round(frame_ms, 2), "ms_per_step": round(ms_per_step, 2),
         "frame_vs_launch": round(frame_ms / max(1e-9, ms_per_step), 4), "frames": K,
         "bytes_per_frame": W * H * 16,
         "path": "each step: launch into one of two device buffers; D2H of the share into pinned memory on a copy "
                 "stream; a worker thread per rank places it into a double-buffered frame in host shared memory; "
                 "rank 0 hands over each completed frame (hrt/delivery.py)"}
    return d, last.get("frame")


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist

        # control plane + host gather only (no RCCL, no device collective).  Gloo prints its connection
        # report on stdout, which carries only the JSON line: send fd 1 to stderr meanwhile.
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo")
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    if args.gpus > 1 and world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE is {world}")
    if args.one_device:
        local = 0
    n_dev = torch.cuda.device_count()
    if local >= n_dev:
        raise SystemExit(f"bench.py rank {rank}: LOCAL_RANK {local} but {n_dev} GPU(s) visible "
                         "(--one-device rehearses N ranks on one GPU)")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    devices = rank_devices(dev, rank, local, world)
    if world > 1 and not args.one_device and distinct_devices(devices) != world:
        if len({d["device"] for d in devices}) == world:  # distinct HIP devices whose PCI / UUID fields collide
            log(f"warning: {world} ranks on {world} HIP device indices report {distinct_devices(devices)} distinct "
                "PCI addresses / UUIDs", all_ranks=True)
        else:
            raise SystemExit(f"bench.py: {world} ranks run on {distinct_devices(devices)} distinct devices "
                             "(--one-device rehearses N ranks on one GPU)")
    turns = args.one_device and world > 1 and args.rehearsal == "turns"

    share_of = world if (world > 1 and args.scaling == "tiles") else max(1, args.share)
    options = chunk_options(args)
    scene = hrt.preset(args.preset, 1, earth_image(), options=options)
    W, H = args.width, args.height
    cam = hrt.preset_camera(scene.info, W, H)
    if args.view == "camera":  # placement hint: the staged part of a stream beyond LDS (never the image)
        scene.set_view(cam)
    scene.commit(local)
    si = scene.scene_info()
    blob_info = hrt.scene_blob(scene)[1]
    bg = tuple(scene.info.background)
    tiled = args.scaling == "tiles"
    share = world if (world > 1 and tiled) else max(1, args.share)
    if world == 1 and share > 1:  # one GPU's part of a share-way frame (config lines of C4 / C5)
        tiles = tiling.split_tiles(W, H, share, 0, args.tile)
        p = hrt.params(W, H, args.spp, args.depth, args.seed, bg)
    elif world == 1:
        tiles = [(0, 0, W, H)]  # the union of the grid: one launch over the frame
        p = hrt.params(W, H, args.spp, args.depth, args.seed, bg)
    elif tiled:
        tiles = tiling.split_tiles(W, H, world, rank, args.tile)
        p = hrt.params(W, H, args.spp, args.depth, args.seed, bg)
    else:
        tiles = [(0, 0, W, H)]
        p = hrt.params(W, H, args.spp, args.depth, args.seed, bg, sample_offset=rank * args.spp)
    n_px = tiling.share_pixels(tiles)
    out = torch.empty(n_px * 4, dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev)

    # exact work of one step: segments are deterministic for a fixed seed and sample range
    tw = time.perf_counter()
    st = hrt.render_tiles_device(scene, cam, p, tiles, out.data_ptr(), stream.cuda_stream, want_stats=True)
    seg_step, samples_step = int(st.segments), int(st.samples)
    warm_s = time.perf_counter() - tw
    progress = warm_s > 20.0  # long frames: a progress line per timed frame
    log(f"work-count frame: {seg_step} rays in {warm_s:.1f} s")
    n_str = 1 if turns else stream_count(args, share_of)
    streams = [stream] + [torch.cuda.Stream(dev) for _ in range(n_str - 1)]
    outs = [out] + [torch.empty_like(out) for _ in range(n_str - 1)]
    # W warm-up steps as the timed ones run them (asynchronous launches: the first one also sizes the
    # library's other in-flight slots, so no timed step allocates device or pinned memory)
    for k in range(max(n_str, args.warmup)):
        hrt.render_tiles_device(scene, cam, p, tiles, outs[k % n_str].data_ptr(), streams[k % n_str].cuda_stream)

    def barrier():
        if world > 1:
            torch.distributed.barrier()

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    switch = torch.zeros(1, device=dev)
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        if turns:  # --one-device rehearsal: rank r launches its share while the others wait at the barrier
            for r in range(world):
                if r == rank:
                    # the GPU switching to this process's queue (up to ~25 ms after the other rank's turn, r05 kernel
                    # traces) happens on a one-element fill before the clock starts: separate GPUs do not pay it
                    with torch.cuda.stream(stream):
                        switch.zero_()
                    torch.cuda.synchronize(dev)
                    ev[k][0].record(stream)
                    hrt.render_tiles_device(scene, cam, p, tiles, out.data_ptr(), stream.cuda_stream)
                    ev[k][1].record(stream)
                    torch.cuda.synchronize(dev)
                barrier()
            continue
        sk = streams[k % n_str]
        ev[k][0].record(sk)
        hrt.render_tiles_device(scene, cam, p, tiles, outs[k % n_str].data_ptr(), sk.cuda_stream)
        ev[k][1].record(sk)
        if progress and k + 1 < args.steps:
            ev[k][1].synchronize()  # progress line per frame (long configs); the clock keeps running
            log(f"timed frame {k + 1}/{args.steps}")
    torch.cuda.synchronize(dev)
    barrier()
    dt = time.perf_counter() - t0
    scene.synchronize()  # raises if the walk watchdog stopped any timed launch (incomplete frame)
    launch = hrt.last_launch()  # what the timed steps ran: kernel, persistent grid, occupancy, VGPRs, scratch
    knobs = knob_report(launch)
    if knobs and not args.allow_knobs:
        raise SystemExit(f"bench.py: library A/B knobs set in the environment ({', '.join(knobs)}): a headline line "
                         "runs the default library; pass --allow-knobs for an A/B line")
    if args.launch_record:
        os.makedirs(os.path.dirname(os.path.abspath(args.launch_record)), exist_ok=True)
        with open(args.launch_record, "w") as fh:
            json.dump(launch, fh)
    log(f"timed steps done: {dt / args.steps * 1e3:.1f} ms per step", all_ranks=True)
    launch_ms = sum(a.elapsed_time(b) for a, b in ev) / max(1, args.steps)
    if n_str > 1:  # overlapping steps: an event pair also spans the wait for the CUs; the step's share of the clock
        launch_ms = dt / max(1, args.steps) * 1e3
    rank_ms = [round(launch_ms, 2)]
    if world > 1:
        import torch.distributed as dist

        t = torch.tensor([dt, float(seg_step), float(samples_step)], dtype=torch.float64)
        tmax = t.clone()
        dist.all_reduce(tmax[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        per = [torch.zeros(1, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(per, torch.tensor([launch_ms], dtype=torch.float64))
        rank_ms = [round(float(x), 2) for x in per]
        dt, seg_all, samples_all = float(tmax[0]), float(t[1]), float(t[2])
    else:
        seg_all, samples_all = float(seg_step), float(samples_step)
    value = seg_all * args.steps / dt / 1e6

    # per-frame delivery (launch + D2H + placement into the host frame, pipelined): frame_ms beside the
    # launch-only ms_per_step; for N > 1 the delivered frame is the host gather that the bit-identity
    # check below uses
    frame_check = None
    frame = None
    deliv = None
    if not args.no_delivery and (world > 1 or share == 1):
        deliv, frame = delivery_phase(args, scene, cam, p, tiles, n_px, dev, stream, world, rank, barrier, W, H,
                                      ms_per_step=dt / args.steps * 1e3)
    if world > 1 and tiled:
        tg = time.perf_counter()
        if deliv is None:  # no delivery phase: gather the last timed frame's shares over gloo
            frame = tiling.gather_frame(out.cpu().numpy(), W, H, world, rank,
                                        shares=lambda r: tiling.split_tiles(W, H, world, r, args.tile))
        gather_s = time.perf_counter() - tg
        if rank == 0:
            frame_check = {"gathered_pixels": int((frame[..., 3] == 1.0).sum()), "frame_pixels": W * H,
                           "gather": "delivered frame (pipelined shared-memory gather)" if deliv else "gloo gather after the timed steps",
                           "gather_ms": None if deliv else round(gather_s * 1e3, 1), "tile": args.tile,
                           "rank_launch_ms": rank_ms, "imbalance": round(max(rank_ms) / max(1e-9, min(rank_ms)), 4)}
            if not args.no_frame_check:
                # the reference is a 1-GPU render of the whole frame with the DEFAULT options (the headline
                # frame's schedule): the N-GPU image must be those bits, whatever N
                ref_scene = scene
                if options is not None:  # an A/B chunk schedule: the default frame comes from a default scene
                    ref_scene = hrt.preset(args.preset, 1, earth_image())
                    if args.view == "camera":
                        ref_scene.set_view(cam)
                    ref_scene.commit(local)
                ref = torch.empty(W * H * 4, dtype=torch.float32, device=dev)
                p1 = hrt.params(W, H, args.spp, args.depth, args.seed, bg)
                hrt.render_tiles_device(ref_scene, cam, p1, [(0, 0, W, H)], ref.data_ptr(), stream.cuda_stream)
                torch.cuda.synchronize(dev)
                ref_np = ref.view(H, W, 4).cpu().numpy()
                same = bool((ref_np == frame).all())
                frame_check["bit_identical_to_1gpu_frame"] = same
                frame_check["reference_frame"] = "1-GPU render of the whole frame, default scene options"
                if options is not None:
                    frame_check["linf_vs_1gpu_frame"] = float(abs(ref_np - frame).max())
                    frame_check["chunk_options"] = options
                elif not same:
                    raise SystemExit("gathered multi-GPU frame differs from the 1-GPU frame")
                del ref_scene
        barrier()
    elif not tiled or share == 1:
        # one GPU's whole frame, or (weak scaling) rank 0's replica: sample offset 0, the default frame; its
        # delivery placed every replica over one shared frame, so the check reads rank 0's own output
        frame = out.view(H, W, 4)

    cpu, parity = None, None
    plan = parity_plan(world, rank, share, tiled, args)
    if plan == "tiles":
        # one GPU's share (C4 / C5 config lines): the oracle on tiles spread over the share, and the metric's
        # L-inf on those tiles of the timed launch's packed output
        cpu, picks, ref_px, cnt = cpu_leg_tiles(args, tiles, seg_step / max(1, samples_step))
        if not args.no_parity:
            import numpy as np

            offs = np.cumsum([0] + [t[2] * t[3] for t in tiles])
            packed = out.cpu().numpy()
            got = np.concatenate([packed[4 * offs[i]:4 * offs[i + 1]] for i in picks])
            sel = [tiles[i] for i in picks]
            band_out = torch.empty(tiling.share_pixels(sel) * 4, dtype=torch.float32, device=dev)
            band = hrt.render_tiles_device(scene, cam, p, sel, band_out.data_ptr(), stream.cuda_stream, want_stats=True)
            band_same = bool((band_out.cpu().numpy() == got).all())
            linf = float(abs(got - ref_px).max())
            rays_equal = int(band.segments) == cnt["segments"]
            parity = {"linf": linf, "tol": TOL, "pass": bool(linf <= TOL and rays_equal), "rays_equal": rays_equal,
                      "gpu_rays": int(band.segments), "cpu_rays": cnt["segments"], "tiles": len(picks),
                      "pixels": tiling.share_pixels(sel), "spp": args.spp, "band_render_equals_share_tiles": band_same,
                      "reference": "oracle/ CPU restatement of the reference path, same seed and samples"}
    elif plan == "rows":
        # the whole frame: 1 GPU's timed frame, or at N > 1 the frame delivered from every rank's share (tiles)
        # or rank 0's replica (weak, sample offset 0): the rows of THAT frame against the oracle
        def band_render(rows):
            band_out = torch.empty(len(rows) * W * 4, dtype=torch.float32, device=dev)
            st_b = hrt.render_tiles_device(scene, cam, p, [(0, y, W, 1) for y in rows], band_out.data_ptr(),
                                           stream.cuda_stream, want_stats=True)
            return band_out.view(len(rows), W, 4).cpu().numpy(), int(st_b.segments)

        cpu, parity = rows_parity(args, frame, band_render, seg_all / max(1.0, samples_all))
        if parity is not None and world > 1:
            parity["frame"] = ("the frame delivered from the N ranks' tile shares" if tiled
                               else "rank 0's replica (sample offset 0)")
    barrier()  # the other ranks wait for rank 0's CPU leg here, with no GPU work

    roofline = None
    if rank == 0:
        roofline = roofline_obj(args, scene, cam, bg, tiles, p, out.data_ptr(), stream.cuda_stream, launch_ms, seg_step, n_px,
                                share=share)

    if rank == 0 and args.save and frame is not None:
        hrt.write_image(args.save, frame.cpu().numpy() if torch.is_tensor(frame) else frame)

    if rank == 0:
        line = {
            "metric": "Mrays/sec at 1920x1080, 500 spp, RTIOW final scene; per-pixel Linf vs CPU ref",
            "value": round(value, 2),
            "unit": "Mrays/s",
            "n_gpus": distinct_devices(devices),
            "steps": args.steps,
            "warmup": args.warmup,
            "streams": n_str,
            "ms_per_step": round(dt / args.steps * 1e3, 2),
            "higher_is_better": True,
            "scaling": "strong" if tiled else "weak",  # tiles: the frame is the fixed total at every N
            "vs_baseline": None,
            "dtype": "f32",
            "data": SCENE_DATA.get(args.preset, "synthetic (seeded scene builder)"),
            "config": {
                "workload": f"Scene::{args.preset} ({SCENE_LABEL.get(args.preset, args.preset)}) {W}x{H}, {args.spp} spp, max_depth {args.depth}",
                "width": W, "height": H, "spp": args.spp, "max_depth": args.depth,
                "rays_per_step": int(seg_all), "samples_per_step": int(samples_all),
                "rays_per_sample": round(seg_all / max(1.0, samples_all), 4),
                "msamples_per_s": round(samples_all * args.steps / dt / 1e6, 2),
                "parallelism": (f"{world} GPU(s), frame tiled ({args.tile}-px tiles, diagonal interleave), host gather, no collectives"
                                if world > 1 and tiled else f"{world} GPU(s), " + ("replicas" if world > 1 else "one launch per frame")),
                **({"share": f"rank 0 of a {share}-way tile split ({args.tile}-px tiles): one GPU's part of a {share}-GPU frame",
                    "share_pixels": n_px} if world == 1 and share > 1 else {}),
                "cull_mode": {0: "reference", 1: "slab (approximate)", 2: "exact (reference test + provably safe culling)"}[si.cull_mode],
                "sample_chunks": {**hrt.sample_chunks(scene, p), "options": options or "frame default"},
                "placement": ({"staged": ("node parts the rendered camera's rays visit most (hrt_scene_set_view)"
                                          if args.view == "camera" else "node parts under the largest boxes"),
                               "staged_bytes": int(blob_info.walk_hot), "stream_bytes": int(blob_info.walk_bytes)}
                              if blob_info.walk_hot else "the whole walk stream in LDS"),
            },
            "launch": launch,
            "ranks": world,
            "devices": devices,
            "launcher": ("bench.py --gpus (hrt/launcher.py)" if os.environ.get("HRT_BENCH_SPAWNED")
                         else ("torch.distributed.run" if world > 1 else "single process")),
            "parity": parity,
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        if deliv is not None:
            line["delivery"] = deliv
        if frame_check is not None:
            line["frame_check"] = frame_check
        if knobs:
            line["knobs"] = knobs
        if args.one_device and world > 1:
            line["rehearsal"] = args.rehearsal
            line["note"] = (f"--one-device: all {world} ranks shared GPU 0 (a rehearsal of the multi-GPU path, not a "
                            "scaling figure): n_gpus counts distinct devices; "
                            + ("the ranks launched their shares in turns, each alone on the GPU" if turns else
                               "the ranks launched at once and their persistent grids contended for the GPU"))
        print(json.dumps(line), flush=True)
    if world > 1:
        barrier()  # every rank ends with rank 0's line
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
