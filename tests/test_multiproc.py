"""Multi-rank path on CPU (gloo, world_size 2): bench.py's tile split (hrt/tiling.py split_tiles, the
diagonal interleave of the 16-px grid) and its host gather (tiling.gather_frame, point-to-point over
gloo) reassemble the single-process frame bit for bit.  Each rank renders its share with the CPU oracle
standing in for its GPU (the GPU's packed tile output equals the full frame:
tests/test_gpu_parity.py::test_multi_tile_call_matches_full_frame and ::test_tiling_split_on_gpu)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

W, H, SPP, DEPTH, SEED = 100, 45, 2, 8, 5


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _render_share(o, tiles):
    """The packed layout hrt_render_tiles_device writes: tiles back to back, each row-major."""
    parts, segs = [], 0
    for t in tiles:
        img, cnt = o.render(W, H, SPP, DEPTH, seed=SEED, region=t, threads=2)
        parts.append(img.reshape(-1))
        segs += cnt["segments"]
    return np.concatenate(parts), segs


def _worker(rank, world, port, q):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "hyper-ray-tracer_amd"), root]
    import torch

    import hrt
    from hrt import tiling
    from oracle import oracle as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    o = O.OracleScene(hrt.PRESETS["random"], 1)
    packed, segs = _render_share(o, tiling.split_tiles(W, H, world, rank))
    frame = tiling.gather_frame(packed, W, H, world, rank)
    t = torch.tensor([float(segs)], dtype=torch.float64)
    dist.all_reduce(t)
    if rank == 0:
        q.put((frame, int(t.item())))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_tile_split_and_gather_match_single_process(world):
    import hrt
    from oracle import oracle as O

    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    pc = mp.start_processes(_worker, args=(world, _free_port(), q), nprocs=world, join=False, start_method="spawn")
    frame, segs = q.get()  # read before joining: the frame does not fit in the pipe buffer
    while not pc.join(timeout=60):
        pass
    ref, cnt = O.OracleScene(hrt.PRESETS["random"], 1).render(W, H, SPP, DEPTH, seed=SEED, threads=4)
    assert not np.isnan(frame).any()
    assert np.array_equal(frame, ref)
    assert segs == cnt["segments"]


STEPS = 4


def _delivery_worker(rank, world, port, q):
    """bench.py's per-frame delivery (hrt/delivery.py): every step a different frame (seed SEED + k), each
    rank's share submitted as it would be after its launch, rank 0 receiving every completed frame."""
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "hyper-ray-tracer_amd"), root]
    import hrt
    from hrt import delivery, tiling
    from oracle import oracle as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    o = O.OracleScene(hrt.PRESETS["random"], 1)
    tiles = tiling.split_tiles(W, H, world, rank, 16)
    shares = []
    for k in range(STEPS):
        parts = [o.render(W, H, SPP, DEPTH, seed=SEED + k, region=t, threads=2)[0].reshape(-1) for t in tiles]
        shares.append(np.concatenate(parts))
    got = {}
    fd = delivery.FrameDelivery(W, H, world, rank, tiles, on_frame=lambda k, f: got.__setitem__(k, f.copy()))
    dist.barrier()
    for k in range(STEPS):
        fd.submit(k, shares[k])
    fd.flush(STEPS)
    dist.barrier()
    fd.close()
    if rank == 0:
        q.put(got)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 3])
def test_pipelined_frame_delivery_matches_single_process(world):
    """The shared-memory delivery (double-buffered frames, a worker thread per rank) hands rank 0 every
    step's frame, each equal bit for bit to the single-process frame of that step."""
    import hrt
    from oracle import oracle as O

    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    pc = mp.start_processes(_delivery_worker, args=(world, _free_port(), q), nprocs=world, join=False,
                            start_method="spawn")
    got = q.get()
    while not pc.join(timeout=60):
        pass
    o = O.OracleScene(hrt.PRESETS["random"], 1)
    assert sorted(got) == list(range(STEPS))
    for k in range(STEPS):
        ref, _ = o.render(W, H, SPP, DEPTH, seed=SEED + k, threads=4)
        assert np.array_equal(got[k], ref), k


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_split_is_a_balanced_partition(world):
    from hrt import tiling

    Wf, Hf = 1920, 1080
    allt = tiling.tile_grid(Wf, Hf)
    parts = [tiling.split_tiles(Wf, Hf, world, r) for r in range(world)]
    assert sorted(t for p in parts for t in p) == sorted(allt)
    px = [tiling.share_pixels(p) for p in parts]
    assert sum(px) == Wf * Hf
    assert max(px) - min(px) <= 68 * 16 * 16  # at most one tile per tile row apart
    # every rank's share covers the whole frame evenly: per horizontal band of 8 tile rows, shares agree
    for r, p in enumerate(parts):
        for band in range(0, Hf, 128):
            n = sum(1 for t in p if band <= t[1] < band + 128)
            assert abs(n - len([t for t in allt if band <= t[1] < band + 128]) / world) <= 8


def _failing_delivery_worker(rank, world, port, q):
    """Rank 1 fails before its first share (as if its launch raised) and closes its delivery with failed=True;
    rank 0, waiting for that share, must end with an error soon (not after delivery.WAIT_S), and closing
    must not raise."""
    import sys
    import time

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "hyper-ray-tracer_amd"), root]
    from hrt import delivery, tiling

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tiles = tiling.split_tiles(W, H, world, rank, 16)
    fd = delivery.FrameDelivery(W, H, world, rank, tiles)
    dist.barrier()
    t0 = time.perf_counter()
    err = None
    if rank == 1:
        fd.close(failed=True)
    else:
        fd.submit(0, np.zeros(tiling.share_pixels(tiles) * 4, np.float32))
        try:
            fd.flush(1)
        except RuntimeError as e:
            err = str(e)
        fd.close(failed=err is not None)
        q.put((err, time.perf_counter() - t0))
    dist.destroy_process_group()


def test_delivery_error_path_ends_every_rank():
    """an error on one rank must not leave the others waiting on the shared frame (the shared
    error flag ends their waits) nor hide the first error behind a BufferError at close."""
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    pc = mp.start_processes(_failing_delivery_worker, args=(2, _free_port(), q), nprocs=2, join=False,
                            start_method="spawn")
    err, dt = q.get()
    while not pc.join(timeout=60):
        pass
    assert err is not None and "failed" in err
    assert dt < 30


def _parity_worker(rank, world, port, q):
    """bench.py at N > 1: every rank renders its tile share (the oracle standing in for its GPU), the shares are
    gathered to rank 0, and rank 0 runs bench.rows_parity on the gathered frame while the others wait."""
    import argparse
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "hyper-ray-tracer_amd"), root]
    import hrt
    from hrt import tiling
    from oracle import oracle as O
    import bench

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    o = O.OracleScene(hrt.PRESETS["random"], 1)
    packed, _ = _render_share(o, tiling.split_tiles(W, H, world, rank))
    frame = tiling.gather_frame(packed, W, H, world, rank)
    if rank == 0:
        args = argparse.Namespace(preset="random", width=W, height=H, spp=SPP, depth=DEPTH, seed=SEED, cpu_seconds=0.2,
                                  no_parity=False, no_cpu_baseline=False)
        assert bench.parity_plan(world, rank, world, True, args) == "rows"

        def band_render(rows):  # the GPU's band render, the oracle standing in
            img, cnt = o.render_rows(W, H, SPP, rows, DEPTH, seed=SEED, threads=2)
            return img, cnt["segments"]

        cpu, parity = bench.rows_parity(args, frame, band_render, 2.8)
        q.put((cpu, parity))
    dist.barrier()
    dist.destroy_process_group()


def test_multi_rank_line_has_parity_and_cpu_baseline():
    """an N > 1 line carries the metric's own L-inf (rows of the frame gathered from the ranks'
    shares against the oracle, equal ray counts) and the CPU baseline, as the 1-GPU line does."""
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    pc = mp.start_processes(_parity_worker, args=(2, _free_port(), q), nprocs=2, join=False, start_method="spawn")
    cpu, parity = q.get()
    while not pc.join(timeout=60):
        pass
    assert parity["pass"] and parity["rays_equal"] and parity["band_render_equals_frame_rows"]
    assert parity["linf"] == 0.0 and parity["rows"] >= 2
    assert cpu["value"] > 0 and cpu["kind"] == "port" and cpu["cores"] >= 1
