"""Multi-rank path on CPU (gloo, world_size 2): the tile split bench.py --scaling strong uses
(hrt_tile_grid, round-robin over ranks) followed by a host-side gather reproduces the single-process
frame bit for bit.  Each rank renders its tiles with the CPU oracle standing in for the GPU (the GPU
equivalence of a tile set to the full frame is tests/test_gpu_parity.py::test_multi_tile_call...)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

W, H, SPP, DEPTH, SEED = 160, 90, 2, 8, 5


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "hyper-ray-tracer_amd"), root]
    import hrt
    from oracle import oracle as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    o = O.OracleScene(hrt.PRESETS["random"], 1)
    tiles = hrt.tile_grid(W, H, 80, rank, world)
    mine = []
    for t in tiles:
        img, cnt = o.render(W, H, SPP, DEPTH, seed=SEED, region=t, threads=2)
        mine.append((t, img, cnt["segments"]))
    gathered = [None] * world if rank == 0 else None
    dist.gather_object(mine, gathered, dst=0)
    if rank == 0:
        frame = np.full((H, W, 4), np.nan, np.float32)
        segs = 0
        for part in gathered:
            for (x, y, w, h), img, s in part:
                frame[y:y + h, x:x + w] = img
                segs += s
        q.put((frame, segs))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_two_rank_tile_split_matches_single_process(world):
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
