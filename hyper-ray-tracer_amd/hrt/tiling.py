"""Multi-GPU image tiling: the frame split into tiles dealt to the ranks of one node, each rank rendering
its share with one launch on its own GPU, and a host-side gather of the shares into the frame.

North star: "the image is tiled across the 8 GPUs of one node (embarrassingly parallel: no RCCL, a
host-side gather only)".  The reference tiles the image for its tokio workers (src/application.rs:363-364
grid, :404-415 one task per tile, :461-472 tiles gathered over an mpsc channel to the main thread).

- split_tiles: the tile grid (hrt_tile_grid: integer ragged edges) at a fine pitch (16 px by default),
  dealt by a diagonal interleave, tile (tx, ty) -> rank (tx + ty) mod world, so every rank's share is
  spread evenly over sky, ground and spheres: shares differ by at most one tile per row and their costs
  by far less than a coarse 80 px deal (whose columns repeat every world tiles).
- gather_frame: every rank's packed output (tiles back to back, the layout hrt_render_tiles_device
  writes) goes to rank 0 over the control-plane process group (gloo, host memory): point-to-point
  sends, no device collective.  Rank 0 places the tiles into the (H, W, 4) frame.
Pixels are keyed by their global index (RNG per (seed, pixel, sample)), so the gathered frame is bit
for bit the 1-GPU frame whatever the split (tests/test_multiproc.py, tests/test_gpu_parity.py).
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

Tile = Tuple[int, int, int, int]
TILE = 16


def tile_grid(width: int, height: int, tile: int = TILE) -> List[Tile]:
    """The whole grid in row-major order (application.rs:363-364 with integer ragged edges)."""
    out = []
    for y in range(0, height, tile):
        for x in range(0, width, tile):
            out.append((x, y, min(tile, width - x), min(tile, height - y)))
    return out


def split_tiles(width: int, height: int, world: int, rank: int, tile: int = TILE) -> List[Tile]:
    """Rank `rank`'s share of the grid: tile (tx, ty) goes to rank (tx + ty) % world."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("need 0 <= rank < world")
    return [t for t in tile_grid(width, height, tile) if (t[0] // tile + t[1] // tile) % world == rank]


def share_pixels(tiles: Sequence[Tile]) -> int:
    return int(sum(t[2] * t[3] for t in tiles))


def place_tiles(frame: np.ndarray, tiles: Sequence[Tile], packed: np.ndarray) -> None:
    """Write a packed share (tiles back to back, each row-major, 4 floats per pixel) into the frame."""
    flat = np.asarray(packed, np.float32).reshape(-1)
    off = 0
    for x, y, w, h in tiles:
        frame[y:y + h, x:x + w] = flat[off * 4:(off + w * h) * 4].reshape(h, w, 4)
        off += w * h


def gather_frame(packed: np.ndarray, width: int, height: int, world: int, rank: int,
                 shares: Optional[Callable[[int], Sequence[Tile]]] = None, group=None) -> Optional[np.ndarray]:
    """Host gather of every rank's packed share to rank 0; returns the (H, W, 4) frame on rank 0, None
    elsewhere.  `shares(r)` gives rank r's tile list (default: split_tiles)."""
    import torch
    import torch.distributed as dist

    shares = shares or (lambda r: split_tiles(width, height, world, r))
    mine = torch.from_numpy(np.ascontiguousarray(packed, np.float32).reshape(-1))
    if rank != 0:
        dist.send(mine, dst=0, group=group)
        return None
    frame = np.full((height, width, 4), np.nan, np.float32)
    place_tiles(frame, shares(0), mine.numpy())
    for r in range(1, world):
        t = shares(r)
        buf = torch.empty(share_pixels(t) * 4, dtype=torch.float32)
        dist.recv(buf, src=r, group=group)
        place_tiles(frame, t, buf.numpy())
    return frame
