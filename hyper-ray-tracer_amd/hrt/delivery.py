"""Per-frame delivery of the multi-GPU frame to the host: every rank's share copied back and placed into
one frame in host shared memory, pipelined behind the next frame's launch.

Reference: the tile tasks send each finished tile over an mpsc channel (src/application.rs:461-472) and
the main thread places it into the displayed frame (:284-306).  Here, one node and one process per GPU:

  step k on rank r:  launch into device buffer out[k % 2]  (compute stream)
                     D2H copy of out[k % 2] into pinned staging[k % 2]  (copy stream, after the launch)
                     worker thread: wait for that copy, place the share's tiles into frame[k % 2] of a
                     node-wide shared-memory segment, publish ready[r] = k + 1
  rank 0's worker:   once every ready[r] > k the frame is complete: `on_frame(k, frame)`, consumed = k + 1

Both device buffers, both staging buffers and both shared frames are double-buffered, so launch k + 1
runs while frame k is copied, placed and handed over.  The slot reuse rules:
  - the launch of step k + 2 into out[k % 2] waits (on the GPU: stream wait on an event) for the D2H
    copy of step k out of it;
  - the D2H copy of step k + 2 into staging[k % 2] waits (host semaphore) for the worker to have placed
    step k;
  - placing step k into frame[k % 2] waits until rank 0 has handed over frame k - 2 (consumed >= k - 1).
No device collective and no xGMI traffic (north star: "a host-side gather only"); the control plane
(barrier, the segment's name) is the gloo group.  Pixels are keyed by their global index, so the
delivered frame equals the 1-GPU frame bit for bit (tests/test_multiproc.py).
"""
from __future__ import annotations

import queue
import threading
import time
import uuid
from multiprocessing import shared_memory
from typing import Callable, Optional, Sequence

import numpy as np

from . import tiling

HDR_BYTES = 4096
WAIT_S = 120.0  # longest any wait may take before the delivery declares itself stuck (raises)


def share_index(width: int, tiles: Sequence[tiling.Tile]) -> Optional[np.ndarray]:
    """Frame pixel index (y * width + x) of every pixel of a packed share, in packed order; None when the
    share is the whole frame as one tile (the packed layout is then the frame itself)."""
    if len(tiles) == 1 and tiles[0][0] == 0 and tiles[0][1] == 0 and tiles[0][2] == width:
        return None
    parts = []
    for x, y, w, h in tiles:
        yy, xx = np.mgrid[y:y + h, x:x + w]
        parts.append((yy * width + xx).reshape(-1))
    return np.concatenate(parts).astype(np.int64)


def _wait(cond: Callable[[], bool], what: str) -> None:
    t0 = time.perf_counter()
    pause = 2e-5
    while not cond():
        if time.perf_counter() - t0 > WAIT_S:
            raise RuntimeError(f"frame delivery stuck waiting for {what}")
        time.sleep(pause)
        pause = min(pause * 2, 1e-3)


class FrameDelivery:
    """One rank's end of the pipelined host gather (see the module docstring).

    submit(k, out, stream)   after the launch of step k into `out` (a float32 tensor holding this rank's
                             packed share) was enqueued on `stream` (None: `out` is host memory, copied
                             synchronously: the CPU tests)
    before_launch(k, stream) before the launch of step k: makes `stream` wait until out[k % 2] was read
    flush(n)                 waits until n frames were delivered (rank 0: handed over; others: placed)
    """

    def __init__(self, width: int, height: int, world: int, rank: int, tiles: Sequence[tiling.Tile],
                 on_frame: Optional[Callable[[int, np.ndarray], None]] = None, group=None, device=None):
        import torch
        import torch.distributed as dist

        self.W, self.H, self.world, self.rank = width, height, world, rank
        self.n_px = tiling.share_pixels(tiles)
        self.idx = share_index(width, tiles)
        self.on_frame = on_frame
        self.frame_bytes = width * height * 16
        name = [f"hrt_frame_{uuid.uuid4().hex[:12]}" if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(name, src=0, group=group)
        if rank == 0:
            self.shm = shared_memory.SharedMemory(name=name[0], create=True, size=HDR_BYTES + 2 * self.frame_bytes)
            np.ndarray((HDR_BYTES // 8,), np.int64, self.shm.buf)[:] = 0
        if world > 1:
            dist.barrier(group=group)
        if rank != 0:
            self.shm = shared_memory.SharedMemory(name=name[0])
            try:  # rank 0 owns (and unlinks) the segment: keep this process's tracker from unlinking it too
                from multiprocessing import resource_tracker

                resource_tracker.unregister(self.shm._name, "shared_memory")
            except Exception:
                pass
        self.hdr = np.ndarray((HDR_BYTES // 8,), np.int64, self.shm.buf)  # ready[0..world-1], consumed, error
        self.frames = [np.ndarray((height * width, 4), np.float32, self.shm.buf, HDR_BYTES + s * self.frame_bytes)
                       for s in range(2)]
        self.cuda = device is not None
        if self.cuda:
            self.copy_stream = torch.cuda.Stream(device=device)
            self.staging = [torch.empty(self.n_px * 4, dtype=torch.float32, pin_memory=True) for _ in range(2)]
            self.copied = [torch.cuda.Event() for _ in range(2)]
            self.read_done = [None, None]  # event recorded after the D2H copy out of out[slot]
        else:
            self.staging = [np.empty(self.n_px * 4, np.float32) for _ in range(2)]
        self.free = threading.Semaphore(2)  # staging slots the worker has finished placing
        self.q: "queue.Queue" = queue.Queue()
        self.err: Optional[BaseException] = None
        self.placed = 0      # steps this rank has placed (worker)
        self.delivered = 0   # rank 0: frames handed over
        self.frame_times: list = []
        self.worker = threading.Thread(target=self._run, daemon=True)
        self.worker.start()

    # ---------------------------------------------------------------- main thread
    def before_launch(self, k: int, stream) -> None:
        ev = self.read_done[k % 2] if self.cuda else None
        if ev is not None:
            stream.wait_event(ev)

    def submit(self, k: int, out, stream=None) -> None:
        if self.err:
            raise self.err
        if not self.free.acquire(timeout=WAIT_S):
            raise RuntimeError("frame delivery stuck: staging slot never freed")
        slot = k % 2
        if self.cuda:
            import torch

            done = torch.cuda.Event()
            done.record(stream)
            with torch.cuda.stream(self.copy_stream):
                self.copy_stream.wait_event(done)
                self.staging[slot].copy_(out, non_blocking=True)
                self.copied[slot].record(self.copy_stream)
            self.read_done[slot] = self.copied[slot]
        else:
            np.copyto(self.staging[slot], np.asarray(out, np.float32).reshape(-1))
        self.q.put(k)

    def flush(self, n: int) -> None:
        target = (lambda: self.delivered >= n) if self.rank == 0 else (lambda: self.placed >= n)
        _wait(lambda: target() or self.err is not None or self.hdr[self.world + 1] != 0, f"frame {n - 1}")
        if self.hdr[self.world + 1] != 0 and not self.err:
            self.err = RuntimeError("another rank's frame delivery failed")
        if self.err:
            raise self.err

    def close(self, failed: bool = False) -> None:
        """Stop the worker and release the segment.  failed=True (an error on this rank): raise the shared
        error flag first, so that this worker's and every other rank's waits end instead of running into
        WAIT_S.  A worker still blocked after the join keeps its views of the segment: the segment is then
        left to the OS (closing it under live views would raise BufferError and hide the first error)."""
        if failed or self.err is not None:
            try:
                self.hdr[self.world + 1] = 1
            except Exception:
                pass
        self.q.put(None)
        self.worker.join(timeout=30)
        if self.worker.is_alive():
            import sys

            print(f"[delivery rank {self.rank}] worker still running at close; shared frame left open",
                  file=sys.stderr, flush=True)
            return
        del self.hdr, self.frames
        self.shm.close()
        if self.rank == 0:
            try:
                self.shm.unlink()
            except FileNotFoundError:
                pass

    # ---------------------------------------------------------------- worker thread
    def _run(self) -> None:
        try:
            while True:
                k = self.q.get()
                if k is None:
                    return
                slot = k % 2
                if self.cuda:
                    self.copied[slot].synchronize()
                src = self.staging[slot]
                src = src.numpy() if self.cuda else src
                hdr = self.hdr
                _wait(lambda: hdr[self.world] >= k - 1 or hdr[self.world + 1] != 0, f"frame {k - 2} handed over")
                if hdr[self.world + 1] != 0:
                    raise RuntimeError("another rank's frame delivery failed")
                dst = self.frames[slot]
                if self.idx is None:
                    np.copyto(dst.reshape(-1), src)
                else:
                    dst.view(np.complex128).reshape(-1)[self.idx] = src.view(np.complex128)
                hdr[self.rank] = k + 1
                self.placed = k + 1
                self.free.release()
                if self.rank == 0:
                    _wait(lambda: bool((hdr[:self.world] >= k + 1).all()) or hdr[self.world + 1] != 0, f"frame {k}'s shares")
                    if hdr[self.world + 1] != 0:
                        raise RuntimeError("another rank's frame delivery failed")
                    if self.on_frame is not None:
                        self.on_frame(k, dst.reshape(self.H, self.W, 4))
                    self.frame_times.append(time.perf_counter())
                    hdr[self.world] = k + 1
                    self.delivered = k + 1
        except BaseException as e:  # surfaced by submit / flush on the main thread
            import sys
            import traceback

            print(f"[delivery rank {self.rank}] worker failed: {e!r}", file=sys.stderr, flush=True)
            traceback.print_exc(file=sys.stderr)
            self.err = e
            try:
                self.hdr[self.world + 1] = 1
            except Exception:
                pass
            self.free.release()
