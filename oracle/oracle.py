"""ctypes wrapper of liboracle.so — TEST INFRASTRUCTURE ONLY.

The CPU restatement of the reference renderer (oracle/oracle.cpp).  Imported only by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg, always as the checker / the CPU baseline,
never as the thing measured or shipped.  Parity status: UNPINNED against the reference binary (Rust,
unbuildable here, unseeded); pinned by the KAT fixtures of tests/golden (see oracle.cpp header).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.environ.get("ORACLE_LIB") or os.path.join(HERE, "liboracle.so")  # ORACLE_LIB: the ASan build (scripts/sanitize.sh)
COUNTERS = ["segments", "aabb", "sphere", "moving", "rect", "medium", "tex_solid", "tex_checker", "tex_noise", "tex_image", "samples", "pixels"]

_lib = None


def build() -> None:
    subprocess.check_call(["make", "-s", "-C", HERE])


def load() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB):
        build()
    L = ctypes.CDLL(LIB)
    vp, f, u32, u64, i32 = ctypes.c_void_p, ctypes.c_float, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
    L.oracle_last_error.restype = ctypes.c_char_p
    L.oracle_preset_build.restype = vp
    L.oracle_preset_build.argtypes = [i32, u64, vp, u32, u32, u32, vp]
    L.oracle_scene_destroy.argtypes = [vp]
    L.oracle_scene_count.restype = u32
    L.oracle_scene_count.argtypes = [vp]
    L.oracle_scene_bbox.restype = i32
    L.oracle_scene_bbox.argtypes = [vp, vp]
    L.oracle_render.restype = i32
    L.oracle_render.argtypes = [vp, u32, u32, u32, u32, u32, u64, f, u32, u32, u32, u32, vp, i32, vp]
    L.oracle_render_rows.restype = i32
    L.oracle_render_rows.argtypes = [vp, u32, u32, u32, u32, u32, u64, f, vp, u32, u32, u32, u32, vp, i32, vp]
    L.oracle_camera.argtypes = [vp, vp, f, f, f, f, f, i32, i32, vp]
    L.oracle_camera_ray.argtypes = [vp, vp, f, f, f, i32, i32, f, f, vp, f, vp]
    L.oracle_aabb_hit.restype = i32
    L.oracle_aabb_hit.argtypes = [vp, vp, vp, vp, f, f]
    L.oracle_prim_hit.restype = i32
    L.oracle_prim_hit.argtypes = [i32, vp, vp, f, f, vp]
    L.oracle_vec_op.argtypes = [i32, vp, vp, f, vp]
    L.oracle_perlin.restype = f
    L.oracle_perlin.argtypes = [vp, vp, i32, vp, u32]
    L.oracle_perlin_tables.argtypes = [u64, vp, vp]
    L.oracle_texture.argtypes = [i32, vp, f, f, f, vp, vp, vp, u32, u32, u32, vp]
    L.oracle_math.argtypes = [i32, vp, vp, vp, u32]
    L.oracle_math_libm.argtypes = [i32, vp, vp, vp, u32]
    L.oracle_set_libm.argtypes = [i32]
    L.oracle_record_math.argtypes = [vp, u32, vp]
    L.oracle_rng.argtypes = [u64, u32, u32, i32, u32, vp]
    _lib = L
    return L


def _p(a):
    return a.ctypes.data


class OracleScene:
    def __init__(self, preset: int, scene_seed: int = 1, image: np.ndarray | None = None):
        L = load()
        img = np.zeros((1, 1, 3), np.uint8) if image is None else np.ascontiguousarray(image, np.uint8)
        self._img = img
        info = np.zeros(16, np.float32)
        h, w, c = img.shape
        self.h = L.oracle_preset_build(preset, scene_seed, _p(img), w, h, c, _p(info))
        if not self.h:
            raise RuntimeError(L.oracle_last_error().decode())
        self.look_from, self.look_at = info[0:3].copy(), info[3:6].copy()
        self.fov, self.aperture, self.focus_dist, self.time0, self.time1 = [float(x) for x in info[6:11]]
        self.background = info[11:14].copy()
        self.n_media = int(info[14])

    def __del__(self):
        try:
            if self.h:
                load().oracle_scene_destroy(self.h)
        except Exception:
            pass

    def count(self) -> int:
        return load().oracle_scene_count(self.h)

    def bbox(self):
        b = np.zeros(6, np.float32)
        return b if load().oracle_scene_bbox(self.h, _p(b)) else None

    def render(self, width, height, spp, depth=50, seed=1, region=None, threads=8, sample_offset=0, t_min=0.001):
        x0, y0, w, h = region if region is not None else (0, 0, width, height)
        out = np.zeros((h, w, 4), np.float32)
        cnt = np.zeros(16, np.uint64)
        st = load().oracle_render(self.h, width, height, spp, depth, sample_offset, seed, t_min, x0, y0, w, h, _p(out), threads, _p(cnt))
        if st != 0:
            raise RuntimeError(load().oracle_last_error().decode())
        return out, dict(zip(COUNTERS, [int(c) for c in cnt[: len(COUNTERS)]]))

    def render_rows(self, width, height, spp, rows, depth=50, seed=1, threads=8, sample_offset=0, t_min=0.001,
                    x0=0, w=None, task_w=80):
        """Columns [x0, x0 + w) (default: all) of rows `rows` of the width x height frame, in tasks of
        task_w pixels: (len(rows), w, 4) f32 and counters."""
        r = np.ascontiguousarray(rows, np.uint32)
        w = width - x0 if w is None else w
        out = np.zeros((r.size, w, 4), np.float32)
        cnt = np.zeros(16, np.uint64)
        st = load().oracle_render_rows(self.h, width, height, spp, depth, sample_offset, seed, t_min, _p(r), r.size,
                                       x0, w, task_w, _p(out), threads, _p(cnt))
        if st != 0:
            raise RuntimeError(load().oracle_last_error().decode())
        return out, dict(zip(COUNTERS, [int(c) for c in cnt[: len(COUNTERS)]]))


def math(op: int, x: np.ndarray, y: np.ndarray | None = None) -> np.ndarray:
    x = np.ascontiguousarray(x, np.float32)
    out = np.zeros_like(x)
    yy = None if y is None else np.ascontiguousarray(y, np.float32)
    load().oracle_math(op, _p(x), None if yy is None else _p(yy), _p(out), x.size)
    return out


def math_libm(op: int, x: np.ndarray, y: np.ndarray | None = None) -> np.ndarray:
    """glibc's f32 function for op (0 sinf, 1 cosf, 2 acosf, 3 atan2f(x, y), 4 logf, 5 powf(x, 5), 6 tanf):
    the reference platform's arithmetic (Rust f32 methods call these on Linux)."""
    x = np.ascontiguousarray(x, np.float32)
    out = np.zeros_like(x)
    yy = None if y is None else np.ascontiguousarray(y, np.float32)
    load().oracle_math_libm(op, _p(x), None if yy is None else _p(yy), _p(out), x.size)
    return out


class libm_arithmetic:
    """Context manager: oracle renders and scene builds inside use glibc's f32 transcendentals."""

    def __enter__(self):
        load().oracle_set_libm(1)
        return self

    def __exit__(self, *exc):
        load().oracle_set_libm(0)
        return False


N_OPS = 7


def record_math(fn, cap: int = 1 << 22):
    """Run fn() (single-threaded oracle renders) and return {op: (n_calls, args[:min(n, cap), 2])}."""
    bufs = [np.zeros(2 * cap, np.float32) for _ in range(N_OPS)]
    ptrs = (ctypes.c_void_p * N_OPS)(*[b.ctypes.data for b in bufs])
    counts = np.zeros(N_OPS, np.uint32)
    L = load()
    L.oracle_record_math(ptrs, cap, None)
    try:
        fn()
    finally:
        L.oracle_record_math(None, 0, counts.ctypes.data)
    return {k: (int(counts[k]), bufs[k][: 2 * min(int(counts[k]), cap)].reshape(-1, 2)) for k in range(N_OPS)}
