"""hrt — Python binding of libhrt.so, the MI355X path-tracing inner loop.

Host side of the drop-in boundary (include/hrt/hrt.h) for tests, bench and scripts.  Names follow
the reference (SkillerRaptor/hyper-ray-tracer): Scene presets mirror `arguments::Scene`
(src/arguments.rs:9-19), `render()` replaces `Application::render` (src/application.rs:393-475).

The library is the HIP build in hyper-ray-tracer_amd/lib/libhrt.so; importing this module never
falls back to anything else: a missing library raises.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)
LIB_PATH = os.environ.get("HRT_LIB") or os.path.join(PKG_ROOT, "lib", "libhrt.so")  # HRT_LIB: A/B against another build

# ---------------------------------------------------------------------------------------- enums
OK = 0
ERR_INVALID_ARG, ERR_EMPTY, ERR_NO_BBOX, ERR_NAN, ERR_STATE, ERR_HIP, ERR_OOM, ERR_UNSUPPORTED = range(1, 9)
PLANE_XY, PLANE_YZ, PLANE_ZX = 0, 1, 2
AXIS_X, AXIS_Y, AXIS_Z = 0, 1, 2

PRESETS = {
    "random": 0,
    "two_spheres": 1,
    "two_perlin_spheres": 2,
    "earth": 3,
    "simple_light": 4,
    "cornell": 5,
    "cornell_smoke": 6,
    "final": 7,
    "earth_perlin": 8,
    "random_10k": 9,
    "features": 10,
    "random_40k": 11,  # build-defined: 39.9k leaves, the device-built walk hierarchy by default
    "motion": 12,  # build-defined: moving spheres with their own shutter intervals (no scene-wide factor)
}


class HrtError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"hrt status {status}: {msg}")
        self.status = status


# ---------------------------------------------------------------------------------------- structs
class Camera(ctypes.Structure):
    _fields_ = [
        ("origin", ctypes.c_float * 3),
        ("lower_left_corner", ctypes.c_float * 3),
        ("horizontal", ctypes.c_float * 3),
        ("vertical", ctypes.c_float * 3),
        ("u", ctypes.c_float * 3),
        ("v", ctypes.c_float * 3),
        ("w", ctypes.c_float * 3),
        ("lens_radius", ctypes.c_float),
        ("time0", ctypes.c_float),
        ("time1", ctypes.c_float),
    ]


class RenderParams(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_uint32),
        ("height", ctypes.c_uint32),
        ("samples", ctypes.c_uint32),
        ("max_depth", ctypes.c_uint32),
        ("sample_offset", ctypes.c_uint32),
        ("flags", ctypes.c_uint32),
        ("t_min", ctypes.c_float),
        ("background", ctypes.c_float * 3),
        ("seed", ctypes.c_uint64),
    ]


class Tile(ctypes.Structure):
    _fields_ = [("x", ctypes.c_uint32), ("y", ctypes.c_uint32), ("w", ctypes.c_uint32), ("h", ctypes.c_uint32)]


class RenderStats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in ("segments", "samples", "pixels", "node_visits", "prim_tests", "tex_evals",
                                                      "walk_slots", "shade_slots", "prim_slots")] + \
        [("phase_cycles", ctypes.c_uint64 * 3), ("park_slots", ctypes.c_uint64), ("wait_slots", ctypes.c_uint64),
         ("leaf_cycles", ctypes.c_uint64), ("walk_steps", ctypes.c_uint64)]


class TilePixels(ctypes.Structure):
    """hrt_tile_pixels (include/hrt/hrt.h)."""
    _fields_ = [("x", ctypes.c_uint32), ("y", ctypes.c_uint32), ("width", ctypes.c_uint32),
                ("height", ctypes.c_uint32), ("pixels", ctypes.POINTER(ctypes.c_float))]


TILE_FN = ctypes.CFUNCTYPE(None, ctypes.POINTER(TilePixels), ctypes.c_void_p)


class BlobInfo(ctypes.Structure):
    """hrt_blob_info (include/hrt/hrt.h)."""
    _fields_ = [(n, ctypes.c_uint64) for n in ("off_nodes", "off_prims", "off_insts", "off_media", "off_mats", "off_texs",
                                                "off_perlin", "off_images")] + \
        [(n, ctypes.c_uint32) for n in ("n_nodes", "main_end", "n_prims", "feature_mask", "cull_mode", "motion_uniform")] + \
        [("motion_t0", ctypes.c_float), ("motion_span", ctypes.c_float), ("ln_e", ctypes.c_float),
         ("media_nested", ctypes.c_uint32), ("box_t0", ctypes.c_float), ("box_t1", ctypes.c_float),
         ("off_walk", ctypes.c_uint64), ("walk_bytes", ctypes.c_uint32), ("walk_regrouped", ctypes.c_uint32),
         ("bvh_tied_sorts", ctypes.c_uint32), ("walk_hot", ctypes.c_uint32),
                ("walk_general", ctypes.c_uint32), ("off_chains", ctypes.c_uint64),
        ("walk_half", ctypes.c_uint32), ("walk_c16", ctypes.c_uint32), ("walk_nodes", ctypes.c_uint32),
        ("walk_pbase", ctypes.c_uint32)]


class PresetInfo(ctypes.Structure):
    _fields_ = [
        ("look_from", ctypes.c_float * 3),
        ("look_at", ctypes.c_float * 3),
        ("fov", ctypes.c_float),
        ("aperture", ctypes.c_float),
        ("focus_dist", ctypes.c_float),
        ("time0", ctypes.c_float),
        ("time1", ctypes.c_float),
        ("background", ctypes.c_float * 3),
        ("root", ctypes.c_uint32),
    ]


class SceneInfo(ctypes.Structure):
    _fields_ = [
        (n, ctypes.c_uint32)
        for n in ("nodes", "prims", "materials", "textures", "instances", "media", "feature_mask", "blob_bytes", "in_lds",
                  "cull_mode", "sah_stream_len", "bvh_tied_sorts", "walk_regrouped", "walk_device_built", "walk_build_us")
    ]


class LaunchInfo(ctypes.Structure):
    """hrt_launch_info: the last render launch of the calling thread (hrt_last_launch)."""
    _fields_ = [("kernel", ctypes.c_char * 160)] + [
        (n, ctypes.c_uint32) for n in ("grid", "block", "blocks_per_cu", "cus", "waves_per_simd", "vgprs", "scratch_bytes",
                                       "lds_bytes")
    ] + [("knobs", ctypes.c_char * 256)]


class SceneOptions(ctypes.Structure):
    """hrt_scene_options: the explicit configuration that can change an image's bits (all-zero = default)."""
    _fields_ = [(n, ctypes.c_uint32) for n in ("bvh_ties", "walk_tree", "chunk_min", "chunk_max", "chunk_uniform")]


# Diagnostics an older build may lack; only tolerated when HRT_LIB points at another build (A/B runs)
OPTIONAL = {"hrt_abi_version", "hrt_last_launch", "hrt_debug_box_test", "hrt_scene_set_options", "hrt_scene_get_options",
            "hrt_debug_sample_chunks", "hrt_scene_set_view"}
HRT_LIB_OVERRIDE = bool(os.environ.get("HRT_LIB"))

# Every entry point of include/hrt/hrt.h (tests/test_abi.py checks the header against this list).
EXPORTS = [
    "hrt_last_error", "hrt_version", "hrt_abi_version", "hrt_scene_create", "hrt_scene_destroy",
    "hrt_tex_solid", "hrt_tex_checker", "hrt_tex_noise", "hrt_tex_image",
    "hrt_mat_lambertian", "hrt_mat_metal", "hrt_mat_dielectric", "hrt_mat_diffuse_light", "hrt_mat_isotropic",
    "hrt_node_sphere", "hrt_node_moving_sphere", "hrt_node_rect", "hrt_node_cuboid", "hrt_node_translate",
    "hrt_node_rotate", "hrt_node_constant_medium", "hrt_node_list", "hrt_node_bvh", "hrt_node_count",
    "hrt_node_bounding_box", "hrt_scene_set_root", "hrt_scene_commit", "hrt_preset_build", "hrt_camera_init",
    "hrt_render_tiles_device", "hrt_render_device", "hrt_render", "hrt_tile_grid", "hrt_scene_get_info", "hrt_last_launch", "hrt_debug_box_test",
    "hrt_debug_device_math", "hrt_debug_trace_path", "hrt_debug_scene_blob", "hrt_image_write", "hrt_render_progressive", "hrt_debug_prim_record",
    "hrt_scene_synchronize", "hrt_debug_poke_blob", "hrt_scene_set_options", "hrt_scene_get_options",
    "hrt_debug_sample_chunks", "hrt_scene_set_view",
]

ABI_VERSION = 6  # include/hrt/hrt.h HRT_ABI_VERSION: the struct layouts below
_lib = None
_U32P = ctypes.POINTER(ctypes.c_uint32)
_F3 = ctypes.c_float * 3


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libhrt.so (raises if it has not been built: there is no fallback path)."""
    global _lib
    if _lib is not None:
        return _lib
    # torch ships its own libamdhip64 (same soname libamdhip64.so.7 as /opt/rocm's).  Loading torch
    # first makes libhrt bind to that already-loaded runtime: ONE HIP runtime per process, so torch
    # device pointers and hipStream_t handles are valid in libhrt.  (Loaded the other way round,
    # torch would map a second runtime by file name and fail to find the device.)
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path} missing: build it with `make -C hyper-ray-tracer_amd` (or __graft_entry__.build())")
    L = ctypes.CDLL(path)
    S = ctypes.c_int32
    vp = ctypes.c_void_p
    f, u32, i32, u64 = ctypes.c_float, ctypes.c_uint32, ctypes.c_int32, ctypes.c_uint64
    sig = {
        "hrt_last_error": (ctypes.c_char_p, []),
        "hrt_version": (ctypes.c_char_p, []),
        "hrt_abi_version": (ctypes.c_uint32, []),
        "hrt_scene_create": (S, [ctypes.POINTER(vp)]),
        "hrt_scene_destroy": (None, [vp]),
        "hrt_tex_solid": (S, [vp, f, f, f, _U32P]),
        "hrt_tex_checker": (S, [vp, u32, u32, _U32P]),
        "hrt_tex_noise": (S, [vp, f, vp, vp, _U32P]),
        "hrt_tex_image": (S, [vp, vp, u32, u32, u32, _U32P]),
        "hrt_mat_lambertian": (S, [vp, u32, _U32P]),
        "hrt_mat_metal": (S, [vp, f, f, f, f, _U32P]),
        "hrt_mat_dielectric": (S, [vp, f, _U32P]),
        "hrt_mat_diffuse_light": (S, [vp, u32, _U32P]),
        "hrt_mat_isotropic": (S, [vp, u32, _U32P]),
        "hrt_node_sphere": (S, [vp, _F3, f, u32, _U32P]),
        "hrt_node_moving_sphere": (S, [vp, _F3, _F3, f, f, f, u32, _U32P]),
        "hrt_node_rect": (S, [vp, i32, f, f, f, f, f, u32, _U32P]),
        "hrt_node_cuboid": (S, [vp, _F3, _F3, u32, _U32P]),
        "hrt_node_translate": (S, [vp, u32, _F3, _U32P]),
        "hrt_node_rotate": (S, [vp, i32, u32, f, _U32P]),
        "hrt_node_constant_medium": (S, [vp, u32, f, u32, _U32P]),
        "hrt_node_list": (S, [vp, vp, u32, _U32P]),
        "hrt_node_bvh": (S, [vp, vp, u32, f, f, _U32P]),
        "hrt_node_count": (S, [vp, u32, _U32P]),
        "hrt_node_bounding_box": (S, [vp, u32, f, f, ctypes.POINTER(i32), _F3, _F3]),
        "hrt_scene_set_root": (S, [vp, u32]),
        "hrt_scene_commit": (S, [vp, i32]),
        "hrt_preset_build": (S, [vp, i32, u64, vp, u32, u32, u32, ctypes.POINTER(PresetInfo)]),
        "hrt_camera_init": (S, [ctypes.POINTER(Camera), _F3, _F3, f, f, f, f, f, i32, i32]),
        "hrt_render_tiles_device": (S, [vp, ctypes.POINTER(Camera), ctypes.POINTER(RenderParams), vp, u32, vp, vp, ctypes.POINTER(RenderStats)]),
        "hrt_render_device": (S, [vp, ctypes.POINTER(Camera), ctypes.POINTER(RenderParams), u32, u32, u32, u32, vp, vp, ctypes.POINTER(RenderStats)]),
        "hrt_render": (S, [vp, ctypes.POINTER(Camera), ctypes.POINTER(RenderParams), u32, u32, u32, u32, vp, ctypes.POINTER(RenderStats)]),
        "hrt_tile_grid": (S, [u32, u32, u32, u32, u32, vp, u32, _U32P]),
        "hrt_scene_get_info": (S, [vp, ctypes.POINTER(SceneInfo)]),
        "hrt_last_launch": (S, [ctypes.POINTER(LaunchInfo)]),
        "hrt_debug_box_test": (S, [ctypes.c_int32, ctypes.c_int32, vp, ctypes.c_uint32, vp, ctypes.c_uint32, ctypes.c_float,
                                   ctypes.c_float, vp]),
        "hrt_debug_device_math": (S, [i32, vp, vp, vp, u32]),
        "hrt_debug_scene_blob": (S, [vp, vp, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(BlobInfo)]),
        "hrt_debug_prim_record": (S, [vp, i32, u32, vp]),
        "hrt_image_write": (S, [ctypes.c_char_p, vp, u32, u32, i32]),
        "hrt_render_progressive": (S, [vp, ctypes.POINTER(Camera), ctypes.POINTER(RenderParams), u32, u32, u32, u32,
                                       TILE_FN, vp, ctypes.POINTER(RenderStats)]),
        "hrt_debug_trace_path": (S, [vp, ctypes.POINTER(Camera), ctypes.POINTER(RenderParams), u32, u32, u32, u32, vp, _U32P]),
        "hrt_scene_synchronize": (S, [vp]),
        "hrt_debug_poke_blob": (S, [vp, u64, vp, u64]),
        "hrt_scene_set_options": (S, [vp, ctypes.POINTER(SceneOptions)]),
        "hrt_scene_get_options": (S, [vp, ctypes.POINTER(SceneOptions)]),
        "hrt_scene_set_view": (S, [vp, ctypes.POINTER(Camera)]),
        "hrt_debug_sample_chunks": (S, [vp, ctypes.POINTER(RenderParams), _U32P]),
    }
    for name, (res, args) in sig.items():
        if name in OPTIONAL and HRT_LIB_OVERRIDE and not hasattr(L, name):
            continue  # an older build loaded for an A/B run (HRT_LIB): diagnostics it lacks stay unbound
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    if hasattr(L, "hrt_abi_version") and L.hrt_abi_version() != ABI_VERSION and not HRT_LIB_OVERRIDE:
        raise RuntimeError(f"{path}: ABI version {L.hrt_abi_version()}, this binding is written for {ABI_VERSION} "
                           "(include/hrt/hrt.h HRT_ABI_VERSION): rebuild the library")
    _lib = L
    return L


def _check(st: int) -> None:
    if st != OK:
        raise HrtError(st, load().hrt_last_error().decode())


def f3(v: Sequence[float]):
    return _F3(*[float(x) for x in v])


# ---------------------------------------------------------------------------------------- scene
class Scene:
    """A hrt_scene handle: constructors mirror the reference's Hittable/Material/Texture types."""

    def __init__(self):
        L = load()
        h = ctypes.c_void_p()
        _check(L.hrt_scene_create(ctypes.byref(h)))
        self.h = h
        self.info: Optional[PresetInfo] = None
        self._keep: list = []

    def close(self):
        if self.h:
            load().hrt_scene_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _id(self, fn, *args) -> int:
        out = ctypes.c_uint32()
        _check(fn(self.h, *args, ctypes.byref(out)))
        return out.value

    # textures
    def solid(self, r, g, b):
        return self._id(load().hrt_tex_solid, r, g, b)

    def checker(self, odd, even):
        return self._id(load().hrt_tex_checker, odd, even)

    def noise(self, scale, ranvec, perm):
        rv = np.ascontiguousarray(ranvec, np.float32).reshape(-1)
        pm = np.ascontiguousarray(perm, np.uint32).reshape(-1)
        assert rv.size == 768 and pm.size == 768
        return self._id(load().hrt_tex_noise, scale, rv.ctypes.data, pm.ctypes.data)

    def image(self, data: Optional[np.ndarray]):
        if data is None:
            return self._id(load().hrt_tex_image, None, 0, 0, 0)
        d = np.ascontiguousarray(data, np.uint8)
        h, w, c = d.shape
        return self._id(load().hrt_tex_image, d.ctypes.data, w, h, c)

    # materials
    def lambertian(self, tex):
        return self._id(load().hrt_mat_lambertian, tex)

    def metal(self, albedo, fuzz):
        return self._id(load().hrt_mat_metal, *[float(a) for a in albedo], fuzz)

    def dielectric(self, ior):
        return self._id(load().hrt_mat_dielectric, ior)

    def diffuse_light(self, tex):
        return self._id(load().hrt_mat_diffuse_light, tex)

    def isotropic(self, tex):
        return self._id(load().hrt_mat_isotropic, tex)

    # hittables
    def sphere(self, center, radius, mat):
        return self._id(load().hrt_node_sphere, f3(center), radius, mat)

    def moving_sphere(self, c0, c1, t0, t1, radius, mat):
        return self._id(load().hrt_node_moving_sphere, f3(c0), f3(c1), t0, t1, radius, mat)

    def rect(self, plane, a0, a1, b0, b1, k, mat):
        return self._id(load().hrt_node_rect, plane, a0, a1, b0, b1, k, mat)

    def cuboid(self, p0, p1, mat):
        return self._id(load().hrt_node_cuboid, f3(p0), f3(p1), mat)

    def translate(self, child, d):
        return self._id(load().hrt_node_translate, child, f3(d))

    def rotate(self, axis, child, angle):
        return self._id(load().hrt_node_rotate, axis, child, angle)

    def constant_medium(self, boundary, density, tex):
        return self._id(load().hrt_node_constant_medium, boundary, density, tex)

    def list(self, children: Sequence[int]):
        arr = (ctypes.c_uint32 * max(1, len(children)))(*children)
        return self._id(load().hrt_node_list, ctypes.cast(arr, ctypes.c_void_p), len(children))

    def bvh(self, children: Sequence[int], t0=0.0, t1=1.0):
        arr = (ctypes.c_uint32 * max(1, len(children)))(*children)
        return self._id(load().hrt_node_bvh, ctypes.cast(arr, ctypes.c_void_p), len(children), t0, t1)

    def count(self, node) -> int:
        out = ctypes.c_uint32()
        _check(load().hrt_node_count(self.h, node, ctypes.byref(out)))
        return out.value

    def bounding_box(self, node, t0=0.0, t1=1.0):
        has = ctypes.c_int32()
        mn, mx = _F3(), _F3()
        _check(load().hrt_node_bounding_box(self.h, node, t0, t1, ctypes.byref(has), mn, mx))
        return (tuple(mn), tuple(mx)) if has.value else None

    def set_options(self, **kw):
        """hrt_scene_set_options: bvh_ties (0 stable / 1 reversed), walk_tree (0 re-grouped / 1 the reference tree),
        chunk_min, chunk_max, chunk_uniform (sample chunks); unnamed fields keep their current values."""
        o = self.options()
        for k, v in kw.items():
            if k not in dict(SceneOptions._fields_):
                raise TypeError(f"unknown scene option {k!r}")
            setattr(o, k, int(v))
        _check(load().hrt_scene_set_options(self.h, ctypes.byref(o)))

    def set_view(self, cam: Optional["Camera"]):
        """hrt_scene_set_view: the camera most renders will use (None: no hint).  Placement only: which node parts
        of a walk stream too large for LDS are staged there; the image is the same bit for bit."""
        if cam is not None:
            self._keep.append(cam)
        _check(load().hrt_scene_set_view(self.h, ctypes.byref(cam) if cam is not None else None))

    def options(self) -> SceneOptions:
        o = SceneOptions()
        _check(load().hrt_scene_get_options(self.h, ctypes.byref(o)))
        return o

    def set_root(self, node):
        _check(load().hrt_scene_set_root(self.h, node))

    def commit(self, device: int = -1):
        _check(load().hrt_scene_commit(self.h, device))

    def synchronize(self):
        """Wait for every render launched on this scene; raises HrtError(ERR_STATE) if one of them
        was stopped by the walk watchdog (hrt_scene_synchronize)."""
        _check(load().hrt_scene_synchronize(self.h))

    def poke_blob(self, offset: int, data: bytes):
        """Fault injection: overwrite bytes of the committed device blob (hrt_debug_poke_blob)."""
        buf = ctypes.create_string_buffer(bytes(data), len(data))
        _check(load().hrt_debug_poke_blob(self.h, offset, buf, len(data)))

    def scene_info(self) -> SceneInfo:
        si = SceneInfo()
        _check(load().hrt_scene_get_info(self.h, ctypes.byref(si)))
        return si


def synthetic_earth(width: int = 1024, height: int = 512) -> np.ndarray:
    """Deterministic stand-in for assets/earthmap.jpg (same shape, RGB8): the asset is not shipped,
    so Earth-textured scenes use this image on both sides of every parity test."""
    y, x = np.mgrid[0:height, 0:width].astype(np.float64)
    lon = x / width * 2 * np.pi
    lat = (y / height - 0.5) * np.pi
    land = (np.sin(3 * lon) * np.cos(2 * lat) + 0.5 * np.sin(7 * lon + 1.3) * np.sin(5 * lat)) > 0.2
    r = np.where(land, 90 + 60 * np.cos(lat), 20)
    g = np.where(land, 120 + 50 * np.sin(2 * lon) ** 2, 60 + 40 * np.cos(lat))
    b = np.where(land, 50, 140 + 80 * np.cos(lat))
    ice = np.abs(lat) > 1.25
    img = np.stack([np.where(ice, 240, r), np.where(ice, 245, g), np.where(ice, 250, b)], -1)
    return np.clip(img, 0, 255).astype(np.uint8)


def load_image(path: str) -> np.ndarray:
    """Decode an image file to the bytes hrt_tex_image takes (H x W x C uint8), as ImageTexture::new
    does with `image::open` (image_texture.rs:19-33).  Decoding is host plumbing (Pillow here; the
    Rust host keeps `image`): the ABI itself takes decoded bytes."""
    from PIL import Image

    im = Image.open(path)
    if im.mode not in ("L", "LA", "RGB", "RGBA"):
        im = im.convert("RGB")
    a = np.asarray(im, dtype=np.uint8)
    return np.ascontiguousarray(a[..., None] if a.ndim == 2 else a)


def preset(name_or_id, scene_seed: int = 1, image: Optional[np.ndarray] = None, options: Optional[dict] = None) -> Scene:
    """Build one of the reference scenes (application.rs:497-935) with a seeded builder stream; `options` are
    hrt_scene_options fields, set before the builder runs (bvh_ties applies to its BvhNode::new calls)."""
    pid = PRESETS[name_or_id] if isinstance(name_or_id, str) else int(name_or_id)
    img = synthetic_earth() if image is None else np.ascontiguousarray(image, np.uint8)
    s = Scene()
    if options:
        s.set_options(**options)
    info = PresetInfo()
    h, w, c = img.shape
    _check(load().hrt_preset_build(s.h, pid, scene_seed, img.ctypes.data, w, h, c, ctypes.byref(info)))
    s.info = info
    s._keep.append(img)
    return s


def camera(look_from, look_at, fov, aperture, focus_dist, time0, time1, width, height) -> Camera:
    cam = Camera()
    _check(load().hrt_camera_init(ctypes.byref(cam), f3(look_from), f3(look_at), fov, aperture, focus_dist, time0, time1, width, height))
    return cam


def preset_camera(info: PresetInfo, width: int, height: int) -> Camera:
    return camera(info.look_from, info.look_at, info.fov, info.aperture, info.focus_dist, info.time0, info.time1, width, height)


RENDER_COUNT_WORK = 1
RENDER_NO_LDS = 2
RENDER_REFERENCE_CULL = 8
RENDER_FAST_CULL = 16
RENDER_SAH = 32


def params(width, height, samples, max_depth=50, seed=1, background=(0.7, 0.8, 1.0), t_min=0.001, sample_offset=0, flags=0) -> RenderParams:
    p = RenderParams()
    p.width, p.height, p.samples, p.max_depth = width, height, samples, max_depth
    p.sample_offset, p.flags, p.t_min, p.seed = sample_offset, flags, t_min, seed
    for i in range(3):
        p.background[i] = float(background[i])
    return p


def tile_grid(width: int, height: int, tile_size: int = 80, rank: int = 0, world: int = 1) -> List[Tuple[int, int, int, int]]:
    """Reference tile grid (application.rs:363-364, 404-430) split round-robin over `world` ranks."""
    L = load()
    n = ctypes.c_uint32()
    _check(L.hrt_tile_grid(width, height, tile_size, rank, world, None, 0, ctypes.byref(n)))
    arr = (Tile * max(1, n.value))()
    _check(L.hrt_tile_grid(width, height, tile_size, rank, world, ctypes.cast(arr, ctypes.c_void_p), n.value, ctypes.byref(n)))
    return [(t.x, t.y, t.w, t.h) for t in arr[: n.value]]


def render(scene: Scene, cam: Camera, p: RenderParams, region=None, stats: bool = False):
    """Render a region into host memory (synchronous); returns (h, w, 4) float32 [, RenderStats]."""
    x0, y0, w, h = region if region is not None else (0, 0, p.width, p.height)
    out = np.zeros((h, w, 4), np.float32)
    st = RenderStats()
    _check(load().hrt_render(scene.h, ctypes.byref(cam), ctypes.byref(p), x0, y0, w, h, out.ctypes.data, ctypes.byref(st)))
    return (out, st) if stats else out


def render_tiles_device(scene: Scene, cam: Camera, p: RenderParams, tiles, d_out_ptr: int, stream_ptr: int = 0, want_stats: bool = False):
    """Asynchronous render of a tile list into device memory (tiles packed back to back)."""
    arr = (Tile * len(tiles))(*[Tile(*t) for t in tiles])
    st = RenderStats()
    _check(load().hrt_render_tiles_device(scene.h, ctypes.byref(cam), ctypes.byref(p), ctypes.cast(arr, ctypes.c_void_p), len(tiles),
                                          ctypes.c_void_p(d_out_ptr), ctypes.c_void_p(stream_ptr), ctypes.byref(st) if want_stats else None))
    return st if want_stats else None


def last_launch() -> Optional[dict]:
    """The calling thread's last render launch (hrt_last_launch): kernel, grid, occupancy, VGPRs, scratch, LDS, and
    the library's A/B environment knobs set in this process.  None with an older build that lacks the entry
    point (an A/B run through HRT_LIB)."""
    L = load()
    if not hasattr(L, "hrt_last_launch"):
        return None
    li = LaunchInfo()
    _check(L.hrt_last_launch(ctypes.byref(li)))
    d = {n: getattr(li, n) for n, _ in LaunchInfo._fields_[1:-1]}
    d["kernel"] = li.kernel.decode()
    d["knobs"] = li.knobs.decode()
    d["waves"] = li.grid * li.block // 64
    return d


def box_test(form: int, boxes: np.ndarray, rays: np.ndarray, tmin: float, tmax: float, on_device: bool = True) -> np.ndarray:
    """hrt_debug_box_test: (n_boxes, n_rays) uint8 pass flags of the walk's inflated box test (form 0 / 1)."""
    b = np.ascontiguousarray(boxes, np.float32).reshape(-1, 8)
    r = np.ascontiguousarray(rays, np.float32).reshape(-1, 6)
    out = np.zeros((len(b), len(r)), np.uint8)
    _check(load().hrt_debug_box_test(form, 1 if on_device else 0, b.ctypes.data, len(b), r.ctypes.data, len(r), tmin, tmax,
                                     out.ctypes.data))
    return out


def device_math(op: int, x: np.ndarray, y: Optional[np.ndarray] = None) -> np.ndarray:
    x = np.ascontiguousarray(x, np.float32)
    out = np.zeros_like(x)
    yy = None if y is None else np.ascontiguousarray(y, np.float32)
    _check(load().hrt_debug_device_math(op, x.ctypes.data, None if yy is None else yy.ctypes.data, out.ctypes.data, x.size))
    return out


def trace_path(scene: Scene, cam: Camera, p: RenderParams, x: int, y: int, sample: int, max_segments: int = 64):
    """Device trace of one path: list of (origin, direction, time, t, winner) per segment, radiance."""
    out = np.zeros(9 * max_segments + 3, np.float32)
    n = ctypes.c_uint32()
    _check(load().hrt_debug_trace_path(scene.h, ctypes.byref(cam), ctypes.byref(p), x, y, sample, max_segments, out.ctypes.data, ctypes.byref(n)))
    segs = []
    for i in range(min(n.value, max_segments)):
        r = out[9 * i:9 * i + 9]
        segs.append((r[0:3].copy(), r[3:6].copy(), float(r[6]), float(r[7]), int(r[8:9].view(np.uint32)[0])))
    return segs, out[9 * max_segments:9 * max_segments + 3].copy()


IMAGE_PFM, IMAGE_PPM = 0, 1


def write_image(path: str, rgba: np.ndarray, fmt: Optional[int] = None) -> None:
    """Write a render result ((h, w, 4) f32, row 0 = bottom) as PFM (exact floats) or 8-bit PPM;
    the format follows the extension unless given."""
    img = np.ascontiguousarray(rgba, np.float32)
    if img.ndim != 3 or img.shape[2] != 4:
        raise ValueError("expected an (h, w, 4) float32 frame")
    if fmt is None:
        fmt = IMAGE_PPM if str(path).lower().endswith(".ppm") else IMAGE_PFM
    _check(load().hrt_image_write(str(path).encode(), img.ctypes.data, img.shape[1], img.shape[0], fmt))


def read_pfm(path: str) -> np.ndarray:
    """Read a PFM written by write_image back into an (h, w, 3) float32 array (row 0 = bottom)."""
    with open(path, "rb") as f:
        assert f.readline().strip() == b"PF"
        w, h = (int(v) for v in f.readline().split())
        scale = float(f.readline())
        data = np.frombuffer(f.read(), "<f4" if scale < 0 else ">f4")
    return data.reshape(h, w, 3).astype(np.float32)


class TileMessage:
    """application.rs:45-52 Tile (the mpsc message): tile-grid position, size, and (height, width, 4)
    RGBA pixels (row 0 = bottom)."""

    def __init__(self, x, y, width, height, pixels):
        self.x, self.y, self.width, self.height, self.pixels = x, y, width, height, pixels


def render_progressive(scene: "Scene", cam: Camera, p: RenderParams, on_tile, tile_size: int = 80, rank: int = 0,
                       world: int = 1, batch: int = 64, stats: bool = False):
    """Application::render with progressive delivery: on_tile(TileMessage) is called for every tile of this
    rank's share of the grid, batch by batch, while the next batch renders (hrt_render_progressive)."""
    err = []

    def cb(tp, _user):
        try:
            t = tp.contents
            px = np.ctypeslib.as_array(t.pixels, shape=(t.height * t.width * 4,)).reshape(t.height, t.width, 4).copy()
            on_tile(TileMessage(t.x, t.y, t.width, t.height, px))
        except BaseException as e:  # noqa: BLE001 - re-raised after the C call returns
            err.append(e)

    fn = TILE_FN(cb)
    st = RenderStats()
    _check(load().hrt_render_progressive(scene.h, ctypes.byref(cam), ctypes.byref(p), tile_size, rank, world, batch,
                                         fn, None, ctypes.byref(st) if stats else None))
    if err:
        raise err[0]
    return st if stats else None


def sample_chunks(scene: "Scene", p: RenderParams) -> dict:
    """hrt_debug_sample_chunks: the chunk schedule a render of `p` would sum each pixel's samples in."""
    out = (ctypes.c_uint32 * 4)()
    _check(load().hrt_debug_sample_chunks(scene.h, ctypes.byref(p), out))
    return {"chunk": out[0], "head": out[1], "first": out[2], "tail": out[3]}


def scene_blob(scene: "Scene"):
    """The flattened scene (layout.h) as the kernels see it, without a device: (bytes, BlobInfo)."""
    size = ctypes.c_uint64()
    info = BlobInfo()
    _check(load().hrt_debug_scene_blob(scene.h, None, 0, ctypes.byref(size), ctypes.byref(info)))
    buf = ctypes.create_string_buffer(size.value)
    _check(load().hrt_debug_scene_blob(scene.h, buf, size.value, ctypes.byref(size), ctypes.byref(info)))
    return buf, info


def prim_record(scene: Scene, index: int, order: int = 0) -> np.ndarray:
    out = np.zeros(12, np.float32)
    _check(load().hrt_debug_prim_record(scene.h, order, index, out.ctypes.data))
    return out
