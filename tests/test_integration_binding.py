"""INTEGRATION.md's Rust binding (`hrt-sys`, section 1) against include/hrt/hrt.h, so that the documented
reference-side binding cannot drift from the C ABI it binds:
  - every `typedef struct` of the header is a `#[repr(C)]` struct of the same name, with the same fields
    in the same order and the corresponding Rust types;
  - the C sizes and field offsets (a C program compiled with gcc prints them) equal those of the Rust
    declarations laid out by C rules (ctypes), and those of the Python binding's ctypes classes;
  - every function the header declares is in the `extern "C"` block, with the same parameter and return
    types (names may differ), and the block declares nothing else.
No Rust toolchain exists in this image, so the Rust text is checked by parsing, not by rustc."""
import ctypes
import os
import re
import subprocess

import pytest
from conftest import tool_env

import hrt

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "hrt", "hrt.h")
DOC = os.path.join(ROOT, "INTEGRATION.md")

C_BASE = {"uint32_t": "u32", "int32_t": "i32", "uint64_t": "u64", "float": "f32", "uint8_t": "u8", "char": "c_char",
          "void": "c_void", "size_t": "usize", "hrt_status": "hrt_status", "hrt_tile_fn": "hrt_tile_fn"}


def _norm(t):
    t = re.sub(r"\s+", " ", t.strip())
    t = re.sub(r"\s*;\s*", "; ", t)
    t = re.sub(r"\[\s*", "[", t)
    return re.sub(r"\s*\]", "]", t)


def _c_type(decl, param):
    """(name, Rust spelling) of one C declarator: `const float center[3]` (a parameter: *const f32)."""
    m = re.match(r"^(const\s+)?([A-Za-z_]\w*)\s*(\**)\s*([A-Za-z_]\w*)?\s*(\[\s*(\d+)\s*\])?$", decl.strip())
    assert m, decl
    const, base, stars, name, arr, n = m.group(1), m.group(2), m.group(3), m.group(4), m.group(5), m.group(6)
    rust = C_BASE.get(base, base)
    if arr and not param:
        return name, f"[{rust}; {n}]"
    depth = len(stars) + (1 if arr else 0)
    for level in range(depth):
        rust = ("*const " if (const and level == 0) else "*mut ") + rust
    return name, _norm(rust)


def header_api():
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    structs = {}
    for name, body in re.findall(r"typedef struct (\w+) \{(.*?)\} \1;", src, flags=re.S):
        fields = []
        for stmt in filter(None, (x.strip() for x in body.split(";"))):
            head, *more = [x.strip() for x in stmt.split(",")]
            base = re.match(r"^((?:const\s+)?[A-Za-z_]\w*\s*\**)", head).group(1)
            fields.append(_c_type(head, False))
            for extra in more:
                fields.append(_c_type(base + " " + extra, False))
        structs[name] = fields
    fns = {}
    for ret, name, args in re.findall(r"^\s*((?:const\s+)?\w+\s*\**)\s*(hrt_\w+)\s*\(([^;]*?)\);", src, flags=re.M | re.S):
        args = " ".join(args.split())
        params = [] if args == "void" else [_c_type(a, True)[1] for a in args.split(",")]
        r = ret.strip()
        rt = None if r == "void" else _c_type(r + " x", True)[1]
        fns[name] = (params, rt)
    return structs, fns


def doc_api():
    text = open(DOC).read()
    sec = text[text.index("## 1."):text.index("## 2.")]
    block = sec[sec.index("```rust") + 7:sec.index("```", sec.index("```rust") + 7)]
    block = re.sub(r"//[^\n]*", "", block)
    structs = {}
    for name, body in re.findall(r"pub struct (\w+)\s*\{(.*?)\}", block, flags=re.S):
        if name == "hrt_scene":
            continue
        fields = []
        for part in re.split(r",(?![^\[]*\])", body):
            part = part.strip()
            if not part:
                continue
            m = re.match(r"^pub (\w+):\s*(.+)$", part, flags=re.S)
            assert m, part
            fields.append((m.group(1), _norm(m.group(2))))
        structs[name] = fields
    ext = block[block.index('extern "C" {'):]
    fns = {}
    for name, args, ret in re.findall(r"pub fn (\w+)\s*\((.*?)\)\s*(?:->\s*([^;]+))?;", ext, flags=re.S):
        params = [_norm(a.split(":", 1)[1]) for a in (x.strip() for x in args.split(",")) if a]
        fns[name] = (params, _norm(ret) if ret else None)
    return structs, fns, block


def test_rust_structs_match_header():
    hs, _ = header_api()
    ds, _, _ = doc_api()
    assert len(hs) >= 8
    assert sorted(ds) == sorted(hs)
    for name, fields in hs.items():
        assert ds[name] == fields, (name, ds[name], fields)


def test_rust_extern_block_matches_header():
    _, hf = header_api()
    _, df, block = doc_api()
    assert sorted(df) == sorted(hf)
    for name, (params, ret) in hf.items():
        assert df[name] == (params, ret), (name, df[name], (params, ret))
    assert re.search(r"pub type hrt_tile_fn = Option<unsafe extern \"C\" fn\(\w+: \*const hrt_tile_pixels, \w+: \*mut c_void\)>;",
                     block)


RUST_CTYPES = {"u32": ctypes.c_uint32, "i32": ctypes.c_int32, "u64": ctypes.c_uint64, "f32": ctypes.c_float,
               "u8": ctypes.c_uint8, "c_char": ctypes.c_char}


def _ctype_of(rust):
    m = re.match(r"^\[(\w+); (\d+)\]$", rust)
    if m:
        return RUST_CTYPES[m.group(1)] * int(m.group(2))
    if rust.startswith("*"):
        return ctypes.c_void_p
    return RUST_CTYPES[rust]


def _c_layout(structs, tmp_path):
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "hrt/hrt.h"', "int main(void) {"]
    for name, fields in structs.items():
        lines.append(f'  printf("{name} size %zu\\n", sizeof({name}));')
        for f, _ in fields:
            lines.append(f'  printf("{name} {f} %zu\\n", offsetof({name}, {f}));')
    lines.append("  return 0;\n}")
    src, exe = tmp_path / "layout.c", tmp_path / "layout"
    src.write_text("\n".join(lines))
    subprocess.check_call(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], env=tool_env())
    out = {}
    for line in subprocess.check_output([str(exe)], text=True).splitlines():
        s, f, v = line.split()
        out[(s, f)] = int(v)
    return out


PY_CLASSES = {"hrt_camera": "Camera", "hrt_render_params": "RenderParams", "hrt_tile": "Tile",
              "hrt_render_stats": "RenderStats", "hrt_tile_pixels": "TilePixels", "hrt_blob_info": "BlobInfo",
              "hrt_preset_info": "PresetInfo", "hrt_scene_info": "SceneInfo", "hrt_launch_info": "LaunchInfo",
              "hrt_scene_options": "SceneOptions"}


def test_struct_sizes_and_offsets_match_c(tmp_path):
    hs, _ = header_api()
    ds, _, _ = doc_api()
    lay = _c_layout(hs, tmp_path)
    for name, fields in ds.items():
        rs = type(name, (ctypes.Structure,), {"_fields_": [(f, _ctype_of(t)) for f, t in fields]})
        assert ctypes.sizeof(rs) == lay[(name, "size")], name
        for f, _ in fields:
            assert getattr(rs, f).offset == lay[(name, f)], (name, f)
        py = getattr(hrt, PY_CLASSES[name])
        assert ctypes.sizeof(py) == lay[(name, "size")], ("python binding", name)
        assert [f for f, *_ in py._fields_] == [f for f, _ in fields], ("python binding", name)


def test_render_stats_is_128_bytes():
    """The struct the round-2 binding had short by 16 bytes (park_slots / wait_slots); r04 added leaf_cycles, r05
    walk_steps (the walk's own node steps: node_visits also counts the nodes leaf programs test)."""
    ds, _, _ = doc_api()
    names = [f for f, _ in ds["hrt_render_stats"]]
    assert names[-4:] == ["park_slots", "wait_slots", "leaf_cycles", "walk_steps"]
    assert ctypes.sizeof(hrt.RenderStats) == 128


@pytest.mark.parametrize("name", ["hrt_scene_synchronize", "hrt_scene_get_info", "hrt_render_device", "hrt_preset_build"])
def test_entry_points_a_rust_host_needs_are_bound(name):
    _, df, _ = doc_api()
    assert name in df
