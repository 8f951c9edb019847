"""examples/render_random.c: the C ABI alone (no Python, no PyTorch) builds, and renders on a GPU."""
import os
import subprocess

import pytest
from conftest import tool_env

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("cex") / "render_random")
    subprocess.run(["gcc", "-O2", "-std=c11", "-Wall", "-Werror", "-I" + os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "examples", "render_random.c"), "-o", out,
                    "-L" + os.path.join(ROOT, "hyper-ray-tracer_amd", "lib"), "-lhrt",
                    "-Wl,-rpath," + os.path.join(ROOT, "hyper-ray-tracer_amd", "lib")], check=True, env=tool_env())
    return out


def _has_gpu():
    import torch

    return torch.cuda.is_available()


@pytest.mark.skipif(_has_gpu(), reason="checks the no-device path")
def test_c_example_fails_loudly_without_a_device(exe, tmp_path):
    r = subprocess.run([exe, "8", "8", "1", str(tmp_path / "x.ppm")], capture_output=True, text=True)
    assert r.returncode == 1
    assert "status 6" in r.stderr          # HRT_ERR_HIP from the scene upload
    assert not (tmp_path / "x.ppm").exists()


@pytest.mark.gpu
@pytest.mark.skipif(not _has_gpu(), reason="needs a GPU")
def test_c_example_renders(exe, tmp_path):
    out = tmp_path / "r.ppm"
    r = subprocess.run([exe, "64", "36", "4", str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert out.read_bytes().startswith(b"P6\n64 36\n255\n")
    assert "rays" in r.stdout


@pytest.fixture(scope="module")
def exe_progressive(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("cexp") / "render_progressive")
    subprocess.run(["gcc", "-O2", "-std=c11", "-Wall", "-Werror", "-I" + os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "examples", "render_progressive.c"), "-o", out,
                    "-L" + os.path.join(ROOT, "hyper-ray-tracer_amd", "lib"), "-lhrt",
                    "-Wl,-rpath," + os.path.join(ROOT, "hyper-ray-tracer_amd", "lib")], check=True, env=tool_env())
    return out


def _read_pfm(path):
    import numpy as np

    data = open(path, "rb").read()
    head, rest = data.split(b"\n", 1)
    size, rest = rest.split(b"\n", 1)
    scale, rest = rest.split(b"\n", 1)
    assert head == b"PF" and float(scale) < 0  # RGB, little-endian
    w, h = map(int, size.split())
    return np.frombuffer(rest, "<f4", count=w * h * 3).reshape(h, w, 3)  # scanlines bottom to top = y up


@pytest.mark.gpu
@pytest.mark.skipif(not _has_gpu(), reason="needs a GPU")
def test_c_progressive_receiver_assembles_config1(exe_progressive, tmp_path, earth):
    """SURVEY f2 end to end in C: the tile consumer of application.rs:284-306 receives every 80x80 tile of
    BASELINE config 1 (Random 400x225, 50 spp) from hrt_render_progressive and assembles the frame,
    which matches the CPU oracle (identical per-pixel bar as the parity tests)."""
    import numpy as np

    import hrt
    from oracle import oracle as O

    out = tmp_path / "c1.pfm"
    r = subprocess.run([exe_progressive, "400", "225", "50", str(out)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "15 tiles received" in r.stdout  # ceil(400/80) x ceil(225/80)
    img = _read_pfm(out)
    ref, _ = O.OracleScene(hrt.PRESETS["random"], 1, earth).render(400, 225, 50, 50, seed=1, threads=16)
    assert float(np.abs(img - ref[..., :3]).max()) <= 1e-3
