"""examples/render_random.c: the C ABI alone (no Python, no PyTorch) builds, and renders on a GPU."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("cex") / "render_random")
    subprocess.run(["gcc", "-O2", "-std=c11", "-Wall", "-Werror", "-I" + os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "examples", "render_random.c"), "-o", out,
                    "-L" + os.path.join(ROOT, "hyper-ray-tracer_amd", "lib"), "-lhrt",
                    "-Wl,-rpath," + os.path.join(ROOT, "hyper-ray-tracer_amd", "lib")], check=True)
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
