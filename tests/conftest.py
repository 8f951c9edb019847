"""Test configuration: `gpu` marks tests that need an MI355X (run with -m gpu on the GPU box)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# scripts/sanitize.sh preloads the clang ASan runtime into the test process itself; the compilers and helper
# programs the tests start run without it (clang under a preloaded ASan runtime reports its own mmapped
# sources as crashes)
if "libclang_rt.asan" in os.environ.get("LD_PRELOAD", ""):
    os.environ["HRT_SANITIZER_PRELOAD"] = os.environ.pop("LD_PRELOAD")
sys.path.insert(0, os.path.join(ROOT, "hyper-ray-tracer_amd"))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD GPU (MI355X); runs via gpurun")
    config.addinivalue_line("markers", "slow: long-running CPU test")


EARTHMAP = os.path.join(ROOT, "tests", "golden", "earthmap_rgb8.png")


@pytest.fixture(scope="session")
def earth():
    """The reference's own texture (assets/earthmap.jpg, decoded by tests/golden/make_earthmap.py)."""
    import hrt

    img = hrt.load_image(EARTHMAP)
    assert img.shape == (512, 1024, 3)
    return img
