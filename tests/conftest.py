"""Test configuration: `gpu` marks tests that need an MI355X (run with -m gpu on the GPU box)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def tool_env():
    """The environment for the compilers the tests run: scripts/sanitize.sh preloads the clang ASan runtime into
    the test processes (they load ASan-built libraries), and clang under a preloaded ASan runtime reports its own
    mmapped sources as crashes, so compilers run without it."""
    env = dict(os.environ)
    if "libclang_rt.asan" in env.get("LD_PRELOAD", ""):
        env.pop("LD_PRELOAD")
    return env
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
