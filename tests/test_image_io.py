"""hrt_image_write: PFM keeps the frame bit for bit in the reference's row order
(row 0 = bottom, application.rs:444-445); PPM is the 8-bit view, top row first."""
import numpy as np
import pytest

import hrt
from oracle import oracle as O


@pytest.fixture(scope="module")
def frame():
    img, _ = O.OracleScene(hrt.PRESETS["random"], 1).render(24, 16, 2, 8, seed=4, threads=4)
    return img


def test_pfm_round_trip_is_exact(tmp_path, frame):
    p = tmp_path / "f.pfm"
    hrt.write_image(str(p), frame)
    back = hrt.read_pfm(str(p))
    assert back.shape == (16, 24, 3)
    assert np.array_equal(back.view(np.uint32), frame[..., :3].view(np.uint32))


def test_ppm_is_top_down_and_clamped(tmp_path):
    img = np.zeros((2, 3, 4), np.float32)
    img[0] = [0.5, 1.5, -1.0, 1.0]       # bottom row
    img[1] = [float("nan"), 0.25, 0.999, 1.0]  # top row
    p = tmp_path / "f.ppm"
    hrt.write_image(str(p), img)
    data = p.read_bytes()
    header = b"P6\n3 2\n255\n"
    assert data.startswith(header)
    px = np.frombuffer(data[len(header):], np.uint8).reshape(2, 3, 3)
    assert (px[0] == [0, 64, 255]).all()    # first stored row = image top
    assert (px[1] == [128, 255, 0]).all()


def test_bad_arguments(tmp_path, frame):
    with pytest.raises(hrt.HrtError):
        hrt.write_image(str(tmp_path / "x.pfm"), frame, fmt=7)
    with pytest.raises(hrt.HrtError):
        hrt.write_image(str(tmp_path / "missing_dir" / "x.pfm"), frame)
    with pytest.raises(ValueError):
        hrt.write_image(str(tmp_path / "x.pfm"), frame[..., :3])
