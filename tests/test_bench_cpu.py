"""bench.py's CPU leg (the cpu_baseline object of the JSON line, and the oracle rows the parity band is
checked against) on a tiny workload: rows spread over the frame, the fields the contract names."""
import argparse

import bench


def test_cpu_leg_fields_and_rows():
    args = argparse.Namespace(preset="random", width=64, height=36, spp=4, depth=10, seed=1, cpu_seconds=0.3)
    cb, rows, img, cnt = bench.cpu_leg(args, 2.8)
    for k in ("value", "unit", "cores", "kind", "sample", "one_core_value", "host_cpu", "nproc", "label",
              "segments_per_sample", "frame_segments_per_sample", "sample_vs_frame", "cpu_quota"):
        assert k in cb, k
    assert cb["kind"] == "port" and cb["unit"] == "Mrays/s"
    assert cb["value"] > 0 and cb["one_core_value"] > 0
    assert cb["segments_per_sample"] > 1.0
    assert cb["cores"] == bench.usable_cpus()[0]
    assert rows == sorted(set(rows)) and 0 <= rows[0] and rows[-1] < 36
    assert img.shape == (len(rows), 64, 4) and cnt["samples"] == len(rows) * 64 * 4


def test_band_rows_spread_over_the_frame():
    r = bench.band_rows(1080, 60)
    assert len(r) == 60 and r[0] < 18 and r[-1] > 1060
    assert bench.band_rows(10, 50) == list(range(10))
