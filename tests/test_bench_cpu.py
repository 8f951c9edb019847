"""bench.py's CPU leg (the cpu_baseline object of the JSON line) on a tiny workload: the oracle is
timed on a band of the same frame plus a one-thread stretch, and the fields the contract names exist."""
import argparse
import sys

import bench


def test_cpu_baseline_fields():
    args = argparse.Namespace(preset="random", width=64, height=36, spp=4, depth=10, seed=1, cpu_seconds=0.3)
    cb = bench.cpu_baseline(args, 2.8)
    for k in ("value", "unit", "cores", "kind", "sample", "one_core_value", "host_cpu", "nproc", "label"):
        assert k in cb, k
    assert cb["kind"] == "port" and cb["unit"] == "Mrays/s"
    assert cb["value"] > 0 and cb["one_core_value"] > 0
    assert cb["segments_per_sample"] > 1.0
