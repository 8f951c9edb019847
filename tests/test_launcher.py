"""bench.py's own multi-rank launcher (hrt/launcher.py): `python bench.py --gpus N` without torchrun starts
N fresh ranks with the process-group environment torchrun would give them, forwards rank 0's stdout, and
ends with a failing rank's status after stopping the others (the reference's per-tile task spawn and
gather it stands in for: src/application.rs:404-415, 461-472).  CPU only: the children here are small
Python programs, and bench.py itself on a box without a GPU, whose ranks must fail loudly and promptly."""
import os
import subprocess
import sys
import textwrap
import time

from hrt import launcher

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_needs_spawn_only_without_a_launcher():
    assert launcher.needs_spawn(2, {})
    assert launcher.needs_spawn(8, {"PATH": "/bin"})
    assert not launcher.needs_spawn(1, {})
    assert not launcher.needs_spawn(2, {"WORLD_SIZE": "2", "RANK": "0"})  # under torch.distributed.run
    assert not launcher.needs_spawn(2, {"RANK": "1"})


def test_no_spawn_under_a_profiler_preload():
    """a process under rocprofv3's preloaded library must not start the ranks itself; profiled ranks
    run as their own programs with the process-group variables set (scripts/gpu.sh rehtrace)."""
    import pytest

    pre = {"LD_PRELOAD": "/opt/rocm/lib/rocprofiler-sdk/librocprofiler-sdk-tool.so"}
    with pytest.raises(launcher.ProfilerPreloadError):
        launcher.needs_spawn(2, pre)
    assert not launcher.needs_spawn(1, pre)
    assert not launcher.needs_spawn(2, {**pre, "WORLD_SIZE": "2", "RANK": "0"})
    assert launcher.needs_spawn(2, {"LD_PRELOAD": "/usr/lib/libfoo.so"})


def test_child_env_is_torchrun_shaped():
    base = {"PATH": "/bin", "HSA_ENABLE_IPC_MODE_LEGACY": "0"}
    e = launcher.child_env(base, 3, 8, 29555)
    assert e["RANK"] == "3" and e["LOCAL_RANK"] == "3" and e["WORLD_SIZE"] == "8" and e["LOCAL_WORLD_SIZE"] == "8"
    assert e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29555"
    assert e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and e["PATH"] == "/bin"  # the parent's environment is kept
    assert e[launcher.SPAWNED] == "1"
    assert "RANK" not in base  # the parent's own environment is not touched


def _script(tmp_path, body):
    p = tmp_path / "rank.py"
    p.write_text(textwrap.dedent(body))
    return [sys.executable, str(p)]


def _run_parent(cmd, world, timeout=60):
    """run_ranks in a fresh interpreter (its signal handlers and stdout are the parent's own)."""
    code = (f"import sys; sys.path.insert(0, {os.path.join(ROOT, 'hyper-ray-tracer_amd')!r});"
            f"from hrt import launcher; sys.exit(launcher.run_ranks({cmd!r}, {world}, grace=2.0))")
    env = {k: v for k, v in os.environ.items() if k not in launcher.ENV_KEYS}
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=timeout, env=env)


def test_ranks_get_their_environment_and_rank0_owns_stdout(tmp_path):
    cmd = _script(tmp_path, """
        import os
        r = os.environ["RANK"]
        print(f"line from rank {r} world {os.environ['WORLD_SIZE']} local {os.environ['LOCAL_RANK']} "
              f"master {os.environ['MASTER_ADDR']}:{os.environ['MASTER_PORT']}", flush=True)
    """)
    res = _run_parent(cmd, 3)
    assert res.returncode == 0, res.stderr
    out = res.stdout.strip().splitlines()
    assert len(out) == 1 and out[0].startswith("line from rank 0 world 3 local 0 master 127.0.0.1:")
    for r in (1, 2):  # the other ranks' stdout goes to stderr
        assert f"line from rank {r} world 3 local {r}" in res.stderr
    assert "started 3 ranks" in res.stderr


def test_a_failing_rank_stops_the_others_and_sets_the_status(tmp_path):
    cmd = _script(tmp_path, """
        import os, sys, time
        if os.environ["RANK"] == "1":
            time.sleep(0.5)
            sys.exit(7)
        time.sleep(120)  # rank 0 stands for a rank blocked in a barrier the failed rank never reaches
    """)
    t0 = time.monotonic()
    res = _run_parent(cmd, 2)
    assert res.returncode == 7, (res.returncode, res.stderr)
    assert time.monotonic() - t0 < 30
    assert "rank 1 exited with status 7" in res.stderr


def test_a_rank_killed_by_a_signal_is_a_failure(tmp_path):
    cmd = _script(tmp_path, """
        import os, signal, time
        if os.environ["RANK"] == "0":
            os.kill(os.getpid(), signal.SIGKILL)
        time.sleep(120)
    """)
    res = _run_parent(cmd, 2)
    assert res.returncode == 128 + 9, res.returncode


def test_bench_gpus_2_spawns_ranks_and_fails_loudly_without_a_gpu():
    """The real script: `python bench.py --gpus 2 --one-device` with no torchrun starts two ranks; on this
    GPU-less container each rank stops with a clear message and the parent's status is non-zero."""
    env = {k: v for k, v in os.environ.items() if k not in launcher.ENV_KEYS}
    res = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--one-device", "--steps", "1"],
                         capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert res.returncode != 0
    assert "started 2 ranks" in res.stderr
    assert "GPU(s) visible" in res.stderr or "No HIP GPUs" in res.stderr or "no GPU" in res.stderr.lower(), res.stderr[-2000:]
    assert res.stdout.strip() == ""  # no line without a measurement
