"""One process per GPU without torchrun: `python bench.py --gpus N` starts its own N ranks.

The reference renders one tokio task per 80x80 tile and gathers the tiles over an mpsc channel
(src/application.rs:404-415 spawn, :461-472 receive).  Here a tile share is one GPU's work, and each GPU
is driven by its own process (bench.py, with gloo for the control plane only).  When bench.py is started
by hand or by a driver as `python bench.py --gpus N` with no WORLD_SIZE in its environment, this module
turns that one process into N ranks:

  - the parent starts N fresh child processes running the same script with the same arguments, BEFORE it
    touches the GPU (it never imports torch or loads the HIP library: a process that has initialised the
    GPU must not fork-exec another program, and the ranks must each own their device from a clean start);
  - each child gets RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE / MASTER_ADDR (127.0.0.1) /
    MASTER_PORT, as torch.distributed.run would give it;
  - rank 0 writes to the parent's stdout (the one JSON line); the other ranks' stdout goes to stderr;
  - the parent waits; when a child fails, the others are terminated (their exact PIDs, SIGTERM then
    SIGKILL after a grace period) and the parent exits with the failing child's status, so a driver sees
    the failure instead of a hang in a barrier.  A signal to the parent is passed on to the children.

No exec anywhere: the parent stays alive as the children's supervisor and exits with their status.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
from typing import Dict, List, Optional, Sequence

ENV_KEYS = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
SPAWNED = "HRT_BENCH_SPAWNED"  # set in the children: the line records who launched the ranks


class ProfilerPreloadError(RuntimeError):
    """This process runs under a profiler's preloaded library and would have to start its ranks."""


def profiler_preloaded(env: Optional[Dict[str, str]] = None) -> bool:
    """True when a profiler's library (rocprofv3's tool library, rocprof's) is in LD_PRELOAD: it may initialise
    the GPU before main runs, so this process must not start other programs."""
    env = os.environ if env is None else env
    pre = env.get("LD_PRELOAD", "")
    return any(k in os.path.basename(x) for x in pre.replace(":", " ").split() for k in ("rocprof", "roctracer"))


def needs_spawn(gpus: int, env: Optional[Dict[str, str]] = None) -> bool:
    """True when this process must start its own ranks: more than one GPU asked for and no launcher
    (torch.distributed.run, or this module) has set up a process group environment.  Raises
    ProfilerPreloadError when that process runs under a profiler's preload: profile each rank as its own
    program instead (set RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE, MASTER_ADDR, MASTER_PORT and put
    `rocprofv3 ... --` in front of each; scripts/gpu.sh rehtrace does)."""
    env = os.environ if env is None else env
    spawn = gpus > 1 and "WORLD_SIZE" not in env and "RANK" not in env
    if spawn and profiler_preloaded(env):
        raise ProfilerPreloadError(
            "bench.py --gpus N under a profiler would start its ranks from a process the profiler's preload may "
            "have attached to the GPU: run one profiled process per rank with the process-group variables set")
    return spawn


def free_port(addr: str = "127.0.0.1") -> int:
    with socket.socket() as s:
        s.bind((addr, 0))
        return s.getsockname()[1]


def child_env(base: Dict[str, str], rank: int, world: int, port: int, addr: str = "127.0.0.1") -> Dict[str, str]:
    """The environment of rank `rank`: the parent's, plus the process-group variables torchrun sets."""
    env = dict(base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               MASTER_ADDR=addr, MASTER_PORT=str(port))
    env[SPAWNED] = "1"
    return env


def _stop(procs: Sequence[subprocess.Popen], grace: float) -> None:
    """Terminate every still-running child by PID, then kill what is left after `grace` seconds."""
    for p in procs:
        if p.poll() is None:
            try:
                p.terminate()
            except OSError:
                pass
    end = time.monotonic() + grace
    for p in procs:
        if p.poll() is None:
            try:
                p.wait(max(0.0, end - time.monotonic()))
            except subprocess.TimeoutExpired:
                pass
    for p in procs:
        if p.poll() is None:
            try:
                p.kill()
            except OSError:
                pass
            p.wait()


def run_ranks(cmd: List[str], world: int, *, env: Optional[Dict[str, str]] = None, port: Optional[int] = None,
              grace: float = 10.0, poll_s: float = 0.1, log=None) -> int:
    """Run `cmd` as `world` ranks and supervise them.  Returns 0 when every rank exits 0, else the status of
    the first rank seen failing (a negative signal number becomes 128 + signal, as a shell reports it)."""
    base = dict(os.environ if env is None else env)
    port = port or free_port()
    log = log or (lambda m: print(f"[launcher] {m}", file=sys.stderr, flush=True))
    procs: List[subprocess.Popen] = []
    prev = {}

    def forward(signum, _frame):
        log(f"signal {signum}: stopping {len(procs)} ranks")
        _stop(procs, grace)
        sys.exit(128 + signum)

    for sig in (signal.SIGTERM, signal.SIGINT):
        prev[sig] = signal.signal(sig, forward)
    try:
        for r in range(world):
            procs.append(subprocess.Popen(cmd, env=child_env(base, r, world, port),
                                          stdout=None if r == 0 else sys.stderr.fileno()))
        log(f"started {world} ranks (pids {[p.pid for p in procs]}, master 127.0.0.1:{port})")
        while True:
            codes = [p.poll() for p in procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                r, c = bad[0]
                log(f"rank {r} exited with status {c}: stopping the other ranks")
                _stop(procs, grace)
                return c if c > 0 else 128 - c
            if all(c == 0 for c in codes):
                return 0
            time.sleep(poll_s)
    finally:
        for sig, h in prev.items():
            if h is not None:  # None: a handler installed outside Python (e.g. a profiler's), left as it is
                signal.signal(sig, h)
