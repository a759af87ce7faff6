"""`--gpus N` launcher for bench.py and bench_pipeline.py: N ranks, or a clear failure.

The bench contract (`python bench.py --gpus N --steps K --warmup W`) is also run WITHOUT torchrun.
Started that way with N > 1, a script used to read WORLD_SIZE = 1 and quietly measure one GPU.
Now the entry process decides first, before torch touches a device:

* WORLD_SIZE set (torchrun or this launcher started us): we are a rank.  `--gpus` must equal
  WORLD_SIZE, or the run stops with an error.
* N == 1: run in this process.
* N > 1 without WORLD_SIZE: check that N devices are visible (`torch.cuda.device_count()`, which
  on this image counts devices without creating a HIP context), then start N child processes of
  the same script with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR = 127.0.0.1 / MASTER_PORT set,
  the environment torchrun gives its workers.  The parent never initialises a device and never
  replaces itself (no exec): it waits, stops the other ranks as soon as one fails, and exits with
  the first failing rank's status.  Only rank 0's JSON lines reach stdout; every other line any
  rank writes to stdout (gloo's connection banners, say) is passed to stderr.
* Too few devices for one rank per GPU over RCCL: exit non-zero before any work.  With
  IMGREC_DIST_BACKEND=gloo (a rehearsal of the N-rank protocol on one box) every rank shares the
  visible device(s), so one device is enough.

The reference has no multi-device code; this serves north_star's "1/2/4/8 MI355X" metric
(BASELINE.json), i.e. `index.search` (/root/reference/main/search_from_image.py:247) over a
row-sharded corpus (sharded.py).
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import threading
import time


class LaunchError(SystemExit):
    """Raised (exit status 2) when the requested launch cannot run as asked."""

    def __init__(self, msg: str):
        super().__init__(2)
        self.msg = msg

    def __str__(self):
        return self.msg


def visible_gpus() -> int:
    """HIP devices this process can see (no context is created: torch's device count)."""
    import torch
    return int(torch.cuda.device_count())


def launch_plan(gpus: int, env, visible, backend: str | None = None,
                require_gpu: bool = True) -> str:
    """Decide how to run `--gpus gpus`: "rank" (we are one of WORLD_SIZE ranks), "single" (this
    process is the whole run) or "spawn" (start `gpus` ranks).  `visible` is the device count or a
    callable returning it (only called when needed).  Raises LaunchError when the run cannot be
    what was asked."""
    backend = backend or env.get("IMGREC_DIST_BACKEND", "nccl")
    if gpus < 1:
        raise LaunchError(f"--gpus {gpus}: need at least one GPU")
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if world != gpus:
            raise LaunchError(f"--gpus {gpus} but WORLD_SIZE={world}: the launcher started a "
                              f"different number of ranks than asked")
        return "rank"
    if gpus == 1:
        return "single"
    n = visible() if callable(visible) else int(visible)
    if backend == "nccl" and n < gpus:
        raise LaunchError(f"--gpus {gpus} needs {gpus} visible GPUs (one rank per GPU over RCCL); "
                          f"this process sees {n}.  Set IMGREC_DIST_BACKEND=gloo to rehearse the "
                          f"{gpus}-rank protocol on fewer devices.")
    if backend != "nccl" and require_gpu and n < 1:
        raise LaunchError(f"--gpus {gpus} with backend {backend}: no visible GPU")
    return "spawn"


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_env(base, rank: int, world: int, port: int) -> dict:
    env = dict(base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
               LOCAL_WORLD_SIZE=str(world), GROUP_RANK="0", ROLE_RANK=str(rank),
               ROLE_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
               TORCHELASTIC_RUN_ID="imgrec-launch")
    return env


def _status(rc: int) -> int:
    return 128 - rc if rc < 0 else rc          # killed by signal s -> 128 + s (the shell's form)


def spawn(script: str, argv, world: int, env=None, poll_s: float = 0.2,
          grace_s: float = 15.0) -> int:
    """Run `python script argv` as `world` ranks; return 0 when every rank succeeded, else the
    status of the first rank that failed (the ranks stopped because of it do not mask it).
    As soon as one rank fails the others are sent SIGTERM (then SIGKILL after grace_s), so a rank
    waiting in a collective for a dead peer does not hang the run."""
    base = dict(os.environ if env is None else env)
    port = free_port()
    procs, pumps = [], []

    def pump(stream, rank):
        for line in iter(stream.readline, ""):
            out = sys.stdout if rank == 0 and line.lstrip().startswith("{") else sys.stderr
            out.write(line)
            out.flush()
        stream.close()
    try:
        for r in range(world):
            procs.append(subprocess.Popen([sys.executable, "-u", script] + list(argv),
                                          env=rank_env(base, r, world, port),
                                          stdout=subprocess.PIPE, text=True, bufsize=1))
            pumps.append(threading.Thread(target=pump, args=(procs[-1].stdout, r), daemon=True))
            pumps[-1].start()
        worst, failed_at = 0, None
        while True:
            alive = 0
            for p in procs:
                rc = p.poll()
                if rc is None:
                    alive += 1
                elif rc != 0:
                    if failed_at is None:
                        worst = _status(rc)
                        failed_at = time.monotonic()
                        print(f"[launch] rank {procs.index(p)} exited with status {_status(rc)}; "
                              f"stopping the other ranks", file=sys.stderr, flush=True)
                        for q in procs:
                            if q.poll() is None:
                                q.send_signal(signal.SIGTERM)
            if alive == 0:
                for t in pumps:
                    t.join(timeout=5.0)
                return worst
            if failed_at is not None and time.monotonic() - failed_at > grace_s:
                for q in procs:
                    if q.poll() is None:
                        q.kill()
            time.sleep(poll_s)
    except BaseException:
        for p in procs:
            if p.poll() is None:
                p.kill()
        for p in procs:
            p.wait()
        raise


def maybe_spawn(gpus: int, script: str, argv, require_gpu: bool = True, visible=None) -> bool:
    """The entry process's decision (module doc).  Returns False when this process should run the
    work itself (a rank, or N == 1); otherwise runs the N ranks and exits with their status.
    On an impossible launch prints the reason and exits 2."""
    try:
        plan = launch_plan(gpus, os.environ, visible if visible is not None else visible_gpus,
                           require_gpu=require_gpu)
    except LaunchError as e:
        print(f"[launch] {e.msg}", file=sys.stderr, flush=True)
        raise
    if plan != "spawn":
        return False
    print(f"[launch] starting {gpus} ranks of {os.path.basename(script)} "
          f"(backend {os.environ.get('IMGREC_DIST_BACKEND', 'nccl')})", file=sys.stderr, flush=True)
    sys.exit(spawn(script, argv, gpus))
