"""`bench.py --gpus N` / `bench_pipeline.py --gpus N` without torchrun on the GPU box (VERDICT r05
item 1): the launcher starts N ranks (here over gloo, every rank on the one visible GPU: the
protocol of the N-GPU run, not its timing) and rank 0's JSON line reports world_size N; under RCCL
with fewer GPUs than N the run exits 2 before any work.  Subprocesses of the test process, which
itself never touches the GPU here."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent


def _run(args, backend, timeout=400):
    env = dict(os.environ, IMGREC_DIST_BACKEND=backend)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return subprocess.run([sys.executable] + args, cwd=ROOT, env=env, capture_output=True, text=True,
                          timeout=timeout)


def test_bench_two_ranks_without_torchrun():
    r = _run(["bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1", "--rows", "200000",
              "--no-cpu-baseline", "--single-query-steps", "2", "--pmc", "off", "--no-phases"], "gloo")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = r.stdout.splitlines()
    assert len(lines) == 1, r.stdout                      # rank 0's line only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["world_size"] == 2
    assert d["recall_at_10"] == 1.0 and d["recall_queries"] == 1024
    assert d["config"]["rows_per_gpu"] == 100_000


def test_bench_pipeline_two_ranks_without_torchrun():
    r = _run(["bench_pipeline.py", "--gpus", "2", "--images", "2048", "--model-batch", "128", "--nq", "128",
              "--search-reps", "1"], "gloo")
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.splitlines()[-1])
    assert d["n_gpus"] == 2 and d["config"]["images_per_gpu"] == 1024
    assert d["stages"]["search"]["self_match_at_rank0"] == 1.0


def test_bench_refuses_more_gpus_than_visible():
    import torch
    n = torch.cuda.device_count()
    r = _run(["bench.py", "--gpus", str(n + 1), "--steps", "1"], "nccl", timeout=120)
    assert r.returncode == 2, (r.returncode, r.stderr[-1000:])
    assert f"needs {n + 1} visible GPUs" in r.stderr and r.stdout == ""
