#!/usr/bin/env python3
"""Benchmark of the exact k-NN hot path on MI355X (BASELINE.json metric).

metric: "k-NN queries/sec + recall@10 on 1M concat vectors at 1/2/4/8 MI355X".
Default workload = SURVEY.md §8d config 3: N = 1,000,000 rows of D = 1968 = 48 (colour, |N(0,1)|)
| 128 (SIFT-VLAD, mixture) | 1792 (DreamSim, mixture), every part L2-normalised (the reference's
stored layout, |x|^2 = 3), queries L2-normalised after concatenation (reference
main/search_from_image.py:305-322), squared-L2 ranking (== cosine ranking on this layout), k = 10,
batches of Q = 1024 queries.  Data are synthetic and generated on device, block-seeded so every
sharding sees the same rows.

A step = one batch of Q queries searched against the whole corpus: on N GPUs each rank searches its
contiguous row shard (fused distance + top-k kernel), the per-shard (Q, k) results are all-gathered
over RCCL and merged (strong scaling: the corpus is fixed, per-GPU rows shrink as N grows).
`--query-groups 2` runs the query x row partition instead (sharded.py; measured slower per rank at
N = 2/4/8: profiles/r02/qr_shapes.jsonl).

Contract: `python bench.py --gpus N --steps K --warmup W` prints ONE JSON line on rank 0.  Under
torchrun (WORLD_SIZE set) this process is one rank and `--gpus` must equal WORLD_SIZE; started
plainly with N > 1 it launches the N ranks itself, or exits non-zero when fewer than N GPUs are
visible (image_recommender_amd/launch.py).  `value` = Q*K / max-over-ranks wall time of the K
steps, inputs resident in HBM.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

MFMA_F32_PEAK_TFLOPS = 157.3     # MI355X dense fp32 matrix peak (MI355X_MICROARCH.md)
MFMA_BF16_PEAK_TFLOPS = 2516.8   # dense bf16 MFMA peak = 16 x the f32 rate (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0            # MI355X HBM3E peak (spec)
BLOCK = 16384                    # rows per generation block (the seed unit)

CONFIGS = {
    2: dict(name="cfg2: 1M x 768 DreamSim-only, L2", rows=1_000_000, parts=(768,), centres=(1000,),
            ranking="squared L2 (faiss IndexFlatL2)"),
    3: dict(name="cfg3: 1M x 1968 concat(color48|sift128|dreamsim1792), cosine ranking",
            rows=1_000_000, parts=(48, 128, 1792), centres=(0, 256, 1000),
            ranking="squared L2 on the normalised query (= cosine ranking: every stored part unit-norm)"),
    4: dict(name="cfg4: 10M x 1968 concat, row-sharded", rows=10_000_000, parts=(48, 128, 1792),
            centres=(0, 256, 1000),
            ranking="squared L2 on the normalised query (= cosine ranking: every stored part unit-norm)"),
}


def parse():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=3, choices=sorted(CONFIGS))
    ap.add_argument("--rows", type=int, default=None, help="override corpus rows (total)")
    ap.add_argument("--nq", type=int, default=1024, help="queries per batch")
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--query-groups", type=int, default=1,
                    help="query slices of the N ranks (sharded.py query x row partition)")
    ap.add_argument("--gt-queries", type=int, default=1024,
                    help="queries checked for recall@k (default: the whole batch)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline budget")
    ap.add_argument("--single-query-steps", type=int, default=50)
    ap.add_argument("--mode", choices=("auto", "exact", "split", "bf16", "i8"), default="auto",
                    help="search arithmetic (include/imgrec_knn.h knn_search_mode)")
    ap.add_argument("--profile-only", action="store_true",
                    help="only the timed steps (for rocprofv3 runs)")
    ap.add_argument("--no-phases", action="store_true",
                    help="skip the per-rank phase region (its event records show in kernel traces)")
    ap.add_argument("--pmc", choices=("auto", "off"), default="auto",
                    help="auto: at N = 1 on configs 2 / 3, measure the dominant kernel's HBM traffic, "
                         "clock and MFMA busy in rocprofv3 --pmc passes of this same workload "
                         "before the timed run (the committed profiles/ records otherwise)")
    return ap.parse_args()


# ------------------------------------------------------------------------------------------------
# synthetic data (device side)
# ------------------------------------------------------------------------------------------------
def make_centres(torch, cfg, device, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    cs = []
    for d, c in zip(cfg["parts"], cfg["centres"]):
        cs.append(torch.randn(c, d, generator=g).to(device) if c > 0 else None)
    return cs


def gen_block(torch, cfg, centres, b, device, seed, n=BLOCK):
    g = torch.Generator(device=device).manual_seed(seed * 1_000_003 + b)
    parts = []
    for (d, c), cen in zip(zip(cfg["parts"], cfg["centres"]), centres):
        if cen is None:
            p = torch.randn(n, d, generator=g, device=device).abs_()
        else:
            idx = torch.randint(0, c, (n,), generator=g, device=device)
            p = cen[idx] + 0.5 * torch.randn(n, d, generator=g, device=device)
        p = p / p.norm(dim=1, keepdim=True).clamp_min(1e-30)
        parts.append(p)
    return torch.cat(parts, 1).contiguous()


def gen_rows(torch, cfg, centres, r0, r1, device, seed):
    """Rows [r0, r1) of the corpus, yielded in blocks (identical for any sharding)."""
    b0, b1 = r0 // BLOCK, (r1 + BLOCK - 1) // BLOCK
    for b in range(b0, b1):
        blk = gen_block(torch, cfg, centres, b, device, seed)
        lo, hi = max(r0, b * BLOCK) - b * BLOCK, min(r1, (b + 1) * BLOCK) - b * BLOCK
        yield blk[lo:hi]


def gen_queries(torch, cfg, centres, nq, device, seed):
    q = gen_block(torch, cfg, centres, 10_000_000 + 7, device, seed + 17, n=nq)
    return (q / q.norm(dim=1, keepdim=True)).contiguous()   # faiss.normalize_L2 after concat


# ------------------------------------------------------------------------------------------------
def exact_ground_truth(torch, dist, world, cfg, centres, r0, r1, q, k, device, seed, rshards=None):
    """float64 exact top-k of this rank's shard, gathered and merged (recall reference); with a
    query x row partition the first `rshards` ranks hold every row once."""
    qd = q.double()
    qn = (qd * qd).sum(1, keepdim=True)
    best_d = torch.full((q.shape[0], k), float("inf"), dtype=torch.float64, device=device)
    best_i = torch.full((q.shape[0], k), -1, dtype=torch.int64, device=device)
    pos = r0
    for blk in gen_rows(torch, cfg, centres, r0, r1, device, seed):
        xd = blk.double()
        dd = qn + (xd * xd).sum(1)[None, :] - 2.0 * (qd @ xd.T)
        kk = min(k, xd.shape[0])
        v, i = torch.topk(dd, kk, dim=1, largest=False)
        cat_d = torch.cat([best_d, v], 1)
        cat_i = torch.cat([best_i, i + pos], 1)
        v2, j = torch.topk(cat_d, k, dim=1, largest=False)
        best_d, best_i = v2, torch.gather(cat_i, 1, j)
        pos += xd.shape[0]
    if world > 1:
        gd = [torch.empty_like(best_d) for _ in range(world)]
        gi = [torch.empty_like(best_i) for _ in range(world)]
        dist.all_gather(gd, best_d)
        dist.all_gather(gi, best_i)
        keep = rshards or world
        cat_d, cat_i = torch.cat(gd[:keep], 1), torch.cat(gi[:keep], 1)
        v2, j = torch.topk(cat_d, k, dim=1, largest=False)
        best_d, best_i = v2, torch.gather(cat_i, 1, j)
    return best_d.cpu().numpy(), best_i.cpu().numpy()


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(torch, cfg, centres, D, k, seed, budget_s, nq=1024):
    """Rank 0, N=1 only: the CPU comparator, timed on the FULL corpus at the GPU's batch size and
    at one query per search (the reference CLI's regime, main/search_from_image.py:247).

    faiss-cpu (the reference's library, north_star's HNSW comparator) is not installed on this
    image, so the comparator is the oracle's restatement of faiss IndexFlatL2's own search at a
    large batch (oracle.flat_knn.search_blas_fp32_blocked: exhaustive_L2sqr_blas's corpus blocks,
    one sgemm of the whole query batch per block on numpy's multithreaded BLAS, per-query top-k
    folded on a thread pool).  The sample: whole batches of the same `nq` queries the GPU step
    searches, against all N rows, until about budget_s of CPU work (at least one batch); then
    single-query searches of the first query against all N rows for about budget_s / 3.

    Threads: the GPU box exports OMP_NUM_THREADS = 16 — the CPU share of ONE GPU of the node that
    the harness assigns every one-GPU job (its rules: size worker pools to that share, do not raise
    it) — although the lease's affinity mask shows the whole host's cores.  The comparator obeys
    that share; both numbers are recorded ("topk_threads" / "blas_threads" vs "affinity_cores").
    """
    from oracle.flat_knn import search_blas_fp32_blocked
    try:
        allowed = len(os.sched_getaffinity(0))       # the cores this process may run on
    except (AttributeError, OSError):
        allowed = os.cpu_count() or 1
    env_threads = int(os.environ.get("OMP_NUM_THREADS", "0"))
    threads = env_threads or allowed
    try:
        from threadpoolctl import threadpool_info
        blas = max([p.get("num_threads", 1) for p in threadpool_info()
                    if p.get("user_api") == "blas"] or [threads])
    except Exception:
        blas = threads
    dev = "cuda"
    n, d = D["rows"], int(sum(cfg["parts"]))
    xb = np.empty((n, d), np.float32)
    pos = 0
    for blk in gen_rows(torch, cfg, centres, 0, n, dev, seed):
        xb[pos:pos + blk.shape[0]] = blk.cpu().numpy()
        pos += blk.shape[0]
    xq = gen_queries(torch, cfg, centres, nq, dev, seed).cpu().numpy()
    search_blas_fp32_blocked(xb[:65536], xq, k, threads=threads)     # warm BLAS threads + pool
    times = []
    t_start = time.perf_counter()
    while True:
        t0 = time.perf_counter()
        search_blas_fp32_blocked(xb, xq, k, threads=threads)
        times.append(time.perf_counter() - t0)
        if time.perf_counter() - t_start > budget_s or len(times) >= 5:
            break
    t = float(np.median(times))
    cap = (f"OMP_NUM_THREADS={env_threads}: the one-GPU CPU share the box's harness assigns "
           f"(affinity mask: {allowed} cores of the whole host)") if env_threads else \
        f"all {allowed} cores of the affinity mask"
    # nq = 1: the reference CLI's search.  faiss IndexFlatL2 at nq < 20 runs exhaustive_L2sqr_seq,
    # OpenMP over QUERIES (one thread for one query); the port instead spreads the one query's
    # scan over the BLAS threads (sgemv per 65536-row block, norms precomputed once as an index
    # would hold them), i.e. it is at least as fast as faiss's own nq = 1 path on this host.
    xn = (xb * xb).sum(1, dtype=np.float32)
    q1 = np.ascontiguousarray(xq[:1])
    search_blas_fp32_blocked(xb[:65536], q1, k, threads=threads, xb_norms=xn[:65536])
    t1s = []
    t_start = time.perf_counter()
    while True:
        t0 = time.perf_counter()
        search_blas_fp32_blocked(xb, q1, k, threads=threads, xb_norms=xn)
        t1s.append(time.perf_counter() - t0)
        if time.perf_counter() - t_start > budget_s / 3 or len(t1s) >= 50:
            break
    t1 = float(np.median(t1s))
    return {
        "value": nq / t, "unit": "queries/s", "cores": int(max(blas, threads)), "kind": "port",
        "cpu_model": cpu_model(), "blas_threads": int(blas), "topk_threads": int(threads),
        "affinity_cores": int(allowed), "host_cpus": int(os.cpu_count() or 0),
        "thread_cap": cap,
        "sample": (f"all {n} rows x {d} of the workload's corpus, {nq} queries per batch (the GPU "
                   f"step's batch), median of {len(times)} batches of {t:.2f} s; "
                   f"oracle.flat_knn.search_blas_fp32_blocked = faiss IndexFlatL2 "
                   f"exhaustive_L2sqr_blas restated (65536-row corpus blocks, one sgemm per block, "
                   f"threaded per-query top-k); faiss-cpu absent on the box"),
        "single_query": {
            "value": 1.0 / t1, "unit": "queries/s", "cores": int(max(blas, threads)), "kind": "port",
            "ms_per_query": t1 * 1e3,
            "sample": (f"one query (the GPU single_query leg's) against all {n} rows, median of "
                       f"{len(t1s)} searches; same port with the row norms precomputed, one sgemv "
                       f"per 65536-row block on the BLAS threads (faiss's own nq = 1 path, "
                       f"exhaustive_L2sqr_seq, uses one thread per query)"),
        },
    }


def kernel_pattern(tile_rows: int, tile_queries: int, path: int, k: int, name: str = ""):
    """(display name, regex) of the fused kernel a search ran: `name` from knn_plan_kernel for the
    256 x 256-tile bf16 kernels (knn_b16w_tile_kernel<KM, L2, PACK>, or the 32 x 32-MFMA form
    knn_b16_tile_kernel<KM, L2>), else knn_tile_topk_kernel<WR, WQ, KM, NS, BK, MODE, WB> (MODE 0
    fp32, 1 split, 2 bf16)."""
    import re
    if path == 2 and tile_rows == 256 and tile_queries == 256:
        if not name:
            name = f"knn_b16w_tile_kernel<{8 if k <= 8 else 10}, 1, true>"
        return name, re.escape(name)
    wr, wq = tile_rows // 128, tile_queries // 32
    return (f"knn_tile_topk_kernel<{wr}, {wq}, ..., mode {path}>",
            rf"knn_tile_topk_kernel<{wr}, {wq}, \d+, \d+, \d+, {path}, \d+>")


def _pmc_files(suffix: str, workload: str = ""):
    """profiles/*<suffix> records of one workload: `workload` "" = the default (config 3) records,
    whose names carry no workload tag; "cfg2" = profiles/*_cfg2<suffix>.  Newest first by the
    round / version in the name."""
    import glob
    import re

    def version(f):
        m = re.search(r"r(\d+)_v(\d+)", os.path.basename(f))
        return (int(m.group(1)), int(m.group(2))) if m else (0, 0)
    files = glob.glob(os.path.join(ROOT, "profiles", "*" + suffix))
    if workload:
        files = [f for f in files if os.path.basename(f).endswith(f"_{workload}{suffix}")]
    else:
        files = [f for f in files if not re.search(r"_cfg\d+" + re.escape(suffix) + "$", f)]
    return sorted(files, key=version, reverse=True)


def pmc_record(pattern: str, suffix: str, workload: str = ""):
    """The record of the newest profiles/*<suffix> of `workload` (_pmc_files) whose kernel name
    matches `pattern`, or None."""
    import re
    pat = re.compile(pattern)
    for f in _pmc_files(suffix, workload):
        try:
            data = json.load(open(f))
        except Exception:
            continue
        for name, rec in data.items():
            if pat.search(name):
                return rec, os.path.basename(f)
    return None


def pmc_traffic(pattern: str, workload: str = ""):
    """HBM bytes per launch of the fused kernel from the newest profiles/*_traffic.json of
    `workload` written by tools/pmc_traffic.sh (rocprofv3 FETCH_SIZE/WRITE_SIZE passes,
    gfx950-corrected), or None."""
    import re
    pat = re.compile(pattern)
    for f in _pmc_files("_traffic.json", workload):
        try:
            data = json.load(open(f))
        except Exception:
            continue
        for name, rec in data.items():
            if pat.search(name):
                return rec["hbm_bytes_per_launch"], os.path.basename(f)
    return None


# ------------------------------------------------------------------------------------------------
# live PMC passes (rocprofv3 child processes, started before this process touches the GPU)
# ------------------------------------------------------------------------------------------------
PMC_PASSES = {
    "fetch": "FETCH_SIZE",
    "write": "WRITE_SIZE",
    "clock": "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA",
}
PMC_KERNELS = "knn_b16w_tile_kernel|knn_b16_tile_kernel|knn_tile_topk_kernel"


def _pmc_rows(d: str):
    import csv
    import glob
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    return rows


def live_pmc(a, budget_s: float = 150.0):
    """Three rocprofv3 --pmc passes (FETCH_SIZE; WRITE_SIZE; GRBM_GUI_ACTIVE + SQ MFMA busy — one
    pass each, within the per-pass block limits) over `bench.py --profile-only` of THIS workload,
    as child processes (this process has not touched the GPU).  Returns {kernel name: record} with
    the gfx950 corrections of MI355X_MICROARCH.md §HBM (read bytes = 2 x FETCH_SIZE KiB), or
    ({}, reason) when rocprofv3 is missing or a pass fails."""
    import shutil
    import signal
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3")
    if not prof:
        return {}, "rocprofv3 not found"
    child = [sys.executable, os.path.abspath(__file__), "--profile-only", "--steps", "3", "--warmup", "1",
             "--no-phases", "--pmc", "off", "--config", str(a.config), "--nq", str(a.nq), "--k", str(a.k),
             "--mode", a.mode] + (["--rows", str(a.rows)] if a.rows else [])
    env = dict(os.environ, TMPDIR="/tmp")
    out = tempfile.mkdtemp(prefix="imgrec_pmc_", dir="/tmp")
    t0 = time.perf_counter()
    recs = {}
    for name, counters in PMC_PASSES.items():
        left = budget_s - (time.perf_counter() - t0)
        if left < 20:
            return {}, f"PMC budget ({budget_s:.0f} s) spent before the {name} pass"
        cmd = [prof, "--kernel-trace", "--kernel-include-regex", PMC_KERNELS, "--pmc", *counters.split(),
               "-d", os.path.join(out, name), "-o", "run", "--output-format", "csv", "--"] + child
        p = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                             text=True, start_new_session=True)
        try:
            _, err = p.communicate(timeout=min(left, 90.0))
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()
            return {}, f"rocprofv3 {name} pass timed out"
        if p.returncode != 0:
            return {}, f"rocprofv3 {name} pass exited {p.returncode}: {err.strip()[-200:]}"
        rows = _pmc_rows(os.path.join(out, name))
        if not rows:
            return {}, f"rocprofv3 {name} pass wrote no counter rows"
        for r in rows:
            k = r["Kernel_Name"].split("(")[0]
            rec = recs.setdefault(k, {})
            rec.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
            if name == "clock":
                rec.setdefault("_dur", []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    res = {}
    for k, rec in recs.items():
        if "FETCH_SIZE" not in rec or "WRITE_SIZE" not in rec or "GRBM_GUI_ACTIVE" not in rec:
            continue
        mean = lambda v: sum(v) / len(v)                 # noqa: E731
        fetch, write = mean(rec["FETCH_SIZE"]), mean(rec["WRITE_SIZE"])
        t = mean(rec["_dur"])
        clk = mean(rec["GRBM_GUI_ACTIVE"]) / 8 / t       # cycles per XCD over the kernel
        busy = mean(rec["SQ_VALU_MFMA_BUSY_CYCLES"]) / (256 * 4 * clk * t)
        res[k] = {"hbm_bytes_per_launch": 2 * fetch * 1024 + write * 1024, "hbm_read_bytes": 2 * fetch * 1024,
                  "hbm_write_bytes": write * 1024, "launches": len(rec["FETCH_SIZE"]),
                  "clock_ghz": clk / 1e9, "mfma_busy": busy, "dur_ms_under_pmc": t * 1e3}
    shutil.rmtree(out, ignore_errors=True)
    return res, f"{len(PMC_PASSES)} rocprofv3 --pmc passes of this workload, {time.perf_counter() - t0:.0f} s"


def main():
    a = parse()
    live = None
    # (not under a profiler already: rocprofv3 exports ROCPROF_* to the program it runs)
    profiled = any(k.startswith("ROCPROF") for k in os.environ)
    if (a.pmc == "auto" and a.gpus == 1 and "WORLD_SIZE" not in os.environ and not a.profile_only
            and a.config in (2, 3) and not profiled):
        try:
            live = live_pmc(a)
        except Exception as e:          # an unexpected profiler output never costs the bench line
            live = ({}, f"live PMC failed: {type(e).__name__}: {e}")
        print(f"[bench] live PMC: {live[1]}", file=sys.stderr, flush=True)
    # --gpus N > 1 without torchrun: start the N ranks here (no device touched in this process)
    # or stop with a non-zero status; never a silent one-GPU run (image_recommender_amd/launch.py)
    from image_recommender_amd.launch import maybe_spawn
    maybe_spawn(a.gpus, os.path.abspath(__file__), sys.argv[1:])
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # IMGREC_DIST_BACKEND=gloo rehearses the N-rank protocol with every rank on one visible GPU
    # (local % device count); the measured runs use RCCL ("nccl"), one rank per GPU
    backend = os.environ.get("IMGREC_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if world > 1 and backend == "nccl" and (ndev < world or local >= ndev):
        # one rank per GPU over RCCL: fail at once, before any collective could hang
        raise SystemExit(f"[bench] rank {rank}: WORLD_SIZE={world} ranks need {world} visible GPUs, "
                         f"this process sees {ndev} (LOCAL_RANK={local})")
    if backend != "nccl":
        local = local % max(ndev, 1)
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        from datetime import timedelta
        # a rank that never arrives ends the run with an error after this long instead of hanging
        tmo = timedelta(seconds=float(os.environ.get("IMGREC_DIST_TIMEOUT_S", "300")))
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device, timeout=tmo)
        else:
            dist.init_process_group(backend, timeout=tmo)
        dist.barrier()           # every rank up (and the RCCL communicator formed) before any work
        print(f"[bench] rank {rank}/{world}: {backend} up on cuda:{local}", file=sys.stderr, flush=True)

    from image_recommender_amd import _lib
    from image_recommender_amd.faiss_compat import METRIC_L2
    from image_recommender_amd.sharded import ShardedIndex

    cfg = dict(CONFIGS[a.config])
    if a.rows:
        cfg["rows"] = a.rows
    D_total = int(sum(cfg["parts"]))
    seed = a.config
    centres = make_centres(torch, cfg, device, seed)
    q = gen_queries(torch, cfg, centres, a.nq, device, seed)

    qgroups = a.query_groups
    nq_local = a.nq // qgroups if a.nq % qgroups == 0 else a.nq      # queries one rank searches
    shard = ShardedIndex(D_total, cfg["rows"], METRIC_L2, device=local, query_groups=qgroups)
    t_build0 = time.perf_counter()
    for blk in gen_rows(torch, cfg, centres, shard.row0, shard.row1, device, seed):
        shard.add_local(blk)
    torch.cuda.synchronize()
    build_s = time.perf_counter() - t_build0
    lib = _lib.load()
    shard.index.search_mode = a.mode
    # every search of this process runs on torch's current stream, which lives as long as the
    # process: the lazy fence is safe here and saves one event record (~6 us of GPU time) per step
    # (include/imgrec_knn.h knn_set_fence_mode)
    shard.index.set_fence_mode(lazy=True)

    def step():
        return shard.search(q, a.k)

    import ctypes as C
    h = shard.index.handle

    def region(fn, steps, kernel_events):
        """Run fn `steps` times between barrier + synchronize on both sides -> (max-over-ranks wall
        seconds, average candidate-kernel ms or None, last output).  kernel_events: the library
        records a HIP event pair around every candidate-kernel launch on its launch stream
        (knn_set_timing).  Each event costs ~5.7 us of GPU time (an idle gap before the next
        kernel, profiles/r03/), so the throughput region records none; the kernel duration comes
        from a second region of the same steps."""
        if kernel_events:
            lib.knn_set_timing(h, 1)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = None
        for _ in range(steps):
            out = fn()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        kms = 0.0
        if kernel_events:
            tot_ms, nl = C.c_double(), C.c_int()
            _lib.check(lib.knn_kernel_time(h, C.byref(tot_ms), C.byref(nl)), "timing")
            lib.knn_set_timing(h, 0)
            kms = tot_ms.value / max(nl.value, 1)
        v = torch.tensor([el, kms], dtype=torch.float64, device=device)
        if world > 1:
            dist.all_reduce(v, op=dist.ReduceOp.MAX)
        return float(v[0]), (float(v[1]) if kernel_events else None), out

    def phases(steps):
        """Per-rank phase times of `steps` searches (a diagnostic region after the timed ones:
        its event records cost GPU time): this rank's local search (query prep, candidate kernel,
        merge, rerank, certificate tail), the all-gather of the packed chunks, the final merge, and
        the candidate kernel alone; plus where this rank runs.  Gathered to every rank."""
        evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(steps)]
        lib.knn_set_timing(h, 1)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        for e in evs:
            shard.search(q, a.k, events=e)
        torch.cuda.synchronize()
        tot_ms, nl = C.c_double(), C.c_int()
        _lib.check(lib.knn_kernel_time(h, C.byref(tot_ms), C.byref(nl)), "timing")
        lib.knn_set_timing(h, 0)
        t = np.array([[e[0].elapsed_time(e[1]), e[1].elapsed_time(e[2]), e[2].elapsed_time(e[3])]
                      for e in evs])
        props = torch.cuda.get_device_properties(device)
        rec = {"rank": rank, "device": f"cuda:{local}",
               "pci_bus_id": (f"{getattr(props, 'pci_domain_id', 0):04x}:{getattr(props, 'pci_bus_id', 0):02x}:"
                              f"{getattr(props, 'pci_device_id', 0):02x}"),
               "rows": shard.local_rows, "local_search_ms": float(np.median(t[:, 0])),
               "candidate_kernel_ms": tot_ms.value / max(nl.value, 1),
               "allgather_ms": float(np.median(t[:, 1])), "merge_ms": float(np.median(t[:, 2])),
               "steps": steps}
        if world > 1:
            allrec = [None] * world
            dist.all_gather_object(allrec, rec)
            return allrec
        return [rec]

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    elapsed, _, (Dr, Ir) = region(step, a.steps, False)          # the bench value
    split_q, fallback_q, err_ratio = shard.index.search_stats(with_error=True)   # last step
    path = lib.knn_last_path(h)                                # 0 exact, 1 split, 2 bf16, 3 i8
    kel, kern_ms, _ = region(step, a.steps, True)               # candidate-kernel duration
    per_rank = None if a.no_phases else phases(a.steps)
    if a.profile_only:
        if rank == 0:
            print(json.dumps({"elapsed_s": elapsed, "ms_per_step": elapsed / a.steps * 1e3,
                              "ms_per_step_with_kernel_events": kel / a.steps * 1e3,
                              "kernel_ms": kern_ms, "split_queries": split_q,
                              "fallback_queries": fallback_q, "err_ratio": err_ratio,
                              "world_size": world, "per_rank": per_rank}))
        if world > 1:
            dist.destroy_process_group()
        return

    # recall@k on the first gt-queries queries, against float64 exact ground truth
    ngt = min(a.gt_queries, a.nq)
    gt_d, gt_i = exact_ground_truth(torch, dist, world, cfg, centres, shard.row0, shard.row1,
                                    q[:ngt], a.k, device, seed, shard.rshards)
    got_i = Ir[:ngt].cpu().numpy()
    got_d = Dr[:ngt].cpu().numpy()
    hits = sum(len(set(x.tolist()) & set(y.tolist())) for x, y in zip(got_i, gt_i))
    recall = hits / (a.k * ngt)
    label_eq = float((got_i == gt_i).mean())       # rank-by-rank equality with float64's labels
    max_dist_err = float(np.max(np.abs(got_d.astype(np.float64) - gt_d)))

    # single-query latency regime (the CLI's nq = 1 path; HBM-bound)
    q1 = q[:1].contiguous()
    for _ in range(3):
        shard.search(q1, a.k)
    torch.cuda.synchronize()
    el1, _, _ = region(lambda: shard.search(q1, a.k), a.single_query_steps, False)
    _, kern1_ms, _ = region(lambda: shard.search(q1, a.k), a.single_query_steps, True)
    # cold: the searches alternate with a second resident index of the same rows, so between two
    # searches of this index another 2.2 GB scan has streamed through the 256 MB MALL (Infinity
    # Cache) and the L2s — the reference CLI's one query arrives cold.  (A 512 MiB copy between
    # searches measured 0.41 ms — its dirty lines drain under the scan; a 512 MiB read 0.316 ms.)
    # The kernel's duration comes from this index's own events; the wall time is per search.
    other = ShardedIndex(D_total, cfg["rows"], METRIC_L2, device=local, query_groups=qgroups)
    for blk in gen_rows(torch, cfg, centres, other.row0, other.row1, device, seed):
        other.add_local(blk)
    other.index.search_mode = a.mode
    other.index.set_fence_mode(lazy=True)
    for _ in range(2):
        other.search(q1, a.k)

    def cold_pair():
        other.search(q1, a.k)
        return shard.search(q1, a.k)
    el1c, _, _ = region(cold_pair, a.single_query_steps, False)
    _, kern1c_ms, _ = region(cold_pair, a.single_query_steps, True)
    del other
    path1 = lib.knn_last_path(h)                               # 0 exact, 1 split, 2 bf16, 3 i8

    tr, tq, sp, wg = C.c_int(), C.c_int(), C.c_int(), C.c_int()
    lib.knn_plan(shard.index.handle, nq_local, a.k, C.byref(tr), C.byref(tq), C.byref(sp), C.byref(wg))

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(torch, cfg, centres, {"rows": cfg["rows"]}, a.k, seed, a.cpu_seconds, a.nq)

    if rank == 0:
        n_local = shard.local_rows
        flops = 2.0 * n_local * D_total * nq_local
        split = split_q > 0
        kbuf = C.create_string_buffer(128)
        lib.knn_plan_kernel(shard.index.handle, nq_local, a.k, kbuf, 128)
        kname, kpat = kernel_pattern(tr.value, tq.value, path, a.k, kbuf.value.decode())
        # the committed PMC records were collected on config 3 (untagged files) and config 2
        # (*_cfg2_*.json), 1M rows, 1024 queries, k = 10, one GPU; any other run reports null
        pmc_run = (world == 1 and a.config in (2, 3) and cfg["rows"] == 1_000_000 and a.nq == 1024
                   and a.k == 10)
        wl = "" if a.config == 3 else f"cfg{a.config}"
        traffic = pmc_traffic(kpat, wl) if pmc_run else None
        busy = pmc_record(kpat, "_clock.json", wl) if pmc_run else None
        import re
        live_rec = next((r for kn, r in (live[0] if live else {}).items() if re.search(kpat, kn)), None)
        if live_rec is not None:
            src = f"live: {live[1]}"
            traffic = (live_rec["hbm_bytes_per_launch"], src)
            busy = (live_rec, src)
        achieved = flops / (kern_ms * 1e-3) / 1e12
        # matrix-pipe ceiling for the algorithmic 2NDQ flop: bf16 path one bf16 MFMA per product
        # (bf16 dense peak); split path three (hi.hi + hi.lo + lo.hi: bf16 peak / 3); exact path
        # the fp32 MFMA peak
        peak = {2: MFMA_BF16_PEAK_TFLOPS, 1: MFMA_BF16_PEAK_TFLOPS / 3}.get(path, MFMA_F32_PEAK_TFLOPS)
        peak_basis = {2: "bf16 dense MFMA 2516.8 TF/s (one MFMA per product)",
                      1: "bf16 dense MFMA 2516.8 TF/s / 3 MFMAs per product"}.get(
                          path, "fp32 dense MFMA (v_mfma_f32_32x32x2_f32)")
        dtype = {2: "bf16 candidates (fp32 accumulate) + fp32 rerank, certified exact",
                 1: "bf16x3 split (fp32-equivalent) + fp32 rerank"}.get(path, "fp32")
        bytes1 = 4.0 * n_local * D_total + 4.0 * n_local    # the fp32 corpus + norms (algorithmic)
        dpb = (D_total + 63) // 64 * 64
        # what the single-query kernel actually streams: the int8 copy (codes + one fp32 scale per
        # 64 elements), the bf16 copy (bf16 path), the split copy (hi + lo, as much as fp32) or
        # the fp32 rows
        stream1 = ({3: 1.0 * n_local * dpb + 4.0 * n_local * (dpb // 64), 2: 2.0 * n_local * dpb}
                   .get(path1, 4.0 * n_local * D_total) + 4.0 * n_local)
        qps = a.nq * a.steps / elapsed
        out = {
            "metric": "k-NN queries/sec + recall@10 on 1M concat vectors at 1/2/4/8 MI355X",
            "value": qps,
            "unit": "queries/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": dtype,
            "search_mode": a.mode,
            "search_path": {0: "exact", 1: "split", 2: "bf16"}.get(path, "?"),
            "candidate_path": {"queries": split_q, "certificate_fallbacks": fallback_q,
                               "max_err_over_bound": err_ratio} if split else None,
            "data": "synthetic, generated on device (Gaussian-mixture parts, per-part L2-normalised)",
            "config": {
                "workload": cfg["name"], "rows": cfg["rows"], "dim": D_total, "k": a.k,
                "queries_per_batch": a.nq, "metric": cfg["ranking"],
                "rows_per_gpu": n_local, "parallelism": (f"query-slice x{qgroups} * row-shard x{world // qgroups}" if qgroups > 1
                                else f"row-shard x{world}") + (" + RCCL all-gather merge" if backend == "nccl"
                                                               else f" + {backend} all-gather merge (rehearsal)"),
                "queries_per_gpu": nq_local,
                "tile_rows": tr.value, "tile_queries": tq.value, "row_splits": sp.value,
                "workgroups": wg.value,
            },
            "recall_at_10": recall,
            "recall_queries": ngt,
            "labels_equal_fp64_frac": label_eq,
            "max_abs_dist_err_vs_fp64": max_dist_err,
            "roofline": {
                "bound": "mfma", "achieved": achieved, "peak": peak,
                "unit": "TFLOP/s", "frac": achieved / peak,
                "peak_basis": peak_basis,
                "traffic": traffic[0] if traffic else None,
                "traffic_source": traffic[1] if traffic else None,
                "kernel": kname,
                "kernel_ms": kern_ms,
                "kernel_timing": (f"HIP events around each launch on its stream, a second region "
                                  f"of {a.steps} steps (the value region records no events)"),
                "mfma_busy": busy[0]["mfma_busy"] if busy else None,
                "clock_ghz": busy[0]["clock_ghz"] if busy else None,
                "busy_source": busy[1] if busy else None,
                "pmc_live": (live[1] if live else "not run (--pmc off, N > 1 or a config without "
                                                  "records)") if rank == 0 else None,
                "algorithmic": f"2*N*D*Q = 2*{n_local}*{D_total}*{nq_local} flop per launch",
            },
            "single_query": {
                "queries_per_s": a.single_query_steps / el1,
                "ms_per_query_cold": el1c / (2 * a.single_query_steps) * 1e3,
                "kernel_ms": kern1_ms,
                "kernel_ms_cold": kern1c_ms,
                "cache_state": ("hbm_gbs / hbm_frac: cold (searches alternate with a second "
                                "resident index of the same rows: another 2.2 GB scan streams "
                                "through the 256 MB MALL and the L2s between two searches of "
                                "this one); *_warm: back-to-back searches of the same index"),
                "path": {0: "exact", 1: "split", 2: "bf16", 3: "i8"}.get(path1, "?"),
                "hbm_gbs": stream1 / (kern1c_ms * 1e-3) / 1e9,
                "hbm_frac": stream1 / (kern1c_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                "hbm_gbs_warm": stream1 / (kern1_ms * 1e-3) / 1e9,
                "hbm_frac_warm": stream1 / (kern1_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                "fp32_equivalent_gbs": bytes1 / (kern1_ms * 1e-3) / 1e9,
                "cpu_baseline": cpu["single_query"] if cpu else None,
            },
            "build_s": build_s,
            "world_size": dist.get_world_size() if world > 1 else 1,
            "per_rank": per_rank,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
