"""Host logic of bench.py (no GPU): which committed PMC records the bench line cites.

The bench attaches `roofline.traffic` (rocprofv3 FETCH_SIZE/WRITE_SIZE passes) and the clock /
MFMA-busy record from the newest `profiles/r01_v*` files whose kernel name matches the kernel the
search ran; a stale or mismatched file would put another kernel's bytes on the line."""
import json
import re

import bench


def test_kernel_pattern_names_the_bf16_tile_kernel():
    name, pat = bench.kernel_pattern(256, 256, 2, 10)            # default: the 16x16 packed form
    assert name == "knn_b16w_tile_kernel<10, 1, true>"
    assert re.search(pat, "void imgrec::knn_b16w_tile_kernel<10, 1, true>")
    assert not re.search(pat, "void imgrec::knn_b16_tile_kernel<10, 1>")
    name, pat = bench.kernel_pattern(256, 256, 2, 10, "knn_b16_tile_kernel<10, 1>")   # 32x32 form
    assert re.search(pat, "void imgrec::knn_b16_tile_kernel<10, 1>")
    assert not re.search(pat, "void imgrec::knn_b16w_tile_kernel<10, 1, true>")
    name, pat = bench.kernel_pattern(256, 32, 2, 10)             # small-batch generic kernel
    assert re.search(pat, "void imgrec::knn_tile_topk_kernel<2, 1, 16, 2, 32, 2, 4>")
    assert not re.search(pat, "void imgrec::knn_b16w_tile_kernel<10, 1, true>")


def test_pmc_records_are_the_newest_matching(tmp_path, monkeypatch):
    prof = tmp_path / "profiles"
    prof.mkdir()
    kern = "void imgrec::knn_b16w_tile_kernel<10, 1, true>"
    for v, b in ((7, 1.0), (16, 2.0), (9, 3.0)):
        (prof / f"r01_v{v}_traffic.json").write_text(json.dumps({kern: {"hbm_bytes_per_launch": b}}))
    (prof / "r01_v20_traffic.json").write_text(json.dumps({"other_kernel": {"hbm_bytes_per_launch": 9.0}}))
    (prof / "r01_v16_clock.json").write_text(json.dumps({kern: {"clock_ghz": 1.7, "mfma_busy": 0.5}}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    _, pat = bench.kernel_pattern(256, 256, 2, 10)
    assert bench.pmc_traffic(pat) == (2.0, "r01_v16_traffic.json")
    rec, f = bench.pmc_record(pat, "_clock.json")
    assert f == "r01_v16_clock.json" and rec["clock_ghz"] == 1.7
    assert bench.pmc_traffic(r"no_such_kernel") is None
    # config-2 records carry a workload tag: never cited for config 3, and the only ones for 2
    (prof / "r01_v30_cfg2_traffic.json").write_text(json.dumps({kern: {"hbm_bytes_per_launch": 7.0}}))
    (prof / "r01_v30_cfg2_clock.json").write_text(json.dumps({kern: {"clock_ghz": 1.8, "mfma_busy": 0.54}}))
    assert bench.pmc_traffic(pat) == (2.0, "r01_v16_traffic.json")
    assert bench.pmc_traffic(pat, "cfg2") == (7.0, "r01_v30_cfg2_traffic.json")
    assert bench.pmc_record(pat, "_clock.json")[1] == "r01_v16_clock.json"
    assert bench.pmc_record(pat, "_clock.json", "cfg2")[0]["mfma_busy"] == 0.54


def test_committed_records_cover_the_bench_kernel():
    _, pat = bench.kernel_pattern(256, 256, 2, 10)
    bytes_, src = bench.pmc_traffic(pat)
    assert src.endswith("_traffic.json") and 5e9 < bytes_ < 7e9     # 1.5x the 3.97 GB bf16 corpus
    rec, src = bench.pmc_record(pat, "_clock.json")
    assert src.endswith("_clock.json") and 0.0 < rec["mfma_busy"] < 1.0


def test_cpu_comparator_is_exact_flat_search():
    """The CPU comparator (faiss exhaustive_L2sqr_blas restated, corpus-blocked, threaded top-k)
    returns the float64 oracle's neighbours: it is a faithful port, timed by bench.py at the GPU
    step's 1024-query batch."""
    import numpy as np
    from oracle.flat_knn import search_blas_fp32_blocked, search_exact
    from tests.datagen import concat_rows
    xb = concat_rows(20000, seed=11)
    xq = concat_rows(64, seed=12)
    D, I = search_blas_fp32_blocked(xb, xq, 10, block=4096, threads=4)
    Dg, Ig = search_exact(xb, xq, 10, "l2")
    assert (I == Ig).mean() > 0.99           # fp32 near-ties may swap
    np.testing.assert_allclose(D, Dg, rtol=0, atol=1e-4)
    assert (np.diff(D, axis=1) >= 0).all()


def test_cpu_comparator_single_query_leg():
    """bench.py's nq = 1 CPU leg (the reference CLI's regime): the same port with the row norms
    precomputed, one query against every row, returns the float64 oracle's neighbours."""
    import numpy as np
    from oracle.flat_knn import search_blas_fp32_blocked, search_exact
    from tests.datagen import concat_rows
    xb = concat_rows(20000, seed=13)
    xq = concat_rows(3, seed=14)
    xn = (xb * xb).sum(1, dtype=np.float32)
    for i in range(3):
        D, I = search_blas_fp32_blocked(xb, xq[i:i + 1], 10, block=4096, threads=4, xb_norms=xn)
        Dg, Ig = search_exact(xb, xq[i:i + 1], 10, "l2")
        assert (I == Ig).mean() > 0.9 and np.allclose(D, Dg, rtol=0, atol=1e-5)


# ------------------------------------------------------------------------------------------------
# `--gpus N` launcher (image_recommender_amd/launch.py)
# ------------------------------------------------------------------------------------------------
def test_launch_plan_decisions():
    import pytest
    from image_recommender_amd.launch import LaunchError, launch_plan
    never = lambda: (_ for _ in ()).throw(AssertionError("device count not needed"))  # noqa: E731
    assert launch_plan(1, {}, never) == "single"
    assert launch_plan(8, {"WORLD_SIZE": "8"}, never) == "rank"          # torchrun started us
    assert launch_plan(2, {}, 8) == "spawn"
    assert launch_plan(8, {}, lambda: 8) == "spawn"
    with pytest.raises(LaunchError, match="sees 1"):                      # one-GPU box, RCCL
        launch_plan(8, {}, 1)
    with pytest.raises(LaunchError, match="WORLD_SIZE=2"):                # mismatched torchrun
        launch_plan(8, {"WORLD_SIZE": "2"}, 8)
    with pytest.raises(LaunchError):
        launch_plan(0, {}, 8)
    # the gloo rehearsal shares the visible device(s): one is enough, none is not
    assert launch_plan(2, {"IMGREC_DIST_BACKEND": "gloo"}, 1) == "spawn"
    with pytest.raises(LaunchError, match="no visible GPU"):
        launch_plan(2, {"IMGREC_DIST_BACKEND": "gloo"}, 0)
    assert launch_plan(2, {"IMGREC_DIST_BACKEND": "gloo"}, 0, require_gpu=False) == "spawn"


def _probe(args, **env):
    import subprocess
    import sys
    from pathlib import Path
    probe = Path(__file__).with_name("launch_probe.py")
    e = dict(__import__("os").environ)
    for key in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(key, None)
    e.update(env)
    return subprocess.run([sys.executable, str(probe)] + args, env=e, capture_output=True,
                          text=True, timeout=120)


def test_launcher_starts_n_ranks_without_torchrun():
    """`script --gpus 3` (no torchrun) runs 3 ranks: rank 0's line reports world_size 3 and the
    all-reduce of 1 + 2 + 3."""
    r = _probe(["3"], IMGREC_DIST_BACKEND="gloo")
    assert r.returncode == 0, r.stderr
    # stdout carries rank 0's JSON line only (gloo's banners and other ranks' output: stderr)
    lines = [json.loads(x) for x in r.stdout.splitlines()]
    assert lines == [{"world_size": 3, "sum": 6.0}], r.stdout


def test_launcher_fails_without_enough_gpus():
    """RCCL needs one GPU per rank: with 1 visible the run exits non-zero before any work."""
    r = _probe(["2"], IMGREC_DIST_BACKEND="nccl", PROBE_VISIBLE="1")
    assert r.returncode == 2 and "needs 2 visible GPUs" in r.stderr, (r.returncode, r.stderr)
    assert r.stdout == ""


def test_launcher_reports_a_failing_rank():
    """A rank that exits 3 ends the run with status 3, and the rank blocked in the collective is
    stopped instead of hanging."""
    r = _probe(["2", "1"], IMGREC_DIST_BACKEND="gloo")
    assert r.returncode == 3, (r.returncode, r.stderr)
    assert "rank 1 exited with status 3" in r.stderr
