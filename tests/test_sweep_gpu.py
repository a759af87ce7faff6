"""Randomised sweep of the search paths against the float64 oracle (tests/knn_check.py contract).

Each case draws a corpus size, dimension (odd ones included: padding paths), batch size, k
(past KNN_MAX_K = 32 too: the GEMM + select path), metric and search mode (auto / exact / split / bf16), adds the corpus in
one or several calls (regrowth), and checks the result of index.search
(main/search_from_image.py:247) against oracle.flat_knn.  Forcing a mode on a shape it does not
serve (split: d < 256; bf16: d < 64) must raise at the setter, and the case then runs in auto.
The case list is fixed by its seed, so a failure reproduces by its id.
"""
import numpy as np
import pytest

from tests.datagen import mixture
from tests.knn_check import check_knn

pytestmark = pytest.mark.gpu

_MODES = ("auto", "exact", "split", "bf16")
_METRICS = ("l2", "ip", "cosine")


def _cases(n_cases=40, seed=2026):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n_cases):
        n = int(rng.choice([1, 7, 255, 256, 257, 1000, 4099, 20000, 70000]))
        d = int(rng.choice([3, 16, 47, 64, 130, 256, 300, 512, 768, 1968]))
        nq = int(rng.choice([1, 2, 31, 33, 129, 257, 520, 1100]))
        k = int(rng.choice([1, 3, 10, 16, 17, 32, 33, 100]))
        metric = _METRICS[int(rng.integers(0, 3))]
        mode = _MODES[int(rng.integers(0, 4))]
        adds = int(rng.choice([1, 1, 3]))
        if n * d > 40_000_000:                  # keep every case a few seconds of oracle work
            n = 40_000_000 // d
        out.append(pytest.param(n, d, nq, k, metric, mode, adds, 1000 + i, id=f"c{i}"))
    return out


@pytest.fixture(scope="module")
def faiss(gpu):
    from image_recommender_amd import faiss_compat
    return faiss_compat


@pytest.mark.parametrize("n,d,nq,k,metric,mode,adds,seed", _cases())
def test_random_case_matches_oracle(faiss, n, d, nq, k, metric, mode, adds, seed):
    xb = mixture(n, d, centres=max(2, min(60, n // 4)), seed=seed)
    xq = mixture(nq, d, centres=max(2, min(60, n // 4)), seed=seed + 1)
    if metric == "l2":
        idx = faiss.IndexFlatL2(d)
    elif metric == "ip":
        idx = faiss.IndexFlatIP(d)
    else:
        idx = faiss.IndexFlat(d, faiss.METRIC_COSINE)
    from image_recommender_amd._lib import KnnError
    unsupported = (mode == "split" and d < 256) or (mode == "bf16" and d < 64)
    if unsupported:
        with pytest.raises(KnnError):
            idx.search_mode = mode
    else:
        idx.search_mode = mode
    for part in np.array_split(xb, adds):
        if len(part):
            idx.add(np.ascontiguousarray(part))
    assert idx.ntotal == n
    D, I = idx.search(xq, k)
    assert D.shape == (nq, k) and I.shape == (nq, k)
    check_knn(D, I, xb, xq, k, metric, min_exact_frac=0.0)


def _i8_cases(n_cases=24, seed=2027):
    """The int8 small-batch path (search_mode "i8", knn_i8.hip): batches of 1-5 queries (and 40:
    served as AUTO), tiny and ragged corpora, d below the path's 64 (refused at the setter), k past
    the fused lists (the large-k path takes it)."""
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n_cases):
        n = int(rng.choice([1, 5, 8, 9, 255, 1000, 4099, 20000, 70000]))
        d = int(rng.choice([16, 64, 65, 130, 256, 300, 512, 1024, 1968, 2500]))
        nq = int(rng.choice([1, 1, 2, 2, 3, 4, 5, 40]))
        k = int(rng.choice([1, 3, 10, 16, 17, 32, 40]))
        metric = _METRICS[int(rng.integers(0, 3))]
        adds = int(rng.choice([1, 1, 3]))
        if n * d > 40_000_000:
            n = 40_000_000 // d
        out.append(pytest.param(n, d, nq, k, metric, adds, 3000 + i, id=f"i{i}"))
    return out


@pytest.mark.parametrize("n,d,nq,k,metric,adds,seed", _i8_cases())
def test_random_i8_case_matches_oracle(faiss, n, d, nq, k, metric, adds, seed):
    from image_recommender_amd import _lib
    from image_recommender_amd._lib import KnnError
    xb = mixture(n, d, centres=max(2, min(60, n // 4)), seed=seed)
    xq = mixture(nq, d, centres=max(2, min(60, n // 4)), seed=seed + 1)
    idx = (faiss.IndexFlatL2(d) if metric == "l2" else faiss.IndexFlatIP(d) if metric == "ip"
           else faiss.IndexFlat(d, faiss.METRIC_COSINE))
    if d < 64:
        with pytest.raises(KnnError):
            idx.search_mode = "i8"
    else:
        idx.search_mode = "i8"
    for part in np.array_split(xb, adds):
        if len(part):
            idx.add(np.ascontiguousarray(part))
    D, I = idx.search(xq, k)
    if d >= 64 and nq <= 4 and k <= 32:
        assert _lib.load().knn_last_path(idx.handle) == 3
    check_knn(D, I, xb, xq, k, metric, min_exact_frac=0.0)


def test_k_above_the_large_k_route(faiss):
    """k > KNN_MAX_K_LARGE is served (faiss's range): 100 rows, k = 1025 — the 100 rows in the
    oracle's order, then label -1 / FLT_MAX padding."""
    from image_recommender_amd._lib import KNN_MAX_K_LARGE
    xb, xq = mixture(100, 64, seed=1), mixture(2, 64, seed=2)
    idx = faiss.IndexFlatL2(64)
    idx.add(xb)
    D, I = idx.search(xq, KNN_MAX_K_LARGE + 1)
    assert (I[:, 100:] == -1).all() and (D[:, 100:] == np.finfo(np.float32).max).all()
    check_knn(D, I, xb, xq, KNN_MAX_K_LARGE + 1, "l2", min_exact_frac=0.5)


@pytest.mark.parametrize("metric", ["l2", "ip", "cosine"])
@pytest.mark.parametrize("n,d,nq,k", [(20000, 96, 9, 33), (20000, 96, 9, 1024), (700, 64, 5, 1000),
                                      (9000, 1968, 3, 100), (5000, 32, 2100, 40)])
def test_large_k_matches_oracle(faiss, metric, n, d, nq, k):
    """k > KNN_MAX_K (knn_largek.hip: fp32 GEMM blocks of 8192 - k rows, running top-k by radix
    select): several corpus blocks, n < k (padding), 2100 queries (two query blocks)."""
    xb = mixture(n, d, centres=40, seed=n + k)
    xq = mixture(nq, d, centres=40, seed=n + k + 1)
    idx = (faiss.IndexFlatL2(d) if metric == "l2" else faiss.IndexFlatIP(d) if metric == "ip"
           else faiss.IndexFlat(d, faiss.METRIC_COSINE))
    idx.add(xb)
    D, I = idx.search(xq, k)
    assert D.shape == (nq, k)
    sel = np.arange(nq) if nq <= 16 else np.random.default_rng(0).choice(nq, 16, replace=False)
    check_knn(D[sel], I[sel], xb, xq[sel], k, metric, min_exact_frac=0.0)


@pytest.mark.parametrize("k", [50, 200])
def test_large_k_multi_device_index(faiss, k):
    """k > KNN_MAX_K on a multi-device index (three shards on device 0): per-shard GEMM + select,
    then the large-k merge of the gathered lists."""
    xb = mixture(30000, 96, centres=40, seed=k)
    xq = mixture(7, 96, centres=40, seed=k + 1)
    idx = faiss.IndexFlatL2(96, devices=[0, 0, 0])
    idx.add(xb)
    D, I = idx.search(xq, k)
    check_knn(D, I, xb, xq, k, "l2", min_exact_frac=0.0)


@pytest.mark.parametrize("n,d,nq,k", [(30000, 64, 100, 100), (130000, 64, 3, 1024),
                                      (20000, 64, 2100, 40), (60000, 200, 40, 300)])
def test_large_k_several_rounds(faiss, n, d, nq, k):
    """Large k over SEVERAL GEMM rounds: the unsorted running list carried from round
    to round (first = 0, nr = k), and with nq <= 64 S stripes carrying lists over rounds
    (30000 x 100 / nq 100: one stripe, 4 rounds; 130000 x 1024 / nq 3: 8 stripes, 3 rounds;
    2100 queries: two query blocks of the per-block workspace, 3 rounds; 60000 x 300 / nq 40:
    27 stripes, 2 rounds)."""
    xb = mixture(n, d, centres=40, seed=n + k + 7)
    xq = mixture(nq, d, centres=40, seed=n + k + 8)
    idx = faiss.IndexFlatL2(d)
    idx.add(xb)
    D, I = idx.search(xq, k)
    sel = np.arange(nq) if nq <= 16 else np.unique(np.concatenate(
        [np.random.default_rng(1).choice(nq, 12, replace=False), [0, nq - 1, min(nq - 1, 2048)]]))
    check_knn(D[sel], I[sel], xb, xq[sel], k, "l2", min_exact_frac=0.0)
