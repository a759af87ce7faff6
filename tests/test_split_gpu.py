"""Parity tests of the split-bf16 search path (include/imgrec_knn.h KNN_SEARCH_SPLIT).

The split path scores rows with bf16 hi/lo MFMAs, reranks K' candidates in exact fp32 and
certifies per query that no row outside the candidates can rank before a returned one; queries
that fail the certificate re-run on the exact kernel.  Its results must satisfy the SAME contract
as the exact path (tests/knn_check.py, against the float64 oracle) — the split arithmetic is an
implementation detail of the reference's index.search (main/search_from_image.py:247).
"""
import numpy as np
import pytest

from tests.datagen import concat_rows, mixture
from tests.knn_check import check_knn

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def faiss(gpu):
    from image_recommender_amd import faiss_compat
    return faiss_compat


def _bound_holds(idx):
    """The observed approximation error of every candidate stays inside the certificate bound."""
    nsplit, _, ratio = idx.search_stats(with_error=True)
    if nsplit:
        assert 0.0 <= ratio < 1.0, ratio


def _index(faiss, d, metric):
    if metric == "l2":
        return faiss.IndexFlatL2(d)
    if metric == "ip":
        return faiss.IndexFlatIP(d)
    return faiss.IndexFlat(d, faiss.METRIC_COSINE)


@pytest.mark.parametrize("d", [256, 300, 392, 512, 768, 1968])     # 300, 392: rows padded to 32
@pytest.mark.parametrize("nq", [1, 130, 300])
def test_split_l2_shapes(faiss, d, nq):
    xb = mixture(6000, d, centres=50, seed=d)
    xq = mixture(nq, d, centres=50, seed=d + 1)
    idx = faiss.IndexFlatL2(d)
    idx.add(xb)
    idx.search_mode = "split"
    D, I = idx.search(xq, 10)
    assert idx.search_stats()[0] == nq
    _bound_holds(idx)
    check_knn(D, I, xb, xq, 10, "l2", min_exact_frac=0.5)


@pytest.mark.parametrize("k", [1, 5, 8, 10, 11, 16])
def test_split_k_values(faiss, k):
    xb = mixture(8000, 512, centres=80, seed=k)
    xq = mixture(260, 512, centres=80, seed=k + 100)
    idx = faiss.IndexFlatL2(512)
    idx.add(xb)
    idx.search_mode = "split"
    D, I = idx.search(xq, k)
    _bound_holds(idx)
    check_knn(D, I, xb, xq, k, "l2", min_exact_frac=0.5)


def test_split_k_above_16_uses_exact(faiss):
    xb = mixture(3000, 256, seed=2)
    idx = faiss.IndexFlatL2(256)
    idx.add(xb)
    idx.search_mode = "split"
    D, I = idx.search(xb[:200], 17)
    assert idx.search_stats() == (0, 0)
    check_knn(D, I, xb, xb[:200], 17, "l2", min_exact_frac=0.5)


@pytest.mark.parametrize("metric", ["ip", "cosine"])
def test_split_ip_and_cosine(faiss, metric):
    xb = mixture(7000, 384, centres=40, seed=5)
    xq = mixture(300, 384, centres=40, seed=6)
    idx = _index(faiss, 384, metric)
    idx.add(xb)
    idx.search_mode = "split"
    D, I = idx.search(xq, 10)
    _bound_holds(idx)
    check_knn(D, I, xb, xq, 10, metric, min_exact_frac=0.5)
    assert np.all(np.diff(D, axis=1) <= 0)


def test_split_concat_layout_self_query(faiss):
    """Config-3 rows (48|128|1792 unit parts): self match at rank 0 with 4 - 2*sqrt(3)."""
    xb = concat_rows(20000, seed=11)
    q = xb[:300].copy()
    faiss.normalize_L2(q)
    idx = faiss.IndexFlatL2(xb.shape[1])
    idx.add(xb)
    idx.search_mode = "split"
    D, I = idx.search(q, 10)
    _bound_holds(idx)
    check_knn(D, I, xb, q, 10, "l2", min_exact_frac=0.5)
    assert (I[:, 0] == np.arange(300)).all()
    np.testing.assert_allclose(D[:, 0], 4 - 2 * np.sqrt(3), rtol=0, atol=1e-5)


def test_split_certificate_fallback_on_ties(faiss):
    """Every row duplicated 40 times: the K'-th candidate ties the k-th, no certificate can hold,
    every query re-runs on the exact kernel and ties still break by the smaller label."""
    base = mixture(200, 256, centres=20, seed=9)
    xb = np.repeat(base, 40, axis=0)
    xq = base[:150] + np.float32(1e-3)
    idx = faiss.IndexFlatL2(256)
    idx.add(xb)
    idx.search_mode = "split"
    D, I = idx.search(xq, 10)
    st = idx.certificate_stats()      # first certificate failed for all; second chance or re-run
    assert st["candidate_queries"] == 150 and st["second_chance"] + st["exact_reruns"] == 150
    check_knn(D, I, xb, xq, 10, "l2")
    assert (I == np.arange(150)[:, None] * 40 + np.arange(10)[None, :]).all()


def test_split_partial_fallback_matches_exact(faiss):
    """A mix of certified and uncertified queries: the scattered exact re-runs land in place."""
    rng = np.random.default_rng(4)
    xb = mixture(12000, 512, centres=100, seed=4)
    xb[6000:6300] = xb[6000]                              # one block of 300 duplicates
    xq = np.concatenate([mixture(200, 512, centres=100, seed=5), xb[6000:6100] + 1e-4])
    xq = xq[rng.permutation(len(xq))].astype(np.float32)
    idx = faiss.IndexFlatL2(512)
    idx.add(xb)
    idx.search_mode = "split"
    D, I = idx.search(xq, 10)
    st = idx.certificate_stats()
    assert st["candidate_queries"] == 300 and 100 <= st["second_chance"] + st["exact_reruns"] < 300
    check_knn(D, I, xb, xq, 10, "l2", min_exact_frac=0.5)
    idx.search_mode = "exact"
    De, Ie = idx.search(xq, 10)
    assert idx.search_stats() == (0, 0)
    same = (I == Ie).mean()
    assert same > 0.95


def test_split_after_incremental_adds_and_regrowth(faiss):
    xb = mixture(9000, 768, centres=60, seed=21)
    idx = faiss.IndexFlatL2(768)
    for part in np.array_split(xb, 5):                    # forces buffer regrowth copies
        idx.add(part)
    idx.search_mode = "split"
    xq = mixture(140, 768, centres=60, seed=22)
    D, I = idx.search(xq, 10)
    check_knn(D, I, xb, xq, 10, "l2", min_exact_frac=0.5)
    idx.reset()
    idx.add(xb[:500])
    D, I = idx.search(xq, 5)
    check_knn(D, I, xb[:500], xq, 5, "l2", min_exact_frac=0.5)


def test_split_tiny_corpus_and_id_offset(faiss):
    xb = mixture(12, 256, seed=3)
    idx = faiss.IndexFlatL2(256)
    idx.add(xb)
    idx.search_mode = "split"
    D, I = idx.search(xb[:5], 10)
    check_knn(D, I, xb, xb[:5], 10, "l2")
    idx.set_id_offset(1000)
    D2, I2 = idx.search(xb[:5], 10)
    np.testing.assert_array_equal(I2, I + 1000)
    np.testing.assert_array_equal(D2, D)


def test_auto_mode_routing(faiss):
    """AUTO: every batch on a candidate path at every corpus size (bf16; int8 for <= 8 queries);
    the exact kernel only for d < 64, k past the fused lists and search_mode "exact"."""
    from image_recommender_amd import _lib
    xb = mixture(20000, 512, centres=100, seed=31)
    idx = faiss.IndexFlatL2(512)
    idx.add(xb)
    assert idx.search_mode == "auto"
    xq = mixture(300, 512, centres=100, seed=32)
    for nq, path in ((300, 2), (64, 2), (9, 2), (8, 3), (1, 3)):
        D, I = idx.search(xq[:nq], 10)
        assert _lib.load().knn_last_path(idx.handle) == path, nq
        assert idx.search_stats()[0] == nq
        check_knn(D, I, xb, xq[:nq], 10, "l2", min_exact_frac=0.5)
    idx.search_mode = "exact"
    idx.search(xq[:64], 10)
    assert _lib.load().knn_last_path(idx.handle) == 0
    assert idx.search_stats() == (0, 0)
    small = faiss.IndexFlatL2(48)                         # d < 64: no bf16 / int8 copy
    small.add(mixture(3000, 48, centres=20, seed=33))
    small.search(mixture(4, 48, centres=20, seed=34), 10)
    assert _lib.load().knn_last_path(small.handle) == 0


def test_split_mode_rejected_for_small_d(faiss):
    idx = faiss.IndexFlatL2(128)
    with pytest.raises(faiss.KnnError):
        idx.search_mode = "split"
    with pytest.raises(ValueError):
        idx.search_mode = "tf32"
