"""Parity tests of the bf16 candidate path (include/imgrec_knn.h KNN_SEARCH_BF16, the AUTO default
for large batches).

The bf16 path scores rows with ONE bf16 MFMA per product, reranks K' = 64 candidates in exact fp32
and certifies per query, from the stored residual norms |x - bf16(x)|, that no row outside the
candidates can rank before a returned one; uncertified queries cascade to the split path (more than
128 of them) or the exact kernel.  Results must satisfy the SAME contract as the exact path
(tests/knn_check.py against the float64 oracle): the arithmetic is an implementation detail of the
reference's index.search (main/search_from_image.py:247).
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
    ncand, _, ratio = idx.search_stats(with_error=True)
    if ncand:
        assert 0.0 <= ratio < 1.0, ratio


def _index(faiss, d, metric):
    if metric == "l2":
        return faiss.IndexFlatL2(d)
    if metric == "ip":
        return faiss.IndexFlatIP(d)
    return faiss.IndexFlat(d, faiss.METRIC_COSINE)


@pytest.mark.parametrize("d", [64, 100, 256, 768, 1968])
@pytest.mark.parametrize("nq", [1, 130, 300])
def test_bf16_l2_shapes(faiss, d, nq):
    xb = mixture(6000, d, centres=50, seed=d)
    xq = mixture(nq, d, centres=50, seed=d + 1)
    idx = faiss.IndexFlatL2(d)
    idx.add(xb)
    idx.search_mode = "bf16"
    D, I = idx.search(xq, 10)
    assert idx.search_stats()[0] == nq
    _bound_holds(idx)
    check_knn(D, I, xb, xq, 10, "l2", min_exact_frac=0.5)


@pytest.mark.parametrize("k", [1, 5, 10, 16, 17, 32])
def test_bf16_k_values(faiss, k):
    xb = mixture(8000, 512, centres=80, seed=k)
    xq = mixture(260, 512, centres=80, seed=k + 100)
    idx = faiss.IndexFlatL2(512)
    idx.add(xb)
    idx.search_mode = "bf16"
    D, I = idx.search(xq, k)
    assert idx.search_stats()[0] == 260
    _bound_holds(idx)
    check_knn(D, I, xb, xq, k, "l2", min_exact_frac=0.5)


@pytest.mark.parametrize("metric", ["ip", "cosine"])
def test_bf16_ip_and_cosine(faiss, metric):
    xb = mixture(7000, 384, centres=40, seed=5)
    xq = mixture(300, 384, centres=40, seed=6)
    idx = _index(faiss, 384, metric)
    idx.add(xb)
    idx.search_mode = "bf16"
    D, I = idx.search(xq, 10)
    _bound_holds(idx)
    check_knn(D, I, xb, xq, 10, metric, min_exact_frac=0.5)
    assert np.all(np.diff(D, axis=1) <= 0)


def test_bf16_concat_layout_self_query(faiss):
    """Config-3 rows (48|128|1792 unit parts): self match at rank 0 with 4 - 2*sqrt(3), and the
    certificate holds for (almost) every query on this layout."""
    xb = concat_rows(20000, seed=11)
    q = xb[:300].copy()
    faiss.normalize_L2(q)
    idx = faiss.IndexFlatL2(xb.shape[1])
    idx.add(xb)
    idx.search_mode = "bf16"
    D, I = idx.search(q, 10)
    ncand, nfb = idx.search_stats()
    assert ncand == 300 and nfb <= 30
    _bound_holds(idx)
    check_knn(D, I, xb, q, 10, "l2", min_exact_frac=0.5)
    assert (I[:, 0] == np.arange(300)).all()
    np.testing.assert_allclose(D[:, 0], 4 - 2 * np.sqrt(3), rtol=0, atol=1e-5)


def test_bf16_cascade_through_split_on_ties(faiss):
    """Every row duplicated 80 times (more than K' = 64): the first certificate cannot hold for any
    query; the second chance or the device-planned exact re-run settles each; ties still break by
    the smaller label."""
    base = mixture(200, 256, centres=20, seed=9)
    xb = np.repeat(base, 80, axis=0)
    xq = base[:150] + np.float32(1e-3)
    idx = faiss.IndexFlatL2(256)
    idx.add(xb)
    idx.search_mode = "bf16"
    D, I = idx.search(xq, 10)
    st = idx.certificate_stats()
    assert st["candidate_queries"] == 150 and st["second_chance"] + st["exact_reruns"] == 150
    check_knn(D, I, xb, xq, 10, "l2")
    assert (I == np.arange(150)[:, None] * 80 + np.arange(10)[None, :]).all()


def test_bf16_partial_fallback_matches_exact(faiss):
    """A few uncertified queries among certified ones: the exact re-runs scatter into place."""
    rng = np.random.default_rng(4)
    xb = mixture(12000, 512, centres=100, seed=4)
    xb[6000:6300] = xb[6000]                              # one block of 300 duplicates (> K')
    xq = np.concatenate([mixture(250, 512, centres=100, seed=5), xb[6000:6040] + 1e-4])
    xq = xq[rng.permutation(len(xq))].astype(np.float32)
    idx = faiss.IndexFlatL2(512)
    idx.add(xb)
    idx.search_mode = "bf16"
    D, I = idx.search(xq, 10)
    st = idx.certificate_stats()
    assert st["candidate_queries"] == 290 and 40 <= st["second_chance"] + st["exact_reruns"] < 290
    check_knn(D, I, xb, xq, 10, "l2", min_exact_frac=0.5)
    idx.search_mode = "exact"
    De, Ie = idx.search(xq, 10)
    assert (I == Ie).mean() > 0.95


def test_bf16_neighbours_packed_in_one_list(faiss):
    """40 near neighbours of each query placed on rows that all feed ONE per-lane list of the fused
    kernel (rows 8m + 0): the list keeps 16, the merge floor must stop a false certificate."""
    d = 256
    rng = np.random.default_rng(7)
    xb = mixture(30000, d, centres=30, seed=7)
    xq = mixture(140, d, centres=30, seed=8)
    for qi in range(0, 140, 7):
        rows = 8 * np.arange(40) + 320 * (qi // 7) + 1000
        xb[rows] = xq[qi] + (0.002 * (1 + np.arange(40))[:, None] *
                             rng.standard_normal((40, d))).astype(np.float32)
    idx = faiss.IndexFlatL2(d)
    idx.add(xb)
    idx.search_mode = "bf16"
    for k in (10, 16, 32):
        D, I = idx.search(xq, k)
        _bound_holds(idx)
        check_knn(D, I, xb, xq, k, "l2", min_exact_frac=0.5)


def test_bf16_after_incremental_adds_and_regrowth(faiss):
    xb = mixture(9000, 768, centres=60, seed=21)
    idx = faiss.IndexFlatL2(768)
    for part in np.array_split(xb, 5):                    # forces buffer regrowth copies
        idx.add(part)
    idx.search_mode = "bf16"
    xq = mixture(140, 768, centres=60, seed=22)
    D, I = idx.search(xq, 10)
    check_knn(D, I, xb, xq, 10, "l2", min_exact_frac=0.5)
    idx.reset()
    idx.add(xb[:500])
    D, I = idx.search(xq, 5)
    check_knn(D, I, xb[:500], xq, 5, "l2", min_exact_frac=0.5)


def test_bf16_tiny_corpus_and_id_offset(faiss):
    xb = mixture(12, 256, seed=3)
    idx = faiss.IndexFlatL2(256)
    idx.add(xb)
    idx.search_mode = "bf16"
    D, I = idx.search(xb[:5], 10)
    check_knn(D, I, xb, xb[:5], 10, "l2")
    idx.set_id_offset(1000)
    D2, I2 = idx.search(xb[:5], 10)
    np.testing.assert_array_equal(I2, I + 1000)
    np.testing.assert_array_equal(D2, D)


def test_bf16_large_values_scale_invariant(faiss):
    """Rows with norms ~1e3 (not unit): the bound scales with |q| max|x|, results stay exact."""
    xb = mixture(10000, 300, centres=40, seed=12) * np.float32(800.0)
    xq = mixture(200, 300, centres=40, seed=13) * np.float32(800.0)
    idx = faiss.IndexFlatL2(300)
    idx.add(xb)
    idx.search_mode = "bf16"
    D, I = idx.search(xq, 10)
    _bound_holds(idx)
    check_knn(D, I, xb, xq, 10, "l2", min_exact_frac=0.5)


def test_bf16_mode_rejected_for_tiny_d(faiss):
    idx = faiss.IndexFlatL2(32)
    with pytest.raises(faiss.KnnError):
        idx.search_mode = "bf16"
    with pytest.raises(ValueError):
        idx.search_mode = "fp8"


@pytest.mark.parametrize("n,d,nq,k,metric", [
    (20000, 1968, 600, 10, "l2"),     # config-3 width, two query blocks (second one partial)
    (5000, 100, 1100, 8, "ip"),       # narrow rows (2 stages per tile), five query blocks
    (777, 256, 513, 1, "l2"),         # tiny corpus: partial last tile, splits of one tile
    (30000, 768, 1024, 10, "cosine"),
    (40000, 512, 1024, 5, "l2"),
    (5, 64, 600, 10, "l2"),           # fewer rows than k: one 8-row group, padded results
    (2061, 128, 777, 9, "ip"),        # ragged last group (2061 = 257 x 8 + 5), partial tiles
])
def test_bf16_big_tile_kernel(faiss, n, d, nq, k, metric):
    """Batches of >= 512 queries with k <= 10 run the 256 x 256-tile kernel (knn_b16.hip)."""
    if d == 1968:
        xb = concat_rows(n, seed=n)
        xq = xb[:nq] + np.float32(0.01)
    else:
        xb = mixture(n, d, centres=70, seed=n + d)
        xq = mixture(nq, d, centres=70, seed=n + d + 1)
    idx = _index(faiss, d, metric)
    idx.add(xb)
    idx.search_mode = "bf16"
    D, I = idx.search(xq, k)
    assert idx.search_stats()[0] == nq
    _bound_holds(idx)
    sel = np.arange(0, nq, 7)                  # the oracle check on a subsample keeps it fast
    check_knn(D[sel], I[sel], xb, xq[sel], k, metric, min_exact_frac=0.5)
    idx.search_mode = "exact"
    De, Ie = idx.search(xq, k)
    assert (I == Ie).mean() > 0.97


def test_bf16_big_tile_self_query_concat(faiss):
    xb = concat_rows(50000, seed=17)
    q = xb[:1024].copy()
    faiss.normalize_L2(q)
    idx = faiss.IndexFlatL2(xb.shape[1])
    idx.add(xb)
    idx.search_mode = "bf16"
    D, I = idx.search(q, 10)
    ncand, nfb = idx.search_stats()
    assert ncand == 1024 and nfb <= 100
    assert (I[:, 0] == np.arange(1024)).all()
    np.testing.assert_allclose(D[:, 0], 4 - 2 * np.sqrt(3), rtol=0, atol=1e-5)


@pytest.mark.parametrize("nq", [1, 5, 64])
def test_auto_small_batch_on_large_corpus_takes_bf16(faiss, nq):
    """AUTO routes small batches to a candidate path (int8 for <= 8 queries, bf16 above: the
    copies stream a quarter / half of the fp32 bytes); many row splits per query exercise the
    two-level candidate merge."""
    xb = mixture(140000, 256, centres=300, seed=41)
    xq = mixture(nq, 256, centres=300, seed=42)
    idx = faiss.IndexFlatL2(256)
    idx.add(xb)
    D, I = idx.search(xq, 10)
    assert idx.search_stats()[0] == nq
    _bound_holds(idx)
    check_knn(D, I, xb, xq, 10, "l2", min_exact_frac=0.5)
    for k in (1, 16, 32):
        D, I = idx.search(xq, k)
        check_knn(D, I, xb, xq, k, "l2", min_exact_frac=0.5)


@pytest.mark.parametrize("nq", [300, 1024])
def test_bf16_cluster_sorted_storage(faiss, nq):
    """Rows stored cluster by cluster (the reference numbers images folder by folder, so similar
    images sit on adjacent rows): results stay exact, and interleaved row splits keep most
    queries certified (a query's neighbourhood spreads over several per-split lists)."""
    rng = np.random.default_rng(51)
    n, d, ncent = 60000, 384, 60
    cent = rng.standard_normal((ncent, d))
    lab = np.repeat(np.arange(ncent), n // ncent)                      # contiguous clusters
    xb = (cent[lab] + 0.5 * rng.standard_normal((n, d))).astype(np.float32)
    xq = (cent[rng.integers(0, ncent, nq)] + 0.5 * rng.standard_normal((nq, d))).astype(np.float32)
    idx = faiss.IndexFlatL2(d)
    idx.add(xb)
    idx.search_mode = "bf16"
    D, I = idx.search(xq, 10)
    ncand, nfb = idx.search_stats()
    assert ncand == nq
    _bound_holds(idx)
    sel = np.arange(0, nq, 5)
    check_knn(D[sel], I[sel], xb, xq[sel], 10, "l2", min_exact_frac=0.5)
    print(f"cluster-sorted storage: {nfb} of {nq} queries re-run")
    assert nfb <= nq // 20


def test_bf16_stats_per_search(faiss):
    """The certificate counters are per search and per index: the device-side fold (two chunk
    parities + per-search totals, csrc/knn_refine.hip fallback_prep_kernel) resets them, so an
    all-failing search followed by a clean one reports 0, and two indexes searched in turn keep
    their own counts (knn_search_stats2 waits for the search it reports)."""
    base = mixture(200, 256, centres=20, seed=19)
    dup = faiss.IndexFlatL2(256)
    dup.add(np.repeat(base, 80, axis=0))                 # 80 copies of each row: no certificate
    dup.search_mode = "bf16"
    clean = faiss.IndexFlatL2(256)
    xc = mixture(9000, 256, centres=60, seed=20)
    clean.add(xc)
    clean.search_mode = "bf16"
    qd = base[:40] + np.float32(1e-3)
    qc = mixture(200, 256, centres=60, seed=21)
    for _ in range(3):
        dup.search(qd, 10)
        st = dup.certificate_stats()
        assert st["candidate_queries"] == 40 and st["second_chance"] + st["exact_reruns"] == 40
        D, I = clean.search(qc, 10)
        ncand, nfb = clean.search_stats()
        assert ncand == 200 and nfb <= 4
        _bound_holds(clean)
        check_knn(D, I, xc, qc, 10, "l2", min_exact_frac=0.5)
    D, I = dup.search(qd, 10)
    assert (I == np.arange(40)[:, None] * 80 + np.arange(10)[None, :]).all()
    dup.search(qd[:1], 10)
    st = dup.certificate_stats()
    assert st["candidate_queries"] == 1 and st["second_chance"] + st["exact_reruns"] == 1


def test_bf16_two_query_chunks(faiss):
    """9000 queries = two 8192-query chunks, each with its own candidate pass, rerank and mailbox
    wait; the certificate counts add up over the chunks and the rows at the seam are exact."""
    xb = mixture(20000, 256, centres=90, seed=61)
    xq = mixture(9000, 256, centres=90, seed=62)
    idx = faiss.IndexFlatL2(256)
    idx.add(xb)
    D, I = idx.search(xq, 10)                             # AUTO: bf16 for this batch and corpus
    ncand, nfb = idx.search_stats()
    assert ncand == 9000 and nfb <= 450
    _bound_holds(idx)
    sel = np.r_[0:30, 8170:8215, 8980:9000]
    check_knn(D[sel], I[sel], xb, xq[sel], 10, "l2", min_exact_frac=0.5)
