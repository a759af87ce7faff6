"""Parity tests of the int8 small-batch candidate path (include/imgrec_knn.h KNN_SEARCH_I8, the AUTO
default for batches of <= 8 queries; csrc/knn_i8.hip).

The int8 path scores rows on a block-scaled int8 copy (one fp32 scale per 64 elements) with a
two-level int8 query (exact int32 dot4 products), reranks K' = 64 candidates in exact fp32 and certifies per query, from the stored
residual norms |x - s c|, that no row outside the candidates can rank before a returned one;
uncertified queries get the second chance over the per-split lists, then the exact re-run.  The
results must satisfy the SAME contract as the exact path (tests/knn_check.py against the float64
oracle): this is the arithmetic behind the reference CLI's one-query index.search
(main/search_from_image.py:247).
"""
import numpy as np
import pytest

from tests.datagen import concat_rows, mixture
from tests.knn_check import check_knn, check_knn_tight

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def faiss(gpu):
    from image_recommender_amd import faiss_compat
    return faiss_compat


def _lib():
    from image_recommender_amd import _lib
    return _lib.load()


def _index(faiss, d, metric):
    if metric == "l2":
        return faiss.IndexFlatL2(d)
    if metric == "ip":
        return faiss.IndexFlatIP(d)
    return faiss.IndexFlat(d, faiss.METRIC_COSINE)


def _stats(idx, nq):
    ncand, reruns, ratio = idx.search_stats(with_error=True)
    assert ncand == nq
    assert 0.0 <= ratio < 1.0, ratio
    return reruns


@pytest.mark.parametrize("d", [64, 100, 300, 768, 1024, 1968])
@pytest.mark.parametrize("nq", [1, 2, 3, 4])
def test_i8_l2_shapes(faiss, d, nq):
    xb = mixture(6001, d, centres=50, seed=d)                 # not a multiple of the 8-row group
    xq = mixture(nq, d, centres=50, seed=d + 1)
    idx = faiss.IndexFlatL2(d)
    idx.add(xb)
    idx.search_mode = "i8"
    D, I = idx.search(xq, 10)
    assert _lib().knn_last_path(idx.handle) == 3
    _stats(idx, nq)
    # (at d >= 1024 the mixture's neighbours crowd inside the RIGOROUS fp32 window (~1e-4 of the
    # key): check_knn_tight checks the labels at the empirical ~1e-6 window, against the float64
    # oracle and faiss's fp32 form)
    check_knn(D, I, xb, xq, 10, "l2", min_exact_frac=0.5 if d < 1024 else 0.25)
    if d >= 1024:
        from oracle.flat_knn import search_blas_fp32_blocked
        check_knn_tight(D, I, xb, xq, 10, "l2", blas=search_blas_fp32_blocked(xb, xq, 10),
                        min_rank_frac=0.95, min_set_frac=1.0, tag=f"i8 d={d} nq={nq}")


@pytest.mark.parametrize("k", [1, 5, 10, 16, 17, 32])
def test_i8_k_values(faiss, k):
    xb = mixture(9000, 512, centres=80, seed=k)
    xq = mixture(2, 512, centres=80, seed=k + 100)
    idx = faiss.IndexFlatL2(512)
    idx.add(xb)
    idx.search_mode = "i8"
    D, I = idx.search(xq, k)
    _stats(idx, 2)
    check_knn(D, I, xb, xq, k, "l2", min_exact_frac=0.5)


@pytest.mark.parametrize("metric", ["ip", "cosine"])
def test_i8_ip_and_cosine(faiss, metric):
    xb = mixture(7000, 384, centres=40, seed=5)
    xq = mixture(2, 384, centres=40, seed=6)
    idx = _index(faiss, 384, metric)
    idx.add(xb)
    idx.search_mode = "i8"
    D, I = idx.search(xq, 10)
    _stats(idx, 2)
    check_knn(D, I, xb, xq, 10, metric, min_exact_frac=0.5)
    assert np.all(np.diff(D, axis=1) <= 0)


def test_i8_concat_layout_self_query(faiss):
    """The reference's stored layout (colour 48 | SIFT 128 | DreamSim 1792, unit-norm parts), a
    stored row as the query: the row itself first at distance ~0."""
    xb = concat_rows(20000, seed=11)
    idx = faiss.IndexFlatL2(xb.shape[1])
    idx.add(xb)
    idx.search_mode = "i8"
    for qi in (0, 12345):
        D, I = idx.search(xb[qi:qi + 1], 10)
        assert I[0, 0] == qi and D[0, 0] < 1e-4
        check_knn(D, I, xb, xb[qi:qi + 1], 10, "l2", min_exact_frac=0.5)


def test_i8_auto_picks_int8_for_single_queries(faiss):
    """AUTO: one to eight queries take the int8 path, nine the bf16 path; below 8 blocks per row
    (d <= 448: most of a row's 16 scan lanes idle) one or two queries always (HBM-bound at every
    width, round 5), three to eight only while the int8 copy is small."""
    d = 1024
    xb = mixture(140000, d, centres=200, seed=3)
    xq = mixture(9, d, centres=200, seed=4)
    idx = faiss.IndexFlatL2(d)
    idx.add(xb)
    from oracle.flat_knn import search_exact
    orc = search_exact(xb, xq, 11, "l2")
    for nq, path in ((1, 3), (2, 3), (4, 3), (5, 3), (8, 3), (9, 2)):
        D, I = idx.search(xq[:nq], 10)
        assert _lib().knn_last_path(idx.handle) == path
        check_knn(D, I, xb, xq[:nq], 10, "l2", min_exact_frac=0.5,
                  oracle=(orc[0][:nq], orc[1][:nq]))
    del idx
    narrow = faiss.IndexFlatL2(256)                          # 4 blocks: 4 of 16 lanes live
    xn = mixture(260000, 256, centres=100, seed=5)
    narrow.add(xn[:30000])                                   # 8 MB int8 copy: int8
    narrow.search(xn[:1], 10)
    assert _lib().knn_last_path(narrow.handle) == 3
    narrow.add(xn[30000:])                                   # 71 MB: bf16 from 3 queries
    D, I = narrow.search(xn[:1], 10)
    assert _lib().knn_last_path(narrow.handle) == 3
    assert I[0, 0] == 0
    D, I = narrow.search(xn[:3], 10)
    assert _lib().knn_last_path(narrow.handle) == 2
    assert (I[:, 0] == np.arange(3)).all()


def test_i8_rows_added_after_the_copy_exists(faiss):
    """Adds after the first int8 search (copy built) extend it, across a capacity regrowth."""
    d = 192
    xb = mixture(30000, d, centres=60, seed=8)
    xq = mixture(2, d, centres=60, seed=9)
    idx = faiss.IndexFlatL2(d)
    idx.add(xb[:5000])
    idx.search_mode = "i8"
    idx.search(xq, 10)                                        # builds the int8 copy of 5000 rows
    idx.add(xb[5000:12000])
    idx.add(xb[12000:])                                       # regrowth
    D, I = idx.search(xq, 10)
    _stats(idx, 2)
    check_knn(D, I, xb, xq, 10, "l2", min_exact_frac=0.5)
    idx.reset()
    idx.add(xb[:3000])
    D, I = idx.search(xq, 10)
    check_knn(D, I, xb[:3000], xq, 10, "l2", min_exact_frac=0.5)


def test_i8_many_near_ties_fall_back_exactly(faiss):
    """200 copies of one row plus tiny perturbations around the query: far more rows inside the
    certificate's band than K' = 64, so the first certificate fails; the second chance / exact
    re-run must still return the exact answer."""
    d = 128
    rng = np.random.default_rng(5)
    base = mixture(20000, d, centres=30, seed=10)
    q = base[7].copy()
    near = q[None, :] + rng.normal(0, 1e-4, size=(200, d)).astype(np.float32)
    xb = np.concatenate([base, near]).astype(np.float32)
    idx = faiss.IndexFlatL2(d)
    idx.add(xb)
    idx.search_mode = "i8"
    D, I = idx.search(q[None, :], 10)
    # every rank sits in a tie window by construction: positions and exact distances are checked
    check_knn(D, I, xb, q[None, :], 10, "l2", min_exact_frac=0.0)
    assert set(I[0].tolist()) <= set(range(20000, 20200)) | {7}


def test_i8_clustered_storage(faiss):
    """Rows stored cluster by cluster (similar images on adjacent rows, as a folder-ordered
    database numbers them): the 8-row groups interleaved over the splits keep every split's list
    from filling with one cluster."""
    d = 256
    xb = mixture(60000, d, centres=30, seed=21)
    rng = np.random.default_rng(0)
    lab = np.argsort(((xb @ rng.normal(size=(d, 30))).argmax(1)), kind="stable")
    xb = np.ascontiguousarray(xb[lab])
    xq = xb[[5, 40000]] + 0.01
    idx = faiss.IndexFlatL2(d)
    idx.add(xb)
    idx.search_mode = "i8"
    D, I = idx.search(xq, 10)
    reruns = _stats(idx, 2)
    assert reruns == 0
    check_knn(D, I, xb, xq, 10, "l2", min_exact_frac=0.5)


@pytest.mark.parametrize("nq", [5, 6, 8])
@pytest.mark.parametrize("metric", ["l2", "cosine"])
def test_i8_batches_of_five_to_eight(faiss, nq, metric):
    """The NQ = 8 scan instance (one row per lane and step): every query's 16 lists are folded."""
    xb = mixture(12001, 300, centres=60, seed=nq)
    xq = mixture(nq, 300, centres=60, seed=nq + 50)
    idx = _index(faiss, 300, metric)
    idx.add(xb)
    idx.search_mode = "i8"
    D, I = idx.search(xq, 12)
    assert _lib().knn_last_path(idx.handle) == 3
    _stats(idx, nq)
    check_knn(D, I, xb, xq, 12, metric, min_exact_frac=0.5)


def test_i8_mode_batch_above_eight_served_as_auto(faiss):
    xb = mixture(5000, 128, centres=20, seed=1)
    xq = mixture(40, 128, centres=20, seed=2)
    idx = faiss.IndexFlatL2(128)
    idx.add(xb)
    idx.search_mode = "i8"
    D, I = idx.search(xq, 5)
    assert _lib().knn_last_path(idx.handle) != 3
    check_knn(D, I, xb, xq, 5, "l2", min_exact_frac=0.5)


@pytest.mark.parametrize("d", [2100, 3000, 4096])
@pytest.mark.parametrize("nq,k", [(1, 10), (4, 32), (8, 10), (8, 32)])
def test_i8_wide_rows_and_list_depths(faiss, d, nq, k):
    """Rows past 2048 elements (33-64 blocks: three and four blocks per lane, one row per lane and
    step) up to the path's 4096, with both list depths (KM = 16 for k <= 16, KM = 32 above)."""
    xb = mixture(4001, d, centres=40, seed=d + nq)
    xq = mixture(nq, d, centres=40, seed=d + nq + 1)
    idx = faiss.IndexFlatL2(d)
    idx.add(xb)
    idx.search_mode = "i8"
    D, I = idx.search(xq, k)
    assert _lib().knn_last_path(idx.handle) == 3
    _stats(idx, nq)
    # (at these widths the mixture's neighbours sit inside the RIGOROUS fp32 window: the labels
    # are checked at the empirical window instead, against float64 and faiss's fp32 form)
    from oracle.flat_knn import search_blas_fp32_blocked
    check_knn_tight(D, I, xb, xq, k, "l2", blas=search_blas_fp32_blocked(xb, xq, k),
                    min_rank_frac=0.95, min_set_frac=0.5, tag=f"i8 wide d={d} nq={nq} k={k}")


def test_i8_mode_refused_outside_its_dimensions(faiss):
    """d < 64 or d > 4096 has no int8 copy: the setter refuses "i8" loudly."""
    for d in (32, 4100):
        idx = faiss.IndexFlatL2(d)
        idx.add(mixture(100, d, centres=5, seed=d))
        with pytest.raises(RuntimeError):
            idx.search_mode = "i8"
        assert idx.search_mode == "auto"


@pytest.mark.parametrize("d", [64, 100, 300, 1968, 4096])
@pytest.mark.parametrize("metric", ["l2", "ip", "cosine"])
def test_i8_fused_query_prep_matches_its_own_launch(faiss, monkeypatch, d, metric):
    """The scan derives the two-level query codes, |q|^2, |q - q~| and the padded fp32 rows itself
    (I8Args::qsrc, round 5) with i8_query_prep_kernel's arithmetic: every returned bit equals the
    separate prep launch's (IMGREC_I8_FUSED_PREP=0) at widths that are not a multiple of 4, 8, 64
    (d = 100, 300) or span 1-64 blocks, for 1-8 queries (one wave quantising two of them at 5-8)
    and every metric (cosine: the in-scan normalisation)."""
    xb = mixture(5003, d, centres=40, seed=d + 7)
    xq = mixture(8, d, centres=40, seed=d + 8)
    idx = {}
    for name, env in (("fused", None), ("separate", "0")):
        if env is not None:
            monkeypatch.setenv("IMGREC_I8_FUSED_PREP", env)
        idx[name] = _index(faiss, d, metric)          # (the knob is read at index creation)
        monkeypatch.delenv("IMGREC_I8_FUSED_PREP", raising=False)
        idx[name].add(xb)
        idx[name].search_mode = "i8"
    for nq in (1, 3, 5, 8):
        q = np.ascontiguousarray(xq[:nq])
        D0, I0 = idx["separate"].search(q, 10)
        D1, I1 = idx["fused"].search(q, 10)
        assert _lib().knn_last_path(idx["fused"].handle) == 3
        assert np.array_equal(I1, I0), (nq, np.argwhere(I1 != I0)[:5])
        assert np.array_equal(D1.view(np.uint32), D0.view(np.uint32)), nq
        _stats(idx["fused"], nq)
    # (at d >= 1024 the mixture's neighbours crowd inside the rigorous window, as in
    # test_i8_l2_shapes: the tight check there, the identity with the separate launch here)
    check_knn(D1, I1, xb, xq, 10, metric, min_exact_frac=0.5 if d < 1024 else 0.25)


@pytest.mark.parametrize("d", [64, 300, 768, 1968])
@pytest.mark.parametrize("metric", ["l2", "ip", "cosine"])
def test_i8_direct_second_chance_matches_first_pass_route(faiss, monkeypatch, d, metric):
    """One-query int8 searches skip the merge and the first rerank (RerankArgs::direct, round 5):
    the certificate tail reranks every list entry under a prefix limit taken from the lists' heads
    and certifies against the list floor — over the scan's 16 unfolded lane lists per split
    (IMGREC_DIRECT_RAW=2; the default unfolds them up to 256 splits) or the folded list (=0).  The returned bits equal the first-pass route's
    (IMGREC_CHANCE_DIRECT=0) whenever neither route needed the exact re-run, for 1-4 queries
    (=4: several second-chance items, the planner picked by the item count); the oracle checks
    both."""
    xb = mixture(20011, d, centres=40, seed=d + 17)
    xq = mixture(4, d, centres=40, seed=d + 18)
    idx = {}
    for name, env in (("first_pass", {"IMGREC_CHANCE_DIRECT": "0"}),
                      ("direct", {"IMGREC_CHANCE_DIRECT": "4", "IMGREC_DIRECT_RAW": "2"}),
                      ("direct_folded", {"IMGREC_CHANCE_DIRECT": "4", "IMGREC_DIRECT_RAW": "0"})):
        for k_, v in env.items():
            monkeypatch.setenv(k_, v)
        idx[name] = _index(faiss, d, metric)          # (the knobs are read at index creation)
        for k_ in env:
            monkeypatch.delenv(k_)
        idx[name].add(xb)
        idx[name].search_mode = "i8"
    for nq in (1, 2, 4):
        q = np.ascontiguousarray(xq[:nq])
        D0, I0 = idx["first_pass"].search(q, 10)
        r0 = _stats(idx["first_pass"], nq)
        for name in ("direct", "direct_folded"):
            D1, I1 = idx[name].search(q, 10)
            r1 = _stats(idx[name], nq)
            st = idx[name].certificate_stats()
            assert st["second_chance"] + st["exact_reruns"] == nq, st     # every query took it
            if r0 == 0 and r1 == 0:
                assert np.array_equal(I1, I0), (name, nq, np.argwhere(I1 != I0)[:5])
                assert np.array_equal(D1.view(np.uint32), D0.view(np.uint32)), (name, nq)
            check_knn(D1, I1, xb, q, 10, metric, min_exact_frac=0.5 if d < 1024 else 0.25)


def test_i8_direct_route_exact_rerun_of_crowded_queries(faiss, monkeypatch):
    """Single queries whose nearest row has 12000 copies (rows of 8-row groups interleaved over
    the 512 splits: ~24 copies per split).  Over the folded lists (IMGREC_DIRECT_RAW=0) more than a
    list of 16 holds, so every list ends in ties, the list floor cannot certify, the direct
    route's second chance fails and the device-planned exact re-run answers each.  Over the 16
    unfolded lane lists per split (=2) every copy is a candidate and the second chance settles
    it.  Either way the ten smallest labels come back."""
    dup = 12000
    base = mixture(4, 256, centres=4, seed=3)
    xb = np.concatenate([np.repeat(base, dup, axis=0), mixture(9000, 256, centres=8, seed=4)])
    src = np.array([0, 1, 2, 3])
    for raw in ("0", "2"):
        monkeypatch.setenv("IMGREC_CHANCE_DIRECT", "4")
        monkeypatch.setenv("IMGREC_DIRECT_RAW", raw)
        idx = faiss.IndexFlatL2(256)
        monkeypatch.delenv("IMGREC_CHANCE_DIRECT")
        monkeypatch.delenv("IMGREC_DIRECT_RAW")
        idx.add(xb)
        idx.search_mode = "i8"
        for nq in (1, 4):
            xq = base[src[:nq]] + np.float32(1e-3)
            D, I = idx.search(xq, 10)
            st = idx.certificate_stats()
            if raw == "0":      # folded lists end in ties: only the exact re-run settles them
                assert st["candidate_queries"] == nq and st["exact_reruns"] == nq, st
            else:               # the 16 lane lists per split hold every copy (~1.5 each)
                assert st["second_chance"] + st["exact_reruns"] == nq, st
            assert (I == src[:nq, None] * dup + np.arange(10)[None, :]).all(), (raw, nq)
            check_knn(D, I, xb, xq, 10, "l2")
        del idx


@pytest.mark.parametrize("d", [100, 768])
@pytest.mark.parametrize("metric", ["l2", "ip"])
def test_i8_weighted_halves_match_the_even_split(faiss, monkeypatch, d, metric):
    """Two scan workgroups per CU (one or two queries): every K-th round of row groups the
    second-half split's group goes to its first-half partner (I8Args::half_k, round 5).  Every
    returned bit equals the even split's for K = 2 (a third of the groups moved) and K = 24, over
    40,003 rows (a ragged last round) and 1-2 queries, search after search."""
    xb = mixture(40003, d, centres=40, seed=d + 41)
    xq = mixture(2, d, centres=40, seed=d + 42)
    idx = {}
    for name, kk in (("even", "0"), ("k2", "2"), ("k24", "24")):
        monkeypatch.setenv("IMGREC_I8_HALF_K", kk)
        idx[name] = _index(faiss, d, metric)          # (the knob is read at index creation)
        monkeypatch.delenv("IMGREC_I8_HALF_K")
        idx[name].add(xb)
        idx[name].search_mode = "i8"
    for rep in range(2):
        for nq in (1, 2):
            q = np.ascontiguousarray(xq[:nq])
            D0, I0 = idx["even"].search(q, 10)
            r0 = _stats(idx["even"], nq)
            for name in ("k2", "k24"):
                D1, I1 = idx[name].search(q, 10)
                r1 = _stats(idx[name], nq)
                if r0 == 0 and r1 == 0:
                    assert np.array_equal(I1, I0), (name, rep, nq, np.argwhere(I1 != I0)[:5])
                    assert np.array_equal(D1.view(np.uint32), D0.view(np.uint32)), (name, rep, nq)
                if rep == 0:
                    check_knn(D1, I1, xb, q, 10, metric, min_exact_frac=0.5)


@pytest.mark.parametrize("d", [768, 1968])
@pytest.mark.parametrize("metric", ["l2", "cosine"])
def test_i8_group_pool_matches_the_static_split(faiss, monkeypatch, d, metric):
    """The scan's run-time pool (I8Args::pool, round 6): the last row groups handed out in chunks
    by a device counter that the scan resets itself.  Every returned bit equals the static split's
    — pool off, the default 4/64, and everything pooled in the smallest chunks (64/64, one group
    per wave) — over a ragged corpus (40,003 and 100,003 rows), one and two queries, search after
    search (a counter left non-zero would skip rows on the next search)."""
    xq = mixture(2, d, centres=40, seed=d + 52)
    for n in (40003, 100003):
        xb = mixture(n, d, centres=40, seed=d + n)
        idx = {}
        for name, pool, ch in (("off", "0", "2"), ("p4", "4", "2"), ("p64", "64", "1")):
            monkeypatch.setenv("IMGREC_I8_POOL", pool)
            monkeypatch.setenv("IMGREC_I8_POOL_CH", ch)
            idx[name] = _index(faiss, d, metric)          # (the knobs are read at index creation)
            monkeypatch.delenv("IMGREC_I8_POOL")
            monkeypatch.delenv("IMGREC_I8_POOL_CH")
            idx[name].add(xb)
            idx[name].search_mode = "i8"
        for rep in range(3):
            for nq in (1, 2):
                q = np.ascontiguousarray(xq[:nq])
                D0, I0 = idx["off"].search(q, 10)
                r0 = _stats(idx["off"], nq)
                for name in ("p4", "p64"):
                    D1, I1 = idx[name].search(q, 10)
                    assert _lib().knn_last_path(idx[name].handle) == 3
                    r1 = _stats(idx[name], nq)
                    if r0 == 0 and r1 == 0:
                        assert np.array_equal(I1, I0), (n, name, rep, nq, np.argwhere(I1 != I0)[:5])
                        assert np.array_equal(D1.view(np.uint32), D0.view(np.uint32)), (n, name, rep, nq)
                    if rep == 0:
                        check_knn(D1, I1, xb, q, 10, metric, min_exact_frac=0.5 if d < 1024 else 0.25)
        del idx
