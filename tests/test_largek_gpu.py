"""k > KNN_MAX_K on the hand-written path (csrc/knn_largek.hip, round 5): the exact fp32 fused
kernel's 32-entry lists, their union's top-k by radix select certified against the lists' floor,
and the exact corpus scan for the queries the certificate cannot settle.  faiss serves any k
(/root/reference/main/search_from_image.py:27, `top_k`; :247 `index.search`).

Checked against the float64 oracle with tests/knn_check.check_knn (rigorous + tight windows).
"""
import ctypes as C

import numpy as np
import pytest

from tests.datagen import mixture
from oracle.flat_knn import search_blas_fp32_blocked
from tests.knn_check import check_knn, check_knn_tight

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def faiss(gpu):
    from image_recommender_amd import faiss_compat
    return faiss_compat


def _fallbacks(idx) -> int:
    from image_recommender_amd import _lib
    n = C.c_int64()
    _lib.check(_lib.load().knn_large_k_fallbacks(idx.handle, C.byref(n)), "knn_large_k_fallbacks")
    return n.value


@pytest.mark.parametrize("nq,k", [(3, 100), (3, 1024), (64, 100), (300, 200)])
def test_large_k_one_million_rows(faiss, nq, k):
    """1M rows (d = 64): every query certified from the lists (no fallback), labels and distances
    equal to the float64 oracle's up to the stated windows."""
    xb = mixture(1_000_000, 64, centres=500, seed=nq + k)
    xq = mixture(nq, 64, centres=500, seed=nq + k + 1)
    idx = faiss.IndexFlatL2(64)
    idx.add(xb)
    D, I = idx.search(xq, k)
    assert D.shape == (nq, k) and (I >= 0).all()
    assert _fallbacks(idx) == 0
    sel = np.arange(nq) if nq <= 8 else np.random.default_rng(k).choice(nq, 8, replace=False)
    check_knn(D[sel], I[sel], xb, xq[sel], k, "l2", min_exact_frac=0.5)


def test_large_k_fallback_on_a_crowded_list(faiss, monkeypatch):
    """(The tile-kernel lists: IMGREC_STREAM_LISTS=0; one query would otherwise take the
    streaming pass, whose lists are per row split — next test.)
    64 exact duplicates of the query on the rows ONE fused-kernel list owns: the exact kernel's
    row split 0 takes tile 0 (split s takes tiles s, s + nsplit, ...), its wave-row 0 holds the
    tile's rows 0-127 and lane half 0 of the 32 x 32 accumulator the rows 0-3 mod 8 of them
    (csrc/knn_kernels.hip tile_topk_item).  That list keeps 32 of the duplicates, its 32nd key (0)
    floors every row it dropped, the union's 100th key is larger: the certificate fails and the
    exact scan answers.  All 64 duplicates come first, in label order (faiss's tie rule)."""
    n, d, k = 200_000, 64, 100
    xb = mixture(n, d, centres=200, seed=5)
    q = mixture(1, d, centres=200, seed=6)
    rows = np.array([r for r in range(128) if r % 8 < 4])
    assert len(rows) == 64
    xb[rows] = q[0]
    monkeypatch.setenv("IMGREC_STREAM_LISTS", "0")
    idx = faiss.IndexFlatL2(d)                              # (knobs are read at creation)
    monkeypatch.delenv("IMGREC_STREAM_LISTS")
    idx.add(xb)
    D, I = idx.search(q, k)
    assert _fallbacks(idx) == 1
    assert (I[0, :64] == rows).all() and (D[0, :64] <= 1e-4 * float((q[0] ** 2).sum())).all()
    check_knn(D, I, xb, q, k, "l2", min_exact_frac=0.0)
    # the same search on a corpus without the crowd is certified from the lists
    idx.reset()
    idx.add(mixture(n, d, centres=200, seed=5))
    idx.search(q, k)
    assert _fallbacks(idx) == 0


@pytest.mark.parametrize("metric", ["ip", "cosine"])
def test_large_k_fallback_when_lists_hold_fewer_than_k(faiss, metric):
    """k close to the corpus size (1,100 rows, k = 1,000): the lists hold fewer than k entries in
    all, so every query goes to the exact scan."""
    xb = mixture(1100, 96, centres=20, seed=9)
    xq = mixture(5, 96, centres=20, seed=10)
    idx = faiss.IndexFlatIP(96) if metric == "ip" else faiss.IndexFlat(96, faiss.METRIC_COSINE)
    idx.add(xb)
    D, I = idx.search(xq, 1000)
    assert _fallbacks(idx) == 5
    check_knn(D, I, xb, xq, 1000, metric, min_exact_frac=0.0)


def _stream_splits():
    import torch
    return 2 * torch.cuda.get_device_properties(0).multi_processor_count


def test_large_k_stream_lists_crowded_split(faiss):
    """The streaming pass (<= 4 queries, csrc/knn_largek.hip largek_stream_kernel) keeps one list of
    32 per row split, split s owning the 8-row groups s, s + S, ... (S = 2 x CUs).  40 duplicates
    of the query on split 0's rows fill its list with key 0: that floor sits below the union's
    100th key, the certificate fails and the exact scan answers — all 40 duplicates first, in
    label order."""
    n, d, k = 300_000, 160, 100                          # (the pass takes rows of >= 128 floats)
    S = _stream_splits()
    xb = mixture(n, d, centres=200, seed=15)
    q = mixture(1, d, centres=200, seed=16)
    rows = np.array([8 * S * i + t for i in range(5) for t in range(8)])
    assert rows.max() < n and len(rows) == 40
    xb[rows] = q[0]
    idx = faiss.IndexFlatL2(d)
    idx.add(xb)
    D, I = idx.search(q, k)
    assert _fallbacks(idx) == 1
    assert (I[0, :40] == rows).all() and (D[0, :40] <= 1e-4 * float((q[0] ** 2).sum())).all()
    check_knn(D, I, xb, q, k, "l2", min_exact_frac=0.0)


@pytest.mark.parametrize("metric", ["l2", "ip", "cosine"])
@pytest.mark.parametrize("nq", [1, 2, 4])
def test_large_k_stream_pass_against_tiles_and_oracle(faiss, monkeypatch, metric, nq):
    """1-4 queries on the streaming pass and on the tile lists (IMGREC_STREAM_LISTS=0): both
    certified (no fallback), the same labels wherever the float64 oracle separates the ranks, and
    each within the stated fp32 tolerance of float64 (tests/knn_check.py)."""
    n, d, k = 200_000, 200, 128
    xb = mixture(n, d, centres=300, seed=nq + 30)
    xq = mixture(nq, d, centres=300, seed=nq + 31)
    mk = {"l2": faiss.IndexFlatL2, "ip": faiss.IndexFlatIP,
          "cosine": lambda dd: faiss.IndexFlat(dd, faiss.METRIC_COSINE)}[metric]
    out = {}
    for name, env in (("stream", None), ("tiles", "0")):
        if env is not None:
            monkeypatch.setenv("IMGREC_STREAM_LISTS", env)
        idx = mk(d)
        monkeypatch.delenv("IMGREC_STREAM_LISTS", raising=False)
        idx.add(xb)
        out[name] = idx.search(xq, k)
        assert _fallbacks(idx) == 0, name
        check_knn(out[name][0], out[name][1], xb, xq, k, metric, min_exact_frac=0.5)


def test_large_k_fallback_many_failed_queries_device_walk(faiss):
    """More failed queries than the scan's fixed grid has workgroup rows (64) and than one chunk
    holds (1,024): 1,500 queries with k = 900 of 1,000 rows — the lists hold fewer than k entries,
    so every query goes to the exact scan, which walks the failed queries the device counted
    (csrc/knn_largek.hip: no host read on the search path).  Every query against the oracle."""
    xb = mixture(1000, 64, centres=20, seed=41)
    xq = mixture(1500, 64, centres=20, seed=42)
    idx = faiss.IndexFlatL2(64)
    idx.add(xb)
    D, I = idx.search(xq, 900)
    assert _fallbacks(idx) == 1500
    sel = np.random.default_rng(0).choice(1500, 40, replace=False)
    check_knn(D[sel], I[sel], xb, xq[sel], 900, "l2", min_exact_frac=0.0)


def test_large_k_search_never_waits_on_the_host(faiss):
    """The large-k route on device pointers only enqueues work (it used to read the
    failed-query count back per chunk, serialising a multi-device index's shards): a
    device-pointer search captured into a HIP graph (a host read or stream sync would break the
    capture) replays to the host search's exact result."""
    import torch
    from image_recommender_amd import _lib
    xb = mixture(50_000, 64, centres=50, seed=43)
    xq = torch.from_numpy(mixture(8, 64, centres=50, seed=44)).cuda()
    idx = faiss.IndexFlatL2(64)
    idx.add(xb)
    k = 200
    D = torch.empty((8, k), dtype=torch.float32, device="cuda")
    I = torch.empty((8, k), dtype=torch.int64, device="cuda")
    s = torch.cuda.Stream()
    idx.search_device(xq.data_ptr(), 8, k, D.data_ptr(), I.data_ptr(), s.cuda_stream)   # workspace
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        idx.search_device(xq.data_ptr(), 8, k, D.data_ptr(), I.data_ptr(), s.cuda_stream)
    D.zero_()
    I.zero_()
    g.replay()
    torch.cuda.synchronize()
    D2, I2 = idx.search(xq.cpu().numpy(), k)
    np.testing.assert_array_equal(I.cpu().numpy(), I2)
    np.testing.assert_array_equal(D.cpu().numpy(), D2)
    assert _lib.load().knn_last_path(idx.handle) == 0


# ------------------------------------------------------------------------------------------------
# k > KNN_MAX_K_LARGE (csrc/knn_hugek.hip): every key, a segmented sort per query
# ------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("metric", ["l2", "ip", "cosine"])
def test_huge_k_4096_on_100k_rows(faiss, metric):
    """k = 4096 on 100k rows: labels and distances against the float64
    oracle (rigorous + tight windows), 12 queries."""
    n, d, k = 100_000, 128, 4096
    xb = mixture(n, d, centres=100, seed=51)
    xq = mixture(12, d, centres=100, seed=52)
    mk = {"l2": faiss.IndexFlatL2, "ip": faiss.IndexFlatIP,
          "cosine": lambda dd: faiss.IndexFlat(dd, faiss.METRIC_COSINE)}[metric]
    idx = mk(d)
    idx.add(xb)
    D, I = idx.search(xq, k)
    assert D.shape == (12, k) and (I >= 0).all()
    # (4,096 neighbours in a 100-centre mixture sit closer than the rigorous fp32 window, ~1e-4 of
    # the key, and ~20 % of them within the empirical window (~3e-6) of a neighbour: every rank
    # separated by more carries the oracle's label, and >= 75 % of the ranks are so separated)
    check_knn(D, I, xb, xq, k, metric, min_exact_frac=0.0)
    blas = search_blas_fp32_blocked(xb, xq, k) if metric == "l2" else None
    check_knn_tight(D, I, xb, xq, k, metric, blas=blas, min_rank_frac=0.75, min_set_frac=0.75,
                    tag=f"k=4096 {metric}")


def test_huge_k_whole_corpus_and_padding(faiss):
    """k = ntotal orders the whole corpus exactly as the oracle (ties by label); k > ntotal pads
    with label -1 and FLT_MAX (faiss IndexFlat's convention); duplicates tie by label."""
    n, d = 3000, 48
    xb = mixture(n, d, centres=10, seed=53)
    xb[[5, 900, 2999]] = xb[100]
    xq = mixture(4, d, centres=10, seed=54)
    xq[0] = xb[100]
    idx = faiss.IndexFlatL2(d)
    idx.add(xb)
    D, I = idx.search(xq, n)
    assert sorted(I[1].tolist()) == list(range(n))
    np.testing.assert_array_equal(I[0, :4], [5, 100, 900, 2999])
    assert (D[0, :4] == 0.0).all()
    check_knn(D, I, xb, xq, n, "l2", min_exact_frac=0.0)
    check_knn_tight(D, I, xb, xq, n, "l2", min_rank_frac=0.75, tag="k=ntotal")
    D2, I2 = idx.search(xq, n + 500)
    np.testing.assert_array_equal(I2[:, :n], I)
    np.testing.assert_array_equal(D2[:, :n], D)
    assert (I2[:, n:] == -1).all() and (D2[:, n:] == np.finfo(np.float32).max).all()


def test_huge_k_multi_shard_index_and_packed_merge(faiss):
    """k = 2000 over an 8-shard index (knn_create_multi on one device: 16,000 gathered entries per
    query, beyond the in-LDS merge) and the packed all-gather merge of 8 row shards
    (knn_merge_packed_device, sharded.py's layout): both equal the one-index search."""
    import torch
    from image_recommender_amd.sharded import merge_packed_device, packed_layout, packed_views, shard_range
    n, d, k, nq = 40_000, 96, 2000, 6
    xb = mixture(n, d, centres=40, seed=55)
    xq = mixture(nq, d, centres=40, seed=56)
    one = faiss.IndexFlatL2(d)
    one.add(xb)
    D1, I1 = one.search(xq, k)
    multi = faiss.IndexFlatL2(d, devices=[0] * 8)
    multi.add(xb)
    Dm, Im = multi.search(xq, k)
    np.testing.assert_array_equal(Im, I1)
    np.testing.assert_array_equal(Dm, D1)
    g = torch.zeros((8, packed_layout(nq, k)[0]), dtype=torch.uint8, device="cuda")
    q = torch.from_numpy(xq).cuda()
    st = torch.cuda.current_stream().cuda_stream
    for r in range(8):
        r0, r1 = shard_range(n, r, 8)
        sh = faiss.IndexFlatL2(d)
        sh.set_id_offset(r0)
        sh.add(xb[r0:r1])
        pD, pI = packed_views(g[r], nq, k)
        sh.search_device(q.data_ptr(), nq, k, pD.data_ptr(), pI.data_ptr(), st)
        torch.cuda.synchronize()
    D, I = merge_packed_device(g, nq, k, k)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(I.cpu().numpy(), I1)
    np.testing.assert_array_equal(D.cpu().numpy(), D1)
    check_knn(D1, I1, xb, xq, k, "l2", min_exact_frac=0.0)
    check_knn_tight(D1, I1, xb, xq, k, "l2", min_rank_frac=0.75, tag="k=2000 multi")
