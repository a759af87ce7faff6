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
from tests.knn_check import check_knn

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


def test_large_k_fallback_on_a_crowded_list(faiss):
    """64 exact duplicates of the query on the rows ONE fused-kernel list owns: the exact kernel's
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
    idx = faiss.IndexFlatL2(d)
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
