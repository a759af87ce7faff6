"""The two oracles against each other (CPU): oracle/c/oracle_ref.c (direct double-precision
sum of squared differences, insertion top-k) vs oracle/flat_knn.py (blocked float64 GEMM form),
and the C colour counts vs oracle/color_hist.py.  Both restate faiss IndexFlat / cv2.calcHist
(parity against those libraries themselves is unpinned: neither is installed)."""
import numpy as np
import pytest

from oracle import c_oracle
from oracle.color_hist import color_counts
from oracle.flat_knn import FLT_MAX, search_exact
from tests.datagen import concat_rows, mixture


def _agree(Dc, Ic, Dp, Ip, rel=1e-9):
    """Distances equal to float64 rounding of the two forms; labels equal wherever the key is
    separated from its neighbours by more than that rounding."""
    scale = np.maximum(np.abs(Dp).max(), 1.0)
    np.testing.assert_allclose(Dc, Dp, rtol=0, atol=rel * scale)
    for q in range(Dp.shape[0]):
        for j in range(Dp.shape[1]):
            lo = j == 0 or abs(Dp[q, j] - Dp[q, j - 1]) > 4 * rel * scale
            hi = j + 1 == Dp.shape[1] or abs(Dp[q, j + 1] - Dp[q, j]) > 4 * rel * scale
            if lo and hi:
                assert Ic[q, j] == Ip[q, j], (q, j, Ic[q], Ip[q])


@pytest.mark.parametrize("metric", ["l2", "ip"])
@pytest.mark.parametrize("n,d,nq,k", [(3000, 200, 24, 10), (5000, 1968, 8, 32), (700, 768, 16, 1)])
def test_c_oracle_matches_numpy_oracle(metric, n, d, nq, k):
    xb = concat_rows(n, seed=n) if d == 1968 else mixture(n, d, seed=d)
    xq = xb[:nq] + 0.05 * mixture(nq, d, seed=99)
    Dc, Ic = c_oracle.flat_search(xb, xq, k, metric)
    Dp, Ip = search_exact(xb, xq, k, metric)
    _agree(Dc, Ic, Dp, Ip)


@pytest.mark.parametrize("metric", ["l2", "ip"])
def test_c_oracle_ties_and_padding(metric):
    """Exact duplicates rank by the smaller label in both; k > n pads with -1 / +-FLT_MAX."""
    rng = np.random.default_rng(5)
    base = rng.standard_normal((4, 64)).astype(np.float32)
    xb = np.repeat(base, 5, axis=0)[rng.permutation(20)]
    xq = base[:2].copy()
    Dc, Ic = c_oracle.flat_search(xb, xq, 24, metric)
    Dp, Ip = search_exact(xb, xq, 24, metric)
    np.testing.assert_array_equal(Ic, Ip)
    np.testing.assert_allclose(Dc, Dp, rtol=1e-12, atol=1e-9)
    assert (Ic[:, 20:] == -1).all()
    assert (Dc[:, 20:] == (FLT_MAX if metric == "l2" else -FLT_MAX)).all()


def test_c_colour_counts_match_numpy():
    rng = np.random.default_rng(1)
    for h, w in ((1, 1), (7, 5), (64, 48), (256, 256)):
        img = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        for bins in (16, 8, 256, 1):
            np.testing.assert_array_equal(c_oracle.color_counts(img, bins), color_counts(img, bins))
