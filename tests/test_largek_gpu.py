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
