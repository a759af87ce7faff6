"""TEST INFRASTRUCTURE ONLY — exact flat k-NN restated from faiss IndexFlat semantics.

The reference reaches this arithmetic through ``index.search(query_vec, top_k)``
(/root/reference/main/search_from_image.py:247, /root/reference/Analytics/rt_Search.py:63) on the
index built at /root/reference/main/create_index.py:207-234 / 311.  north_star names
``IndexFlatL2`` as the parity target; the semantics restated here are faiss 1.10's
(faiss-cpu==1.10.0, /root/reference/requirements.txt:2, not installed — parity unpinned against
faiss itself):

* L2: squared distance, results ascending; IP: inner product, results descending.
* k > ntotal: trailing labels -1 with distance FLT_MAX (L2) / -FLT_MAX (IP) (faiss heap neutral).
* exact ties: the smaller label first (this build's stated rule; faiss's heap order for equal keys
  depends on which of its code paths ran).
"""
from __future__ import annotations

import numpy as np

FLT_MAX = float(np.finfo(np.float32).max)
U32 = 2.0 ** -24   # unit roundoff of float32


def _topk_rows(keys: np.ndarray, ids: np.ndarray, k: int):
    """Per row, the k smallest (key, id) pairs in lexicographic order."""
    nq, n = keys.shape
    kk = min(k, n)
    outk = np.full((nq, k), np.inf)
    outi = np.full((nq, k), -1, dtype=np.int64)
    if kk == 0:
        return outk, outi
    part = np.argpartition(keys, kk - 1, axis=1)[:, :kk] if kk < n else np.tile(np.arange(n), (nq, 1))
    kth = np.take_along_axis(keys, part, 1).max(axis=1)
    for r in range(nq):
        cand = np.nonzero(keys[r] <= kth[r])[0]          # all ties at the boundary too
        order = np.lexsort((ids[cand], keys[r, cand]))[:kk]
        outk[r, :kk] = keys[r, cand[order]]
        outi[r, :kk] = ids[cand[order]]
    return outk, outi


def search_exact(xb: np.ndarray, xq: np.ndarray, k: int, metric: str = "l2",
                 block: int = 65536):
    """Exact k-NN in float64.  Returns (D float64 (nq,k), I int64 (nq,k)) in faiss conventions.

    metric: "l2" (IndexFlatL2), "ip" (IndexFlatIP), "cosine" (rows and queries normalised, IP).
    Rows are converted to float64 one block at a time, so a float32 corpus of any size is only
    copied block by block (the full-size config-3/4 tests check 1M+ rows this way).
    """
    xq = np.asarray(xq, dtype=np.float64)
    if metric == "cosine":
        xq = _normalize64(xq)
    nq, n = xq.shape[0], xb.shape[0]
    bestk = np.full((nq, k), np.inf)
    besti = np.full((nq, k), -1, dtype=np.int64)
    qn = (xq * xq).sum(1)
    for r0 in range(0, n, block):
        xc = np.asarray(xb[r0:r0 + block], dtype=np.float64)
        if metric == "cosine":
            xc = _normalize64(xc)
        ip = xq @ xc.T
        if metric == "l2":
            keys = qn[:, None] + (xc * xc).sum(1)[None, :] - 2.0 * ip
            keys = np.maximum(keys, 0.0)
        else:
            keys = -ip
        ids = np.arange(r0, r0 + xc.shape[0], dtype=np.int64)
        ck, ci = _topk_rows(keys, ids, k)
        allk = np.concatenate([bestk, ck], 1)
        alli = np.concatenate([besti, ci], 1)
        alli_key = np.where(alli < 0, np.iinfo(np.int64).max, alli)
        order = np.lexsort((alli_key, allk), axis=1)[:, :k]
        bestk = np.take_along_axis(allk, order, 1)
        besti = np.take_along_axis(alli, order, 1)
    D = bestk.copy()
    empty = besti < 0
    if metric == "l2":
        D[empty] = FLT_MAX
    else:
        D = -D
        D[empty] = -FLT_MAX
    return D, besti


def _normalize64(x: np.ndarray) -> np.ndarray:
    n = np.sqrt((x * x).sum(1, keepdims=True))
    return np.where(n > 0, x / np.where(n > 0, n, 1.0), x)


def fp32_error_bound(xb: np.ndarray, xq: np.ndarray, metric: str = "l2") -> np.ndarray:
    """Worst-case |fp32 result - exact| per (query, row) pair for this build's arithmetic.

    An fp32 dot product of length d accumulated by a chain of fused multiply-adds has error at
    most gamma_d * sum|q_i x_i| with gamma_d = d u / (1 - d u) (Higham, Accuracy and Stability of
    Numerical Algorithms, Thm 3.5); |q|^2 and |x|^2 carry gamma_d times themselves; the final
    (|q|^2 + |x|^2) - 2 ip adds <= 2 u (|q|^2 + |x|^2 + 2|ip|).  Returns an (nq, n) array for L2
    (for IP/cosine the dot-product term alone).  Used for the distance tolerance of every parity
    test and for deciding which rank positions are tie-free.
    """
    xb = np.asarray(xb, dtype=np.float64)
    xq = np.asarray(xq, dtype=np.float64)
    d = xb.shape[1]
    g = d * U32 / (1 - d * U32)
    absip = np.abs(xq) @ np.abs(xb).T
    if metric == "l2":
        qn = (xq * xq).sum(1)[:, None]
        xn = (xb * xb).sum(1)[None, :]
        return g * (qn + xn) + 2 * g * absip + 2 * U32 * (qn + xn + 2 * absip)
    if metric == "cosine":
        return (g + 4 * U32) * absip / np.maximum(
            np.sqrt((xq * xq).sum(1))[:, None] * np.sqrt((xb * xb).sum(1))[None, :], 1e-300) \
            + 4 * U32
    return g * absip + U32 * absip


def search_blas_fp32(xb: np.ndarray, xq: np.ndarray, k: int, xb_norms: np.ndarray | None = None):
    """faiss exhaustive_L2sqr_blas restated (the CPU comparator, not a checker).

    Per query block: ip = xq @ xb.T (sgemm), dis = (|q|^2 + |x|^2) - 2 ip clamped at 0, top-k by
    argpartition.  Runs on numpy's multithreaded BLAS like faiss's.
    """
    xb = np.ascontiguousarray(xb, dtype=np.float32)
    xq = np.ascontiguousarray(xq, dtype=np.float32)
    xn = (xb * xb).sum(1, dtype=np.float32) if xb_norms is None else xb_norms
    qn = (xq * xq).sum(1, dtype=np.float32)
    ip = xq @ xb.T
    dis = (qn[:, None] + xn[None, :]) - 2.0 * ip
    np.maximum(dis, 0, out=dis)
    kk = min(k, xb.shape[0])
    part = np.argpartition(dis, kk - 1, axis=1)[:, :kk]
    pd = np.take_along_axis(dis, part, 1)
    order = np.argsort(pd, axis=1, kind="stable")
    return np.take_along_axis(pd, order, 1), np.take_along_axis(part, order, 1)


def search_blas_fp32_blocked(xb: np.ndarray, xq: np.ndarray, k: int, block: int = 65536,
                             threads: int | None = None, xb_norms: np.ndarray | None = None):
    """faiss IndexFlatL2.search at a large batch, restated: exhaustive_L2sqr_blas's corpus blocking
    (the CPU comparator of bench.py, not a checker).

    faiss (faiss/utils/distances.cpp, exhaustive_L2sqr_blas) walks the corpus in blocks of bs_y
    rows, runs one sgemm of the whole query block against each corpus block, forms
    dis = |q|^2 + |x|^2 - 2 ip, and folds every block into per-query heaps with OpenMP over
    queries.  Here: one sgemm per corpus block (numpy's multithreaded BLAS), then the per-query
    top-k of the block and its merge with the running top-k by argpartition on `threads` threads
    (numpy releases the GIL in argpartition).  Returns (D float32, I int64), ascending.
    """
    from concurrent.futures import ThreadPoolExecutor
    import os
    xq = np.ascontiguousarray(xq, dtype=np.float32)
    nq, n = xq.shape[0], xb.shape[0]
    threads = threads or os.cpu_count() or 1
    qn = (xq * xq).sum(1, dtype=np.float32)
    best_d = np.full((nq, k), np.inf, np.float32)
    best_i = np.full((nq, k), -1, np.int64)
    chunks = [slice(c, min(nq, c + max(1, -(-nq // threads)))) for c in range(0, nq, max(1, -(-nq // threads)))]
    with ThreadPoolExecutor(threads) as ex:
        for r0 in range(0, n, block):
            xc = np.ascontiguousarray(xb[r0:r0 + block], dtype=np.float32)
            xn = (xc * xc).sum(1, dtype=np.float32) if xb_norms is None else xb_norms[r0:r0 + block]
            dis = xq @ xc.T
            dis *= -2.0
            dis += qn[:, None]
            dis += xn[None, :]
            np.maximum(dis, 0, out=dis)
            kk = min(k, xc.shape[0])

            def fold(s, dis=dis, kk=kk, r0=r0):
                part = np.argpartition(dis[s], kk - 1, axis=1)[:, :kk]
                cd = np.concatenate([best_d[s], np.take_along_axis(dis[s], part, 1)], 1)
                ci = np.concatenate([best_i[s], part + r0], 1)
                sel = np.argpartition(cd, k - 1, axis=1)[:, :k]
                best_d[s] = np.take_along_axis(cd, sel, 1)
                best_i[s] = np.take_along_axis(ci, sel, 1)
            list(ex.map(fold, chunks))
    order = np.argsort(best_d, axis=1, kind="stable")
    return np.take_along_axis(best_d, order, 1), np.take_along_axis(best_i, order, 1)


def recall_at_k(I: np.ndarray, I_gt: np.ndarray, k: int) -> float:
    """|I[:, :k] ∩ I_gt[:, :k]| / k averaged over queries (BASELINE.json metric)."""
    hits = 0
    for a, b in zip(I[:, :k], I_gt[:, :k]):
        hits += len(set(a[a >= 0].tolist()) & set(b[b >= 0].tolist()))
    return hits / (k * len(I))
