"""TEST INFRASTRUCTURE ONLY — IVF-PQ search arithmetic restated from faiss IndexIVFPQ semantics.

The reference builds ``faiss.IndexIVFPQ(IndexHNSWFlat(d, 32), d, nlist=2048, m, nbits=12)`` and
searches it with nprobe = 1 (/root/reference/main/create_index.py:218-228,
/root/reference/main/search_from_image.py:247).  faiss-cpu 1.10.0 (requirements.txt:2) is not
installed, so this restatement is **parity unpinned** against faiss itself; it states the
algorithm faiss documents for IndexIVFPQ with ``by_residual = True`` (no polysemous codes, no
precomputed term tables — the same distances, summed differently):

* coarse assignment: the nearest centroid (squared L2, ties by the smaller list id);
* encoding: residual r = x - c_list, sub-vector j (dims j*dsub .. ) -> nearest of the ksub
  centroids of sub-quantiser j;
* search: the nprobe nearest centroids; per probed list the table T[j][i] = |q_j - c_j - cb_ji|^2,
  a row's distance = sum_j T[j][code_j]; the k best (distance, label) over the probed rows.

The GPU kernels (csrc/ivfpq.hip) are held to ``search`` given the same centroids, codebooks and
codes; distances agree to fp32 accumulation, labels exactly outside distance ties.
"""
from __future__ import annotations

import numpy as np

FLT_MAX = float(np.finfo(np.float32).max)


def nearest(x: np.ndarray, c: np.ndarray, k: int = 1) -> np.ndarray:
    """Indices of the k nearest rows of c for each row of x (float64 squared L2, ties by index)."""
    x64, c64 = x.astype(np.float64), c.astype(np.float64)
    d = (x64 * x64).sum(1)[:, None] + (c64 * c64).sum(1)[None, :] - 2.0 * x64 @ c64.T
    order = np.lexsort((np.broadcast_to(np.arange(c.shape[0]), d.shape), d), axis=1)
    return order[:, :k]


def encode(x: np.ndarray, centroids: np.ndarray, codebooks: np.ndarray):
    """(list id, codes (n, m)) of each row; codebooks (m, ksub, dsub)."""
    m, ksub, dsub = codebooks.shape
    lists = nearest(x, centroids, 1)[:, 0]
    r = x.astype(np.float64) - centroids[lists].astype(np.float64)
    codes = np.empty((x.shape[0], m), dtype=np.int64)
    for j in range(m):
        codes[:, j] = nearest(r[:, j * dsub:(j + 1) * dsub], codebooks[j], 1)[:, 0]
    return lists, codes


def tables(rq: np.ndarray, codebooks: np.ndarray) -> np.ndarray:
    """Distance tables (nr, m, ksub) of residual queries rq (nr, d)."""
    m, ksub, dsub = codebooks.shape
    r = rq.astype(np.float64).reshape(rq.shape[0], m, 1, dsub)
    return ((r - codebooks.astype(np.float64)[None]) ** 2).sum(-1)


def search(q: np.ndarray, centroids: np.ndarray, codebooks: np.ndarray, lists: np.ndarray,
           codes: np.ndarray, ids: np.ndarray, k: int, nprobe: int = 1):
    """ADC search: (D (nq, k) float64, I (nq, k) int64), ascending, ties by the smaller label."""
    nq = q.shape[0]
    probes = nearest(q, centroids, nprobe)
    D = np.full((nq, k), FLT_MAX)
    I = np.full((nq, k), -1, dtype=np.int64)
    m = codebooks.shape[0]
    for i in range(nq):
        dist, lab = [], []
        for l in probes[i]:
            rows = np.nonzero(lists == l)[0]
            if rows.size == 0:
                continue
            T = tables((q[i].astype(np.float64) - centroids[l].astype(np.float64))[None], codebooks)[0]
            dist.append(T[np.arange(m)[None, :], codes[rows]].sum(1))
            lab.append(ids[rows])
        if not dist:
            continue
        dist, lab = np.concatenate(dist), np.concatenate(lab)
        order = np.lexsort((lab, dist))[:k]
        D[i, :order.size], I[i, :order.size] = dist[order], lab[order]
    return D, I
