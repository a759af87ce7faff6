"""Parity checker for k-NN results against the float64 oracle (test helper).

Contract: for every query row
  1. labels are unique, in [0, ntotal) or -1 only in the padded tail (k > ntotal);
  2. position-wise |D - D_oracle| <= tol, tol = the fp32 error bound of oracle.flat_knn for the
     pairs involved (rigorous worst case of this build's fp32 arithmetic);
  3. every returned label's exact distance is within tol of the returned distance;
  4. labels equal the oracle's exactly at every rank whose oracle distance is separated from its
     neighbours' by more than 2*tol (ranks inside a tie window may permute).
"""
import numpy as np

from oracle.flat_knn import fp32_error_bound, search_exact


def _pair_bound(xb, xq, qi, ids, metric):
    ids = np.where(ids < 0, 0, ids)
    return np.array([fp32_error_bound(xb[ids[j]][None, :], xq[qi][None, :], metric)[0, 0]
                     for j in range(len(ids))])


def _exact_pair(xb, xq, qi, ids, metric):
    x = xb[np.where(ids < 0, 0, ids)].astype(np.float64)
    q = xq[qi].astype(np.float64)
    if metric == "l2":
        return ((x - q) ** 2).sum(1)
    if metric == "cosine":
        x = x / np.maximum(np.linalg.norm(x, axis=1, keepdims=True), 1e-300)
        q = q / max(np.linalg.norm(q), 1e-300)
    return x @ q


def check_knn(D, I, xb, xq, k, metric="l2", min_exact_frac=0.0, oracle=None):
    """oracle: optional precomputed search_exact(xb, xq, k + 1, metric) (reused by tests that check
    several searches of one large corpus)."""
    D = np.asarray(D, dtype=np.float64)
    I = np.asarray(I)
    n = xb.shape[0]
    Dg, Ig = oracle if oracle is not None else search_exact(xb, xq, k + 1, metric)
    assert Dg.shape[1] >= k + 1
    assert D.shape == (xq.shape[0], k) and I.shape == (xq.shape[0], k)
    checked = total = 0
    for q in range(xq.shape[0]):
        row, drow = I[q], D[q]
        valid = row >= 0
        nvalid = min(k, n)
        assert valid[:nvalid].all() and not valid[nvalid:].any(), (q, row)
        assert len(set(row[valid].tolist())) == valid.sum(), f"duplicate labels in row {q}: {row}"
        assert (row[valid] < n).all()
        if nvalid < k:
            pad = np.finfo(np.float32).max * (1 if metric == "l2" else -1)
            assert (drow[nvalid:] == pad).all()
        if nvalid == 0:
            continue
        ids = row[:nvalid]
        tol = np.maximum(_pair_bound(xb, xq, q, ids, metric),
                         _pair_bound(xb, xq, q, Ig[q, :nvalid], metric)) * 1.0001 + 1e-30
        assert np.all(np.abs(drow[:nvalid] - Dg[q, :nvalid]) <= tol), \
            (q, drow[:nvalid], Dg[q, :nvalid], tol)
        ex = _exact_pair(xb, xq, q, ids, metric)
        assert np.all(np.abs(ex - drow[:nvalid]) <= tol), (q, ex, drow[:nvalid])
        gd = Dg[q]
        for j in range(nvalid):
            lo = j == 0 or abs(gd[j] - gd[j - 1]) > 2 * tol[j]
            hi = (j + 1 >= len(gd)) or Ig[q, j + 1] < 0 or abs(gd[j + 1] - gd[j]) > 2 * tol[j]
            total += 1
            if lo and hi:
                checked += 1
                assert row[j] == Ig[q, j], (q, j, row, Ig[q])
    if total:
        assert checked / total >= min_exact_frac, (checked, total)
    return checked, total
