"""Float64 exact top-k of a whole query batch, computed on the device (test helper, GPU tests only).

The host oracle (oracle.flat_knn.search_exact, numpy float64) takes ~1 s per query at 1M x 1968,
so the full-size tests used to check a sample of 16-32 of the 1024 queries.  This scan checks
every query in seconds: the corpus is streamed block by block (device tensors in global row
order), each block's float64 squared-L2 keys (|q|^2 + |x|^2 - 2 q.x in float64 GEMMs on the device
select a block's best; those are recomputed as sum((x - q)^2) in float64, so exact duplicates tie
exactly) are folded into a running top-k in (key, label) order — exact ties by the smaller label, faiss
IndexFlat's order — and, beside it, the top-(k-1) by faiss IndexFlatL2's own fp32 key form (fp32
GEMM per block, clamped at 0: exhaustive_L2sqr_blas restated, the `blas` input of
tests/knn_check.check_knn_tight).

It is an oracle, not the product: only tests call it.
"""
from __future__ import annotations

import numpy as np


def device_topk(torch, blocks, qs, k: int, row0: int = 0, need=None, collect_rows: bool = False):
    """blocks: iterable of (n_b, d) float32 device tensors, rows row0, row0 + 1, ... in order;
    qs: (nq, d) float32 device tensor.

    Returns (Dg float64 (nq, k), Ig int64 (nq, k), rows, (Db float32 (nq, k-1), Ib)) with labels
    global (row0-based).  rows: {label: float32 host row} for every label in `need` and every
    returned label when collect_rows (for checks without a host copy of the corpus), else {}."""
    dev = qs.device
    qd = qs.double()
    qn = (qd * qd).sum(1, keepdim=True)
    nq, d = qs.shape
    bd = torch.full((nq, k), float("inf"), dtype=torch.float64, device=dev)
    bi = torch.full((nq, k), -1, dtype=torch.int64, device=dev)
    q32 = qs.float()
    qn32 = (q32 * q32).sum(1, keepdim=True)
    kb = k - 1
    fd = torch.full((nq, kb), float("inf"), dtype=torch.float32, device=dev)
    fi = torch.full((nq, kb), -1, dtype=torch.int64, device=dev)
    if collect_rows:
        bv = torch.zeros((nq, k, d), dtype=torch.float32, device=dev)
        fv = torch.zeros((nq, kb, d), dtype=torch.float32, device=dev)
    need_t = torch.tensor(sorted(need or ()), dtype=torch.int64, device=dev)
    rows, pos = {}, row0
    imax = torch.iinfo(torch.int64).max
    for blk in blocks:
        n = blk.shape[0]
        # faiss's fp32 form
        d32 = ((qn32 + (blk * blk).sum(1)[None, :]) - 2.0 * (q32 @ blk.T)).clamp_min_(0.0)
        v32, i32 = torch.topk(d32, min(kb, n), dim=1, largest=False)
        c32, ci32 = torch.cat([fd, v32], 1), torch.cat([fi, i32 + pos], 1)
        o32 = torch.topk(c32, kb, dim=1, largest=False).indices
        if collect_rows:
            cv32 = torch.cat([fv, blk[i32]], 1)
            fv = torch.gather(cv32, 1, o32[:, :, None].expand(-1, -1, d))
        fd, fi = torch.gather(c32, 1, o32), torch.gather(ci32, 1, o32)
        del d32
        # float64 exact keys
        xd = blk.double()
        dd = (qn + (xd * xd).sum(1)[None, :] - 2.0 * (qd @ xd.T)).clamp_min_(0.0)
        # a block's k smallest keys, ties at the k-th included (topk may pick any of equal keys)
        v, i = torch.topk(dd, min(k, n), dim=1, largest=False)
        tie = (dd <= v[:, -1:] + 1e-12 * (1.0 + v[:, -1:].abs())).sum(1).max().item()
        if tie > v.shape[1]:
            v, i = torch.topk(dd, min(int(tie), n), dim=1, largest=False)
        del dd, xd
        # the selected keys again in the difference form sum((x - q)^2) (float64): the expanded
        # form leaves ~1e-16 noise on exact duplicates, which would order tied copies at random
        v = torch.stack([((blk[i[:, j]].double() - qd) ** 2).sum(1) for j in range(i.shape[1])], 1)
        cd = torch.cat([bd, v], 1)
        ci = torch.cat([bi, i + pos], 1)
        # (key, label) order: a stable sort by label, then a stable sort by key
        o1 = torch.argsort(torch.where(ci < 0, imax, ci), dim=1, stable=True)
        o2 = torch.argsort(torch.gather(cd, 1, o1), dim=1, stable=True)
        order = torch.gather(o1, 1, o2)[:, :k]
        if collect_rows:
            cv = torch.cat([bv, blk[i]], 1)
            bv = torch.gather(cv, 1, order[:, :, None].expand(-1, -1, d))
        bd, bi = torch.gather(cd, 1, order), torch.gather(ci, 1, order)
        if need_t.numel():
            hit = need_t[(need_t >= pos) & (need_t < pos + n)]
            for lab, r in zip(hit.tolist(), blk[hit - pos].cpu().numpy()):
                rows[lab] = r
        pos += n
    Ig, Ib = bi.cpu().numpy(), fi.cpu().numpy()
    if collect_rows:
        bvh, fvh = bv.cpu().numpy(), fv.cpu().numpy()
        for qi in range(nq):
            for j in range(k):
                rows[int(Ig[qi, j])] = bvh[qi, j]
            for j in range(kb):
                rows[int(Ib[qi, j])] = fvh[qi, j]
    return bd.cpu().numpy(), Ig, rows, (fd.cpu().numpy(), Ib)


def compact(rows: dict):
    """(labels sorted, stacked rows, remap) for checking against a gathered sub-corpus."""
    labels = np.array(sorted(rows))
    xb = np.stack([rows[int(l)] for l in labels])
    return labels, xb, (lambda a: np.searchsorted(labels, a))
