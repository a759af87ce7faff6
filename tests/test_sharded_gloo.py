"""Multi-process (world size 2 and 3, gloo, CPU) test of the row-sharded search protocol (§8e).

What runs on the GPU in production — each shard's fused search and the final merge — is replaced
by the float64 oracle here; everything else is the product code: ``shard_range`` (contiguous
balanced row ranges, labels = global offsets), ``gather_results`` (the all-gather into the
[world][nq][k] layout that knn_merge_device consumes).  The merged result must equal an unsharded
search of the whole corpus, labels included.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.datagen import mixture


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _merge_oracle(gD, gI, k, metric):
    """Reference semantics of knn_merge_device: best k of the gathered lists by (key, label)."""
    world, nq, kin = gD.shape
    D = np.empty((nq, k), np.float64)
    I = np.empty((nq, k), np.int64)
    for q in range(nq):
        d = gD[:, q, :].reshape(-1)
        i = gI[:, q, :].reshape(-1)
        ok = i >= 0
        key = d[ok] if metric == "l2" else -d[ok]
        order = np.lexsort((i[ok], key))[:k]
        n = len(order)
        D[q, :n], I[q, :n] = d[ok][order], i[ok][order]
        D[q, n:], I[q, n:] = (np.finfo(np.float32).max if metric == "l2" else -np.finfo(np.float32).max), -1
    return D, I


def _worker(rank, world, port, n, d, nq, k, metric, out, packed=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from image_recommender_amd.sharded import (gather_packed, gather_results, packed_layout,
                                                   packed_views, shard_range)
        from oracle.flat_knn import search_exact
        xb = mixture(n, d, centres=30, seed=11)
        xq = mixture(nq, d, centres=30, seed=12)
        r0, r1 = shard_range(n, rank, world)
        D, I = search_exact(xb[r0:r1], xq, k, metric)
        I = np.where(I >= 0, I + r0, -1)                # knn_set_id_offset(r0)
        if packed:      # ShardedIndex.search's layout: the shard writes into its packed chunk
            buf = torch.zeros(packed_layout(nq, k)[0], dtype=torch.uint8)
            pD, pI = packed_views(buf, nq, k)
            pD.copy_(torch.from_numpy(D.astype(np.float32)))
            pI.copy_(torch.from_numpy(I))
            g = gather_packed(buf)
            views = [packed_views(g[r], nq, k) for r in range(world)]
            gD = np.stack([v[0].numpy() for v in views])
            gI = np.stack([v[1].numpy() for v in views])
            D = D.astype(np.float32).astype(np.float64)   # what the packed chunk carries
        else:
            gD, gI = gather_results(torch.from_numpy(D), torch.from_numpy(I))
            gD, gI = gD.numpy(), gI.numpy()
        Dm, Im = _merge_oracle(gD, gI, k, metric)
        if rank == 0:
            out.put((Dm, Im, [shard_range(n, r, world) for r in range(world)]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n,k,metric,packed", [(2, 3001, 10, "l2", False),
                                                     (3, 1000, 7, "ip", False),
                                                     (2, 5, 8, "l2", False),
                                                     (2, 3001, 10, "l2", True),
                                                     (3, 1000, 7, "ip", True),
                                                     (3, 7, 3, "l2", True)])
def test_row_sharded_search_equals_unsharded(world, n, k, metric, packed):
    """packed=True: ShardedIndex.search's single-collective layout (keys and labels in one chunk
    per rank, odd nq*k padded) through gather_packed / packed_views."""
    from oracle.flat_knn import search_exact
    ctx = mp.get_context("spawn")
    out = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, 24, 9, k, metric, out, packed))
             for r in range(world)]
    for p in procs:
        p.start()
    Dm, Im, ranges = out.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # contiguous, balanced, covering
    assert ranges[0][0] == 0 and ranges[-1][1] == n
    assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
    assert max(r1 - r0 for r0, r1 in ranges) - min(r1 - r0 for r0, r1 in ranges) <= 1
    xb = mixture(n, 24, centres=30, seed=11)
    xq = mixture(9, 24, centres=30, seed=12)
    D, I = search_exact(xb, xq, k, metric)
    if packed:      # the chunk carries float32 keys
        D = np.where(I >= 0, D.astype(np.float32).astype(np.float64), D)
    np.testing.assert_array_equal(Im, I)
    np.testing.assert_allclose(Dm, D, rtol=0, atol=0)


def _worker_qr(rank, world, qgroups, port, n, d, nq, k, metric, out):
    """ShardedIndex.search's query x row partition with the oracle in place of the GPU search and
    merge: rank -> (query slice, row shard) by `partition`, the slice's chunk packed and gathered
    in one collective, each slice merged from its row-shard chunks."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from image_recommender_amd.sharded import (gather_packed, packed_layout, packed_views,
                                                   partition, query_slices, shard_range)
        from oracle.flat_knn import search_exact
        xb = mixture(n, d, centres=30, seed=21)
        xq = mixture(nq, d, centres=30, seed=22)
        qs, rs, R = partition(world, rank, qgroups)
        r0, r1 = shard_range(n, rs, R)
        per = query_slices(nq, qgroups)
        nql = per or nq
        ql = xq[qs * per:(qs + 1) * per] if per else xq
        D, I = search_exact(xb[r0:r1], ql, k, metric)
        I = np.where(I >= 0, I + r0, -1)
        buf = torch.zeros(packed_layout(nql, k)[0], dtype=torch.uint8)
        pD, pI = packed_views(buf, nql, k)
        pD.copy_(torch.from_numpy(D.astype(np.float32)))
        pI.copy_(torch.from_numpy(I))
        g = gather_packed(buf)
        views = [packed_views(g[c], nql, k) for c in range(world)]
        Dm = np.empty((nq, k)); Im = np.empty((nq, k), np.int64)
        for s in range(qgroups if per else 1):
            ch = range(s * R, (s + 1) * R)
            gD = np.stack([views[c][0].numpy() for c in ch]).astype(np.float64)
            gI = np.stack([views[c][1].numpy() for c in ch])
            sl = slice(s * per, (s + 1) * per) if per else slice(0, nq)
            Dm[sl], Im[sl] = _merge_oracle(gD, gI, k, metric)
        if rank == 0:
            out.put((Dm, Im))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,qgroups,n,nq,k,metric", [(4, 2, 3001, 10, 10, "l2"),
                                                         (4, 2, 1000, 9, 7, "ip"),
                                                         (2, 2, 500, 8, 5, "l2"),
                                                         (4, 4, 777, 12, 4, "l2")])
def test_query_row_partition_equals_unsharded(world, qgroups, n, nq, k, metric):
    """query_groups > 1: equal to an unsharded search (nq = 9 with 2 groups: the uneven batch
    falls back to every group searching all queries)."""
    from oracle.flat_knn import search_exact
    from image_recommender_amd.sharded import partition
    with pytest.raises(ValueError):
        partition(4, 0, 3)
    ctx = mp.get_context("spawn")
    out = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_qr, args=(r, world, qgroups, port, n, 24, nq, k, metric, out))
             for r in range(world)]
    for p in procs:
        p.start()
    Dm, Im = out.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    xb = mixture(n, 24, centres=30, seed=21)
    xq = mixture(nq, 24, centres=30, seed=22)
    D, I = search_exact(xb, xq, k, metric)
    D = np.where(I >= 0, D.astype(np.float32).astype(np.float64), D)
    np.testing.assert_array_equal(Im, I)
    np.testing.assert_allclose(Dm, D, rtol=0, atol=0)
