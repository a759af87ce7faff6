"""ShardedIndex.search end to end on the GPU: two ranks (gloo, both on cuda:0 — the 8-GPU RCCL run
belongs to the driver) each hold a row shard, search into their packed chunk, gather it in one
collective and merge with knn_merge_packed_device; the result equals one index over all rows
(SURVEY.md §8e), and both agree with the float64 oracle (tests/knn_check.py contract)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def faiss(gpu):
    from image_recommender_amd import faiss_compat
    return faiss_compat


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, d, nq, k, mode, out, qgroups=1):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from image_recommender_amd.faiss_compat import METRIC_L2
        from image_recommender_amd.sharded import ShardedIndex
        from tests.datagen import mixture
        torch.cuda.set_device(0)
        xb = mixture(n, d, centres=40, seed=31)
        xq = torch.from_numpy(mixture(nq, d, centres=40, seed=32)).cuda()
        sh = ShardedIndex(d, n, METRIC_L2, device=0, query_groups=qgroups)
        sh.add_local(xb[sh.row0:sh.row1])
        sh.index.search_mode = mode
        for _ in range(2):                                  # second call: cached chunk buffers
            D, I = sh.search(xq, k)
        torch.cuda.synchronize()
        if rank == 0:
            out.put((D.cpu().numpy(), I.cpu().numpy(), sh.index.search_stats()[1]))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n,d,nq,k,mode,world,qgroups", [
    (20000, 96, 64, 10, "exact", 2, 1), (30000, 256, 600, 10, "bf16", 2, 1), (4001, 64, 7, 5, "exact", 2, 1),
    # query x row partition: 2 query slices x 2 row shards; 2 slices of the whole corpus; an
    # uneven batch (every slice searches all 7 queries)
    (30000, 256, 600, 10, "bf16", 4, 2), (20000, 96, 64, 10, "exact", 2, 2), (4001, 64, 7, 5, "exact", 4, 2),
    # k > KNN_MAX_K: per-shard GEMM + select, the packed large-k merge
    (20000, 96, 33, 120, "auto", 2, 1)])
def test_sharded_search_two_ranks_equals_one_index(faiss, n, d, nq, k, mode, world, qgroups):
    import torch.multiprocessing as mp
    from tests.datagen import mixture
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, d, nq, k, mode, q, qgroups))
             for r in range(world)]
    for p in procs:
        p.start()
    D, I, fallbacks = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    xb, xq = mixture(n, d, centres=40, seed=31), mixture(nq, d, centres=40, seed=32)
    full = faiss.IndexFlatL2(d)
    full.add(xb)
    full.search_mode = mode
    Df, If = full.search(xq, k)
    from tests.knn_check import check_knn
    check_knn(D, I, xb, xq, k, "l2", min_exact_frac=0.5)      # the sharded result vs the oracle
    if fallbacks or full.search_stats()[1]:
        assert (I == If).mean() > 0.99
        return
    if k > 32:      # the GEMM + select path: rounding follows the GEMM's blocking (per shard)
        np.testing.assert_allclose(D, Df, rtol=1e-6, atol=1e-6)
        assert (I == If).mean() > 0.99
        return
    np.testing.assert_array_equal(I, If)
    np.testing.assert_array_equal(D, Df)
