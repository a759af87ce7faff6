"""Row-sharded exact k-NN over one node's GPUs.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI).  The corpus is split
into contiguous row ranges, rank r owning global labels [r*N/G, (r+1)*N/G) — the offsets table of
the reference (main/create_index.py:236-249) is unchanged by sharding.  A search runs the fused
kernel on every shard (labels already global via knn_set_id_offset), all-gathers the per-shard
(nq, k) results in one collective (keys and labels packed in one chunk, nq*k*12 bytes per rank:
latency-bound, far below one xGMI link) and merges the
G*k candidates per query with the same (key, label) order as a single-GPU search, so sharded and
unsharded results are identical.

Query x row partition (``query_groups`` Q > 1): the world is Q groups of R = world / Q ranks;
rank r holds row shard r % R of R (rows replicated Q times — a 1M x 1968 corpus is 12 GB per
copy, HBM has 288 GB) and searches query slice r // R of Q against it.  The candidate kernel does
the same MFMA work per rank as the pure row partition (its row splits keep the same length), while
every per-query cost after it — candidate merge, rerank + certificate, the packed chunk — falls by
Q.  One all-gather still moves every chunk; each rank then merges, per query slice, that slice's R
row-shard chunks.  Results are identical to the row partition's (and to one index).

The reference has no multi-device code at all; this module replaces nothing but extends
``index.search`` (main/search_from_image.py:247) to corpora larger than one GPU.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .faiss_compat import METRIC_L2, Index, _METRIC_TO_KNN


def shard_range(ntotal: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous balanced row range of `rank` (same formula as the kernel's row splits)."""
    return ntotal * rank // world, ntotal * (rank + 1) // world


def partition(world: int, rank: int, query_groups: int = 1) -> tuple[int, int, int]:
    """(query slice, row shard, row shards) of `rank` in a query_groups x (world / query_groups)
    partition (query_groups = 1: the pure row partition)."""
    if query_groups < 1 or world % query_groups:
        raise ValueError(f"query_groups={query_groups} must divide the world size {world}")
    rshards = world // query_groups
    return rank // rshards, rank % rshards, rshards


def query_slices(nq: int, query_groups: int) -> int:
    """Queries per slice, or 0 when the batch does not split evenly: then every group searches
    the whole batch and the merge reads group 0's chunks (the same answer, redundant work)."""
    return nq // query_groups if query_groups > 1 and nq % query_groups == 0 else 0


def gather_results(D, I, group=None):
    """All-gather per-rank (nq, k) results into (world, nq, k) tensors on every rank."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if world == 1:
        return D.unsqueeze(0), I.unsqueeze(0)
    gD = torch.empty((world,) + tuple(D.shape), dtype=D.dtype, device=D.device)
    gI = torch.empty((world,) + tuple(I.shape), dtype=I.dtype, device=I.device)
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(gD, D.contiguous(), group=group)
        dist.all_gather_into_tensor(gI, I.contiguous(), group=group)
    else:   # gloo (CPU tests): list form
        dist.all_gather(list(gD.unbind(0)), D.contiguous(), group=group)
        dist.all_gather(list(gI.unbind(0)), I.contiguous(), group=group)
    return gD, gI


def merge_gathered_device(gD, gI, k: int, metric: int = METRIC_L2, stream: int = 0):
    """HIP merge of gathered (world, nq, kin) device results into the final (nq, k)."""
    import torch
    world, nq, kin = gD.shape
    D = torch.empty((nq, k), dtype=torch.float32, device=gD.device)
    I = torch.empty((nq, k), dtype=torch.int64, device=gD.device)
    _lib.check(_lib.load().knn_merge_device(
        C.c_void_p(gD.data_ptr()), C.c_void_p(gI.data_ptr()), int(world), int(nq), int(kin),
        int(k), _METRIC_TO_KNN[metric], C.c_void_p(D.data_ptr()), C.c_void_p(I.data_ptr()),
        C.c_void_p(stream or None)), "knn_merge_device")
    return D, I


def packed_layout(nq: int, k: int) -> tuple[int, int]:
    """(bytes per shard chunk, byte offset of the labels) of the packed key|label layout
    (include/imgrec_knn.h knn_packed_bytes): nq*k float keys padded to an even count, then the
    nq*k int64 labels."""
    n = nq * k
    off = 4 * (n + (n & 1))
    return off + 8 * n, off


def packed_views(buf, nq: int, k: int):
    """(D, I) views (nq, k) of one packed chunk (uint8 tensor of packed_layout bytes)."""
    import torch
    nbytes, off = packed_layout(nq, k)
    D = buf[:4 * nq * k].view(torch.float32).view(nq, k)
    I = buf[off:nbytes].view(torch.int64).view(nq, k)
    return D, I


def gather_packed(buf, group=None, out=None):
    """All-gather of every rank's packed chunk in ONE collective -> (world, nbytes) uint8."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    g = out if out is not None else torch.empty((world, buf.numel()), dtype=torch.uint8,
                                                device=buf.device)
    if world == 1:
        g[0].copy_(buf)
    elif dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(g, buf, group=group)
    else:   # gloo (CPU tests): list form
        dist.all_gather(list(g.unbind(0)), buf, group=group)
    return g


def merge_packed_device(g, nq: int, kin: int, k: int, metric: int = METRIC_L2, stream: int = 0,
                        out=None):
    """HIP merge (knn_merge_packed_device) of gathered packed chunks (nchunks, nbytes) -> (nq, k)
    (out: optional contiguous (D, I) views to write into)."""
    import torch
    world = g.shape[0]
    if out is not None:
        D, I = out
    else:
        D = torch.empty((nq, k), dtype=torch.float32, device=g.device)
        I = torch.empty((nq, k), dtype=torch.int64, device=g.device)
    _lib.check(_lib.load().knn_merge_packed_device(
        C.c_void_p(g.data_ptr()), int(world), int(nq), int(kin), int(k), _METRIC_TO_KNN[metric],
        C.c_void_p(D.data_ptr()), C.c_void_p(I.data_ptr()), C.c_void_p(stream or None)),
        "knn_merge_packed_device")
    return D, I


class ShardedIndex:
    """This rank's shard of a row-partitioned exact index, plus the collective search."""

    def __init__(self, d: int, ntotal_global: int, metric: int = METRIC_L2, group=None,
                 device: int | None = None, query_groups: int = 1):
        import torch
        import torch.distributed as dist
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.d, self.metric, self.ntotal_global = int(d), metric, int(ntotal_global)
        self.query_groups = int(query_groups)
        self.qslice, self.rshard, self.rshards = partition(self.world, self.rank, self.query_groups)
        self.row0, self.row1 = shard_range(self.ntotal_global, self.rshard, self.rshards)
        dev = torch.cuda.current_device() if device is None else device
        self.device = dev
        self.index = Index(d, metric, dev)
        self.index.set_id_offset(self.row0)
        self.index.reserve(self.row1 - self.row0)
        self._packed = {}

    @property
    def local_rows(self) -> int:
        return self.row1 - self.row0

    def add_local(self, x) -> None:
        """Append rows of this shard (torch device tensor or host array, in global order)."""
        import torch
        if isinstance(x, torch.Tensor) and x.is_cuda:
            x = x.contiguous()
            self.index.add_device(x.data_ptr(), x.shape[0],
                                  torch.cuda.current_stream(x.device).cuda_stream)
        else:
            self.index.add(np.asarray(x, dtype=np.float32))

    def search(self, q, k: int, events=None):
        """q: (nq, d) float32 device tensor, identical on every rank -> (D, I) on every rank.

        events: optional 4 torch.cuda.Event recorded on the search stream before the local search,
        after it, after the all-gather and after the merge (bench.py's per-rank phase times; each
        record costs a few us of GPU time, so timed regions leave it None)."""
        import torch
        nq = q.shape[0]
        cs = torch.cuda.current_stream(q.device)
        st = cs.cuda_stream
        mark = (lambda i: events[i].record(cs)) if events is not None else (lambda i: None)
        if self.world == 1:
            D = torch.empty((nq, k), dtype=torch.float32, device=q.device)
            I = torch.empty((nq, k), dtype=torch.int64, device=q.device)
            mark(0)
            self.index.search_device(q.data_ptr(), nq, k, D.data_ptr(), I.data_ptr(), st)
            for i in (1, 2, 3):
                mark(i)
            return D, I
        # the shard searches its query slice straight into its packed chunk; one all-gather moves
        # keys and labels (chunk and gather buffers are kept per (nq, k): every call is
        # stream-ordered on them)
        per = query_slices(nq, self.query_groups)
        nql = per or nq
        ql = q[self.qslice * per:(self.qslice + 1) * per] if per else q
        key = (nq, k, q.device)
        if key not in self._packed:
            buf = torch.empty(packed_layout(nql, k)[0], dtype=torch.uint8, device=q.device)
            g = torch.empty((self.world, buf.numel()), dtype=torch.uint8, device=q.device)
            self._packed = {key: (buf, g) + packed_views(buf, nql, k)}
        buf, g, D, I = self._packed[key]
        ql = ql.contiguous()
        mark(0)
        self.index.search_device(ql.data_ptr(), nql, k, D.data_ptr(), I.data_ptr(), st)
        mark(1)
        gather_packed(buf, self.group, out=g)
        mark(2)
        if not per:      # every slice searched the whole batch: group 0's row-shard chunks
            out = merge_packed_device(g[:self.rshards], nq, k, k, self.metric, st)
            mark(3)
            return out
        Do = torch.empty((nq, k), dtype=torch.float32, device=q.device)
        Io = torch.empty((nq, k), dtype=torch.int64, device=q.device)
        for s in range(self.query_groups):   # slice s: chunks s*R .. s*R + R - 1
            merge_packed_device(g[s * self.rshards:(s + 1) * self.rshards], per, k, k, self.metric,
                                st, out=(Do[s * per:(s + 1) * per], Io[s * per:(s + 1) * per]))
        mark(3)
        return Do, Io
