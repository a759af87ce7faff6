"""GPU IVF-PQ index — the reference's default index structure.

The reference builds ``faiss.IndexIVFPQ(IndexHNSWFlat(d, 32), d, nlist=2048, m, nbits=12)`` and
searches it with nprobe = 1 (/root/reference/main/create_index.py:207-234, 296-311;
main/search_from_image.py:247).  The exact index (faiss_compat.IndexFlatL2 / include/imgrec_knn.h)
stays the parity target and the default everywhere; this class is the approximate alternative
with the same structure, for fidelity with the reference's footprint and recall:

* training: Lloyd k-means for the nlist coarse centroids, then one k-means per sub-quantiser on
  the residual sub-vectors (ksub = 2^nbits centroids each); assignment steps run on the exact
  k-NN kernels (k = 1), centroid updates are tensor reductions;
* add: coarse assignment + residual encoding on the same kernels; rows are kept list-contiguous
  (codes as uint16 per sub-quantiser, labels int64, list offsets) in HBM;
* search: the nprobe nearest centroids (exact k-NN), per (query, probe) the distance table
  (``ivfpq_lut_device``) and the ADC scan of the probed lists (``ivfpq_scan_device``), both
  hand-written gfx950 kernels (csrc/ivfpq.hip).

Differences from faiss, stated: the coarse quantiser is exact (faiss's HNSW quantiser is itself
approximate); codes take 2 bytes per sub-quantiser (faiss packs nbits); k-means initialisation
and empty-cluster handling follow faiss's description (seeded random sample; an empty cluster
takes a random training point) but do not reproduce its random stream.  Parity is pinned
against oracle/ivfpq.py given the same centroids, codebooks and codes.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import KNN_MAX_K
from .faiss_compat import METRIC_L2, IndexFlatL2

__all__ = ["IndexIVFPQ"]


def _torch():
    import torch
    return torch


class IndexIVFPQ:
    """faiss.IndexIVFPQ-shaped GPU index (L2, by-residual PQ, ADC search)."""

    def __init__(self, d: int, nlist: int, m: int, nbits: int = 8, metric: int = METRIC_L2,
                 device: int = 0, niter: int = 10, pq_niter: int = 10, seed: int = 1234,
                 max_points_per_centroid: int = 256):
        if metric != METRIC_L2:
            raise ValueError("IndexIVFPQ: only METRIC_L2 (the reference's metric) is supported")
        if d % m != 0:
            raise ValueError(f"IndexIVFPQ: d={d} is not a multiple of m={m}")
        if d // m > 256:
            raise ValueError("IndexIVFPQ: sub-vectors longer than 256 are not supported")
        if not 1 <= nbits <= 16:
            raise ValueError("IndexIVFPQ: nbits must be in [1, 16]")
        torch = _torch()
        self.d, self.nlist, self.m, self.nbits = int(d), int(nlist), int(m), int(nbits)
        self.dsub, self.ksub = self.d // self.m, 1 << self.nbits
        self.metric_type = metric
        self.niter, self.pq_niter, self.seed = int(niter), int(pq_niter), int(seed)
        self.max_points_per_centroid = int(max_points_per_centroid)
        self.nprobe = 1
        self.device = torch.device("cuda", device if device >= 0 else torch.cuda.current_device())
        self.is_trained = False
        self.centroids = None          # (nlist, d) float32
        self.codebooks = None          # (m, ksub, dsub) float32
        self._cbt = None               # (m, dsub, ksub) float32, the kernels' layout
        self._lists = torch.empty(0, dtype=torch.int64, device=self.device)   # list of each row
        self._codes = torch.empty((0, self.m), dtype=torch.int16, device=self.device)
        self._ids = torch.empty(0, dtype=torch.int64, device=self.device)
        self._list_off = torch.zeros(self.nlist + 1, dtype=torch.int64, device=self.device)

    # ---- helpers ----------------------------------------------------------------------------
    @property
    def ntotal(self) -> int:
        return int(self._ids.numel())

    def _tensor(self, x):
        torch = _torch()
        if isinstance(x, torch.Tensor):
            t = x.to(self.device, torch.float32)
        else:
            t = torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).to(self.device)
        if t.dim() != 2:
            raise ValueError("expected a 2-D array")
        return t.contiguous()

    def _flat(self, c):
        """Exact fp32 k-NN index over the rows of c."""
        torch = _torch()
        idx = IndexFlatL2(c.shape[1], device=self.device.index)
        idx.search_mode = "exact"
        c = c.contiguous()
        idx.add_device(c.data_ptr(), c.shape[0], torch.cuda.current_stream(self.device).cuda_stream)
        return idx

    def _nearest(self, x, c, k: int = 1, idx=None):
        """(n, k) int64 indices of the k nearest rows of c (exact fp32 k-NN kernels)."""
        torch = _torch()
        temp = idx is None
        idx = self._flat(c) if temp else idx
        st = torch.cuda.current_stream(self.device).cuda_stream
        n = x.shape[0]
        D = torch.empty((n, k), dtype=torch.float32, device=self.device)
        I = torch.empty((n, k), dtype=torch.int64, device=self.device)
        for r0 in range(0, n, 1 << 20):
            r1 = min(n, r0 + (1 << 20))
            xs = x[r0:r1].contiguous()
            idx.search_device(xs.data_ptr(), r1 - r0, k, D[r0:r1].data_ptr(), I[r0:r1].data_ptr(), st)
        if temp:        # the temporary index's memory must outlive the enqueued search
            torch.cuda.synchronize(self.device)
        return I

    def _kmeans(self, x, k: int, niter: int, seed: int):
        torch = _torch()
        n = x.shape[0]
        if n < k:
            raise ValueError(f"k-means: {n} training points for {k} centroids")
        g = torch.Generator(device="cpu").manual_seed(seed)
        c = x[torch.randperm(n, generator=g)[:k].to(self.device)].clone()
        for _ in range(niter):
            a = self._nearest(x, c)[:, 0]
            cnt = torch.bincount(a, minlength=k)
            s = torch.zeros_like(c).index_add_(0, a, x)
            nz = cnt > 0
            c[nz] = s[nz] / cnt[nz, None].to(x.dtype)
            empty = torch.nonzero(~nz).flatten()
            if empty.numel():       # faiss splits a large cluster; here: a random training point
                c[empty] = x[torch.randint(0, n, (empty.numel(),), generator=g).to(self.device)]
        return c

    def _sample(self, x, cap: int, seed: int):
        torch = _torch()
        if x.shape[0] <= cap:
            return x
        g = torch.Generator(device="cpu").manual_seed(seed)
        return x[torch.randperm(x.shape[0], generator=g)[:cap].to(self.device)].contiguous()

    # ---- faiss methods ----------------------------------------------------------------------
    def train(self, x) -> None:
        x = self._tensor(x)
        xs = self._sample(x, self.max_points_per_centroid * self.nlist, self.seed)
        cen = self._kmeans(xs, self.nlist, self.niter, self.seed)
        r = xs - cen[self._nearest(xs, cen)[:, 0]]
        books = []
        for j in range(self.m):
            sub = self._sample(r[:, j * self.dsub:(j + 1) * self.dsub].contiguous(),
                               self.max_points_per_centroid * self.ksub, self.seed + 1 + j)
            books.append(self._kmeans(sub, self.ksub, self.pq_niter, self.seed + 1 + j))
        self._set(cen, _torch().stack(books))

    def set_trained(self, centroids, codebooks) -> None:
        """Install trained parameters: centroids (nlist, d), codebooks (m, ksub, dsub)."""
        torch = _torch()
        cen = self._tensor(centroids)
        cb = codebooks if isinstance(codebooks, torch.Tensor) else \
            torch.from_numpy(np.ascontiguousarray(codebooks, dtype=np.float32))
        cb = cb.to(self.device, torch.float32)
        if tuple(cen.shape) != (self.nlist, self.d) or tuple(cb.shape) != (self.m, self.ksub, self.dsub):
            raise ValueError("set_trained: wrong centroid / codebook shapes")
        self._set(cen, cb)

    def _set(self, cen, cb) -> None:
        self.centroids = cen.contiguous()
        self._coarse = self._flat(self.centroids)       # the coarse quantiser, kept resident
        self.codebooks = cb.contiguous()
        self._cbt = cb.permute(0, 2, 1).contiguous()
        self.is_trained = True

    def encode(self, x):
        """(list id (n,), codes (n, m) int64) of the rows of x."""
        torch = _torch()
        x = self._tensor(x)
        lists = self._nearest(x, self.centroids, 1, self._coarse)[:, 0]
        r = x - self.centroids[lists]
        codes = torch.empty((x.shape[0], self.m), dtype=torch.int64, device=self.device)
        for j in range(self.m):
            codes[:, j] = self._nearest(r[:, j * self.dsub:(j + 1) * self.dsub].contiguous(),
                                        self.codebooks[j])[:, 0]
        return lists, codes

    def add(self, x) -> None:
        if not self.is_trained:
            raise RuntimeError("Error in add: index is not trained (call train first)")
        torch = _torch()
        x = self._tensor(x)
        lists, codes = self.encode(x)
        ids = torch.arange(self.ntotal, self.ntotal + x.shape[0], dtype=torch.int64, device=self.device)
        self.add_encoded(lists, codes, ids)

    def add_encoded(self, lists, codes, ids) -> None:
        """Append pre-encoded rows (list id, codes, label); rows stay list-contiguous, each list in
        insertion order."""
        torch = _torch()
        lists = torch.as_tensor(lists, device=self.device).to(torch.int64).flatten()
        codes = torch.as_tensor(codes, device=self.device).to(torch.int64).reshape(-1, self.m)
        ids = torch.as_tensor(ids, device=self.device).to(torch.int64).flatten()
        if not (lists.numel() == codes.shape[0] == ids.numel()):
            raise ValueError("add_encoded: lists, codes and ids disagree in length")
        if lists.numel() and (int(lists.min()) < 0 or int(lists.max()) >= self.nlist):
            raise ValueError("add_encoded: list id out of range")
        if codes.numel() and (int(codes.min()) < 0 or int(codes.max()) >= self.ksub):
            raise ValueError("add_encoded: code out of range")
        if ids.numel() and int(ids.max()) >= 2 ** 31:
            raise ValueError("add_encoded: labels must be < 2^31")
        all_lists = torch.cat([self._lists, lists])
        all_codes = torch.cat([self._codes.to(torch.int64) & 0xffff, codes])
        all_ids = torch.cat([self._ids, ids])
        order = torch.sort(all_lists, stable=True).indices
        self._lists = all_lists[order].contiguous()
        # uint16 codes stored in an int16 tensor (same bytes; torch has no uint16 arithmetic)
        self._codes = all_codes[order].to(torch.int32).to(torch.int16).contiguous()
        self._ids = all_ids[order].contiguous()
        cnt = torch.bincount(self._lists, minlength=self.nlist)
        self._list_off = torch.zeros(self.nlist + 1, dtype=torch.int64, device=self.device)
        self._list_off[1:] = torch.cumsum(cnt, 0)

    def search(self, x, k: int):
        """(D, I) numpy (nq, k): squared-L2 ADC distances ascending, ties by the smaller label; any k
        (k <= 32: per-lane register lists; beyond: every probed row keyed and sorted per query)."""
        torch = _torch()
        if not self.is_trained:
            raise RuntimeError("Error in search: index is not trained")
        k = int(k)
        if k < 1:
            raise ValueError("k must be positive")
        q = self._tensor(x)
        nq, npb = q.shape[0], max(1, min(int(self.nprobe), self.nlist))
        D = torch.empty((nq, k), dtype=torch.float32, device=self.device)
        I = torch.empty((nq, k), dtype=torch.int64, device=self.device)
        if nq == 0:
            return D.cpu().numpy(), I.cpu().numpy()
        lib = _lib.load()
        st = torch.cuda.current_stream(self.device).cuda_stream
        chunk = max(1, (1 << 30) // (npb * self.m * self.ksub * 4))     # <= 1 GB of tables
        for q0 in range(0, nq, chunk):
            q1 = min(nq, q0 + chunk)
            qc = q[q0:q1]
            probes = self._nearest(qc, self.centroids, npb, self._coarse).contiguous()
            resid = (qc[:, None, :] - self.centroids[probes]).reshape(-1, self.d).contiguous()
            lut = torch.empty((resid.shape[0], self.m, self.ksub), dtype=torch.float32, device=self.device)
            _lib.check(lib.ivfpq_lut_device(C.c_void_p(resid.data_ptr()), resid.shape[0], self.d,
                                            self.m, self.ksub, C.c_void_p(self._cbt.data_ptr()),
                                            C.c_void_p(lut.data_ptr()), C.c_void_p(st)),
                       "ivfpq_lut_device")
            if k <= KNN_MAX_K:      # register top-k lists per lane (ivfpq_scan_kernel)
                _lib.check(lib.ivfpq_scan_device(C.c_void_p(lut.data_ptr()), C.c_void_p(probes.data_ptr()),
                                                 q1 - q0, npb, C.c_void_p(self._list_off.data_ptr()),
                                                 C.c_void_p(self._codes.data_ptr()),
                                                 C.c_void_p(self._ids.data_ptr()), self.m, self.ksub, k,
                                                 C.c_void_p(D[q0:q1].data_ptr()),
                                                 C.c_void_p(I[q0:q1].data_ptr()), C.c_void_p(st)),
                           "ivfpq_scan_device")
                continue
            # any k: every probed row's ADC key, sorted per query (ivfpq_scan_all_device); the
            # slots of each (query, probe) and each query come from the probed lists' sizes
            pr = probes.reshape(-1)
            cnt = torch.where(pr >= 0, self._list_off[pr.clamp_min(0) + 1] - self._list_off[pr.clamp_min(0)],
                              torch.zeros_like(pr))
            probe_off = (torch.cumsum(cnt, 0) - cnt).contiguous()
            total = int(cnt.sum())
            qoff = torch.cat([probe_off.reshape(q1 - q0, npb)[:, 0],
                              torch.tensor([total], dtype=torch.int64, device=self.device)])
            if total >= 2 ** 32:
                raise ValueError("IVF-PQ search: more than 2^32 probed entries in one chunk")
            seg_off = qoff.to(torch.int32).contiguous()     # (the int32 bits are the uint32 offsets)
            _lib.check(lib.ivfpq_scan_all_device(C.c_void_p(lut.data_ptr()), C.c_void_p(probes.data_ptr()),
                                                 q1 - q0, npb, C.c_void_p(self._list_off.data_ptr()),
                                                 C.c_void_p(self._codes.data_ptr()),
                                                 C.c_void_p(self._ids.data_ptr()), self.m, self.ksub,
                                                 C.c_void_p(probe_off.data_ptr()),
                                                 C.c_void_p(seg_off.data_ptr()), total, k,
                                                 C.c_void_p(D[q0:q1].data_ptr()),
                                                 C.c_void_p(I[q0:q1].data_ptr()), C.c_void_p(st)),
                       "ivfpq_scan_all_device")
        torch.cuda.synchronize(self.device)
        return D.cpu().numpy(), I.cpu().numpy()

    # ---- persistence ----------------------------------------------------------------------------
    def write(self, path) -> None:
        """Save to an .npz file (plain arrays; read back with ``IndexIVFPQ.read``).  faiss's own
        IVF-PQ file layout is not reproduced (it would need faiss to verify)."""
        if not self.is_trained:
            raise RuntimeError("write: index is not trained")
        lists, codes, ids = self.list_contents()
        with open(path, "wb") as f:
            np.savez(f, header=np.array([self.d, self.nlist, self.m, self.nbits, self.nprobe], np.int64),
                     centroids=self.centroids.cpu().numpy(), codebooks=self.codebooks.cpu().numpy(),
                     lists=lists, codes=codes.astype(np.uint16), ids=ids)

    @classmethod
    def read(cls, path, device: int = 0) -> "IndexIVFPQ":
        with np.load(path, allow_pickle=False) as z:
            d, nlist, m, nbits, nprobe = (int(v) for v in z["header"])
            idx = cls(d, nlist, m, nbits, device=device)
            idx.set_trained(z["centroids"], z["codebooks"])
            idx.add_encoded(z["lists"], z["codes"].astype(np.int64), z["ids"])
        idx.nprobe = nprobe
        return idx

    # ---- introspection (tests) ----------------------------------------------------------------
    def list_contents(self):
        """(list id, codes (n, m) int64, labels) of the stored rows, in storage order (numpy)."""
        return (self._lists.cpu().numpy(), (self._codes.to(_torch().int64) & 0xffff).cpu().numpy(),
                self._ids.cpu().numpy())
