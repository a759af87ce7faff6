"""faiss-compatible index objects backed by the MI355X k-NN kernels (libimgrec.so).

This module is the drop-in boundary of SURVEY.md §8b: it provides exactly the faiss Python
surface that the reference's hot path touches, so ``import faiss`` in the reference can be
replaced by ``from image_recommender_amd import faiss_compat as faiss``:

================================  =================================================================
reference call                    where
================================  =================================================================
``faiss.IndexHNSWFlat(d, M)``     main/create_index.py:219, 230 (+ ``.hnsw.efConstruction/
                                  efSearch`` sets at :220-221, 231-232)
``faiss.IndexIVFPQ(q,d,nl,m,nb)`` main/create_index.py:226
``index.is_trained / train``      main/create_index.py:296-298
``index.add(arr)``                main/create_index.py:311
``index.ntotal``                  main/create_index.py:321, main/search_from_image.py:340
``faiss.write_index``             main/create_index.py:320
``faiss.read_index``              main/search_from_image.py:339
``faiss.normalize_L2``            main/search_from_image.py:322
``index.search(q, k)``            main/search_from_image.py:247, Analytics/rt_Search.py:63
================================  =================================================================

Semantics: every index class here is an EXACT flat index (the north_star parity target is
``IndexFlatL2``).  ``IndexHNSWFlat`` and ``IndexIVFPQ`` keep their constructor signatures and
attributes (``hnsw.efSearch``, ``nprobe``, ``nlist``, ...) so the reference code runs unchanged,
but they search exactly; their results are therefore the ones the reference's approximate index
approximates.  Results follow faiss conventions: ``D`` float32 (n, k), ``I`` int64 (n, k), rows
sorted best-first, missing neighbours as label -1 with distance FLT_MAX (L2) / -FLT_MAX (IP).
Exact ties are broken by the smaller label.

All arithmetic runs in the HIP kernels; there is no CPU fallback (``NativeLibraryError`` when the
library is missing, ``KnnError`` with the C-ABI message on any failure).

Several GPUs from one process: ``devices=[0, 1, ...]`` on any index class (or on ``read_index``), or
the environment variable ``IMGREC_DEVICES=0,1,...`` for code that cannot pass it — the reference's
own CLI (main/search_from_image.py:430-441) then searches row shards on every listed GPU
(include/imgrec_knn.h knn_create_multi); results are the same as on one device.
"""
from __future__ import annotations

import ctypes as C
import os
from types import SimpleNamespace

import numpy as np

from . import _lib
from ._lib import KNN_MAX_K, KnnError

METRIC_INNER_PRODUCT = 0
METRIC_L2 = 1
METRIC_COSINE = 2   # extension: rows and queries L2-normalised on entry, then inner product

_METRIC_TO_KNN = {METRIC_L2: _lib.KNN_METRIC_L2, METRIC_INNER_PRODUCT: _lib.KNN_METRIC_IP,
                  METRIC_COSINE: _lib.KNN_METRIC_COSINE}
_KNN_TO_METRIC = {v: k for k, v in _METRIC_TO_KNN.items()}


def _as_matrix(x, d: int, what: str) -> np.ndarray:
    """faiss's swig replacement_* wrappers: ``n, d = x.shape; x = ascontiguousarray(x, float32)``."""
    x = np.asarray(x)
    if x.ndim != 2:
        raise ValueError(f"{what}: expected a 2-D array, got shape {x.shape}")
    if x.shape[1] != d:
        raise ValueError(f"{what}: array has {x.shape[1]} columns, index dimension is {d}")
    return np.ascontiguousarray(x, dtype=np.float32)


def _ptr(a: np.ndarray) -> C.c_void_p:
    return C.c_void_p(a.ctypes.data)


def _device_list(device: int, devices):
    """The devices an index spans: `devices` if given, else IMGREC_DEVICES when `device` is the
    default (-1), else None (one device)."""
    if devices is None and device == -1 and os.environ.get("IMGREC_DEVICES"):
        devices = [int(v) for v in os.environ["IMGREC_DEVICES"].split(",") if v.strip()]
    if devices is None:
        return None
    devices = [int(v) for v in devices]
    if not devices:
        raise ValueError("devices must list at least one device")
    return devices


class Index:
    """Exact flat index on one HIP device, or row-sharded over several (faiss.IndexFlat
    semantics either way)."""

    def __init__(self, d: int, metric: int = METRIC_L2, device: int = -1, devices=None):
        if metric not in _METRIC_TO_KNN:
            raise ValueError(f"unsupported metric {metric}")
        self._h = None
        lib = _lib.load()
        h = C.c_void_p()
        devs = _device_list(device, devices)
        if devs is not None and len(devs) > 1:
            arr = (C.c_int * len(devs))(*devs)
            _lib.check(lib.knn_create_multi(int(d), _METRIC_TO_KNN[metric], arr, len(devs),
                                            C.byref(h)), "knn_create_multi")
        else:
            dev = devs[0] if devs else device
            _lib.check(lib.knn_create(int(d), _METRIC_TO_KNN[metric], int(dev), C.byref(h)),
                       "knn_create")
        self._h = h
        self.d = int(d)
        self.metric_type = metric
        self.verbose = False

    @classmethod
    def _wrap(cls, handle: C.c_void_p) -> "Index":
        obj = cls.__new__(cls)
        lib = _lib.load()
        obj._h = handle
        obj.d = lib.knn_dim(handle)
        obj.metric_type = _KNN_TO_METRIC[lib.knn_metric(handle)]
        obj.verbose = False
        return obj

    def __del__(self):
        h = getattr(self, "_h", None)
        lib = getattr(_lib, "_lib", None) if _lib is not None else None
        if h is not None and lib is not None:
            lib.knn_free(h)
            self._h = None

    # ---- faiss attributes -------------------------------------------------------------------
    @property
    def ntotal(self) -> int:
        return int(_lib.load().knn_ntotal(self._h))

    @property
    def is_trained(self) -> bool:
        return bool(_lib.load().knn_is_trained(self._h))

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    @property
    def num_shards(self) -> int:
        """Row shards (devices) the index spans: 1 unless created with several devices."""
        return int(_lib.load().knn_num_shards(self._h))

    # ---- faiss methods ----------------------------------------------------------------------
    def train(self, x) -> None:
        x = _as_matrix(x, self.d, "train")
        _lib.check(_lib.load().knn_train(self._h, _ptr(x), x.shape[0]), "knn_train")

    def add(self, x) -> None:
        x = _as_matrix(x, self.d, "add")
        if not self.is_trained:
            raise RuntimeError("Error in add: index is not trained (call train first)")
        _lib.check(_lib.load().knn_add(self._h, _ptr(x), x.shape[0]), "knn_add")

    def search(self, x, k: int, *, D=None, I=None):
        x = _as_matrix(x, self.d, "search")
        k = int(k)
        if k <= 0:
            raise ValueError("k must be positive")
        n = x.shape[0]
        D = np.empty((n, k), dtype=np.float32) if D is None else D
        I = np.empty((n, k), dtype=np.int64) if I is None else I
        if D.shape != (n, k) or I.shape != (n, k) or D.dtype != np.float32 or I.dtype != np.int64 \
                or not D.flags.c_contiguous or not I.flags.c_contiguous:
            raise ValueError("D/I must be C-contiguous float32/int64 arrays of shape (n, k)")
        if n:
            _lib.check(_lib.load().knn_search(self._h, _ptr(x), n, k, _ptr(D), _ptr(I)),
                       "knn_search")
        return D, I

    def reset(self) -> None:
        _lib.check(_lib.load().knn_reset(self._h), "knn_reset")

    def reconstruct_n(self, i0: int = 0, n: int | None = None) -> np.ndarray:
        n = self.ntotal - i0 if n is None else n
        out = np.empty((n, self.d), dtype=np.float32)
        _lib.check(_lib.load().knn_reconstruct_n(self._h, int(i0), int(n), _ptr(out)),
                   "knn_reconstruct_n")
        return out

    def reconstruct(self, key: int) -> np.ndarray:
        return self.reconstruct_n(int(key), 1)[0]

    # ---- device-resident entry points (multi-GPU shards, bench) ---------------------------------
    def add_device(self, x_ptr: int, n: int, stream: int = 0) -> None:
        _lib.check(_lib.load().knn_add_device(self._h, C.c_void_p(x_ptr), int(n),
                                              C.c_void_p(stream or None)), "knn_add_device")

    def search_device(self, q_ptr: int, nq: int, k: int, d_ptr: int, i_ptr: int,
                      stream: int = 0) -> None:
        _lib.check(_lib.load().knn_search_device(self._h, C.c_void_p(q_ptr), int(nq), int(k),
                                                 C.c_void_p(d_ptr), C.c_void_p(i_ptr),
                                                 C.c_void_p(stream or None)), "knn_search_device")

    def set_id_offset(self, off: int) -> None:
        _lib.check(_lib.load().knn_set_id_offset(self._h, int(off)), "knn_set_id_offset")

    def reserve(self, n: int) -> None:
        _lib.check(_lib.load().knn_reserve(self._h, int(n)), "knn_reserve")

    def set_fence_mode(self, lazy: bool) -> None:
        """Cross-stream fence of the *_device calls (include/imgrec_knn.h knn_set_fence_mode):
        lazy=True records no event while every call uses one stream, which must then stay valid
        until the next call on the index."""
        mode = _lib.KNN_FENCE_LAZY if lazy else _lib.KNN_FENCE_EAGER
        _lib.check(_lib.load().knn_set_fence_mode(self._h, mode), "knn_set_fence_mode")

    # -- search arithmetic (extension; include/imgrec_knn.h knn_search_mode) -------------------
    SEARCH_MODES = {"auto": _lib.KNN_SEARCH_AUTO, "exact": _lib.KNN_SEARCH_EXACT,
                    "split": _lib.KNN_SEARCH_SPLIT, "bf16": _lib.KNN_SEARCH_BF16,
                    "i8": _lib.KNN_SEARCH_I8}

    @property
    def search_mode(self) -> str:
        return getattr(self, "_mode", "auto")

    @search_mode.setter
    def search_mode(self, mode: str) -> None:
        if mode not in self.SEARCH_MODES:
            raise ValueError(f"search_mode must be one of {sorted(self.SEARCH_MODES)}")
        _lib.check(_lib.load().knn_set_search_mode(self._h, self.SEARCH_MODES[mode]),
                   "knn_set_search_mode")
        self._mode = mode

    def search_stats(self, with_error: bool = False):
        """(queries of the last search on a candidate path (split / bf16), of which re-run on the
        exact kernel because no certificate held)
        [+ largest observed approximation error / certificate bound, with_error=True]."""
        st = self.certificate_stats()
        return ((st["candidate_queries"], st["exact_reruns"], st["max_err_over_bound"])
                if with_error else (st["candidate_queries"], st["exact_reruns"]))

    def certificate_stats(self) -> dict:
        """The last search's certificate counts: queries on a candidate path, queries the second
        chance (all per-split list entries reranked) certified, queries re-run exactly, and the
        largest observed error / bound.  Waits for that search to finish.

        On the int8 direct route (batches of <= 4 queries, RerankArgs::direct: no merge and no
        first rerank) every query goes straight to the second chance, so there `second_chance +
        exact_reruns` equals the batch size by construction; it does not mean a first-pass
        certificate failed."""
        a, b, c, r = C.c_int64(), C.c_int64(), C.c_int64(), C.c_float()
        _lib.check(_lib.load().knn_search_stats2(self._h, C.byref(a), C.byref(b), C.byref(c),
                                                 C.byref(r)), "knn_search_stats2")
        return {"candidate_queries": a.value, "second_chance": c.value, "exact_reruns": b.value,
                "max_err_over_bound": r.value}


class IndexFlat(Index):
    def __init__(self, d: int, metric: int = METRIC_L2, device: int = -1, devices=None):
        super().__init__(d, metric, device, devices)


class IndexFlatL2(Index):
    def __init__(self, d: int, device: int = -1, devices=None):
        super().__init__(d, METRIC_L2, device, devices)


class IndexFlatIP(Index):
    def __init__(self, d: int, device: int = -1, devices=None):
        super().__init__(d, METRIC_INNER_PRODUCT, device, devices)


class IndexHNSWFlat(IndexFlatL2):
    """Constructor-compatible with ``faiss.IndexHNSWFlat(d, M[, metric])``; searches exactly.

    ``hnsw.efConstruction`` / ``hnsw.efSearch`` / ``hnsw.max_level`` are accepted and recorded
    (main/create_index.py:220-221, 231-232) but have no effect on an exact search.
    """

    def __init__(self, d: int, M: int = 32, metric: int = METRIC_L2, device: int = -1,
                 devices=None):
        Index.__init__(self, d, metric, device, devices)
        self.hnsw = SimpleNamespace(efConstruction=40, efSearch=16, max_level=0, M=int(M))


class IndexIVFPQ(Index):
    """Constructor-compatible with ``faiss.IndexIVFPQ(quantizer, d, nlist, m, nbits)``
    (main/create_index.py:226); searches exactly (nprobe is recorded, not used).

    Like faiss it starts untrained, so the reference's ``if not index.is_trained: train`` runs.
    """

    def __init__(self, quantizer, d: int, nlist: int, m: int, nbits: int = 8,
                 metric: int = METRIC_L2, device: int = -1, devices=None):
        if d % m != 0:
            raise ValueError(f"IndexIVFPQ: d={d} is not a multiple of m={m}")
        Index.__init__(self, d, metric, device, devices)
        self.quantizer = quantizer
        self.nlist, self.pq_m, self.pq_nbits = int(nlist), int(m), int(nbits)
        self.nprobe = 1
        self._trained = False

    @property
    def is_trained(self) -> bool:
        return self._trained

    def train(self, x) -> None:
        super().train(x)
        self._trained = True


def normalize_L2(x: np.ndarray) -> None:
    """In-place row L2 normalisation (faiss.normalize_L2; rows with norm 0 are left unchanged)."""
    if not isinstance(x, np.ndarray) or x.dtype != np.float32 or not x.flags.c_contiguous:
        raise TypeError("normalize_L2 expects a C-contiguous float32 numpy array")
    if x.ndim == 1:
        n, d = 1, x.shape[0]
    elif x.ndim == 2:
        n, d = x.shape
    else:
        raise ValueError("normalize_L2 expects a 1-D or 2-D array")
    if n and d:
        _lib.check(_lib.load().knn_normalize_L2(_ptr(x), n, d), "knn_normalize_L2")


def write_index(index: Index, fname) -> None:
    """Write in faiss's IndexFlat layout (fourcc IxF2 / IxFI), readable by faiss.read_index."""
    _lib.check(_lib.load().knn_write(index.handle, str(fname).encode()), "knn_write")


def read_index(fname, device: int = -1, devices=None) -> Index:
    h = C.c_void_p()
    devs = _device_list(device, devices)
    if devs is not None and len(devs) > 1:
        arr = (C.c_int * len(devs))(*devs)
        rc = _lib.load().knn_read_multi(str(fname).encode(), arr, len(devs), C.byref(h))
    else:
        rc = _lib.load().knn_read(str(fname).encode(), int(devs[0] if devs else device), C.byref(h))
    if rc < 0:
        # faiss raises RuntimeError from read_index; the recommender logs and returns None
        raise KnnError(f"read_index({fname}) failed (code {rc}): {_lib.last_error()}")
    m = _lib.load().knn_metric(h)
    cls = IndexFlatL2 if m == _lib.KNN_METRIC_L2 else (IndexFlatIP if m == _lib.KNN_METRIC_IP
                                                       else IndexFlat)
    return cls._wrap(h)


__all__ = ["Index", "IndexFlat", "IndexFlatL2", "IndexFlatIP", "IndexHNSWFlat", "IndexIVFPQ",
           "normalize_L2", "read_index", "write_index", "METRIC_L2", "METRIC_INNER_PRODUCT",
           "METRIC_COSINE", "KnnError"]
