"""Decode -> histogram pipeline for the colour feature.

The reference decodes every image with ``cv2.imread`` + ``cvtColor`` in a
``ProcessPoolExecutor(max_workers=os.cpu_count())`` and runs ``cv2.calcHist`` in the same worker
(/root/reference/vector_scripts/create_color_vector.py:46-51, 75-77;
/root/reference/vector_scripts/create_vector_base.py:242-247).  Here the CPU does only what it
must — the decode — and the histogram runs on the GPU, with the two overlapped:

* worker processes (from a forkserver, so independent of this process's GPU state) decode chunks of images with
  PIL straight into slots of ONE shared-memory ring; a slot holds a chunk's RGB bytes back to back
  (each image 48-byte aligned, so the HIP kernel's pixel-phase fast path applies) and, at its end,
  the chunk's image offsets and pixel counts;
* the ring is page-locked once (``color_host_register`` = hipHostRegister), so the parent moves a
  finished slot with one asynchronous DMA (``color_hist_batch_async``: pixels + meta H2D, then
  ``color_hist_fixed_kernel``) on a HIP stream and hands the slot back to the workers when the
  stream's event for it has completed; two device buffers alternate, so the upload of slot i+1
  overlaps the histograms of slot i, and both overlap the decoding of later chunks;
* results stay on the device until the end (one D2H copy of n x 48 floats).

Unreadable or non-RGB images give None, as the reference's worker returns None
(create_color_vector.py:38-45).  There is no CPU histogram anywhere on this path.
"""
from __future__ import annotations

import ctypes as C
import multiprocessing as mp
import os
from concurrent.futures import ProcessPoolExecutor
from multiprocessing import shared_memory
from pathlib import Path

import numpy as np

from .. import _lib
from .create_vector_base import load_image

_ALIGN = 48              # 16-B aligned and a whole number of pixels
_W = {}                  # worker-side state (set by _attach in each worker process)


def _pix_cap(slot_bytes: int, meta_cap: int) -> int:
    """Pixel bytes of a slot: what precedes its meta block, rounded down to a multiple of _ALIGN
    (an image placed at an aligned offset that fits ends within it, and so does the rounded
    offset after it)."""
    return (slot_bytes - 16 * meta_cap) // _ALIGN * _ALIGN


def _attach(shm_name: str, slot_bytes: int, meta_cap: int):
    _W["shm"] = shared_memory.SharedMemory(name=shm_name)
    _W["slot_bytes"] = slot_bytes
    _W["meta_cap"] = meta_cap


def _hold(seconds: float):
    import time
    time.sleep(seconds)
    return os.getpid()


def _decode_chunk(args):
    """Worker: decode `paths` into slot `slot`.  Returns (slot, per-image status, pixel bytes used,
    images in the slot, spilled images as arrays): status[i] = j >= 0 (j-th image of the slot),
    -1 unreadable / wrong shape, -2 spilled (did not fit the slot: returned as an array)."""
    slot, paths = args
    shm, sb, mc = _W["shm"], _W["slot_bytes"], _W["meta_cap"]
    pix_cap = _pix_cap(sb, mc)
    base = slot * sb
    buf = np.ndarray((sb,), dtype=np.uint8, buffer=shm.buf, offset=base)
    meta = np.ndarray((2 * mc,), dtype=np.int64, buffer=shm.buf, offset=base + sb - 16 * mc)
    offs, npix = [], []
    off, end, n, status, spill = 0, 0, 0, [], {}
    for i, p in enumerate(paths):
        img = load_image(p, normalize=False, as_array=True)
        if img is None or img.ndim != 3 or img.shape[2] != 3 or img.dtype != np.uint8:
            status.append(-1)
            continue
        nb = img.nbytes
        if off + nb > pix_cap or n >= mc:
            status.append(-2)
            spill[i] = np.ascontiguousarray(img)
            continue
        buf[off:off + nb] = img.reshape(-1)
        offs.append(off)
        npix.append(img.shape[0] * img.shape[1])
        status.append(n)
        n += 1
        end = off + nb                            # bytes the upload must move (<= pix_cap)
        off += (nb + _ALIGN - 1) // _ALIGN * _ALIGN
    meta[:n] = offs                               # [n offsets | n pixel counts], compact
    meta[n:2 * n] = npix
    return slot, status, end, n, spill


class ColorDecodePipeline:
    """Decode workers + a page-locked shared-memory ring + a HIP stream (see module docstring).

    ``histograms(paths)`` -> list of (3*bins,) float32 vectors (None for unreadable images), in
    input order.  Use as a context manager (or call close()).
    """

    def __init__(self, workers: int | None = None, chunk: int = 64, slot_mb: int = 16,
                 slots: int | None = None, bins: int = 16, device: int | None = None):
        import torch
        self.torch = torch
        self.workers = workers or min(16, os.cpu_count() or 1)
        self.chunk = int(chunk)
        self.bins = int(bins)
        self.nslots = slots or 2 * self.workers + 2
        self.slot_bytes = int(slot_mb) << 20
        self.meta_cap = self.chunk
        self.lib = _lib.load()
        self.shm = shared_memory.SharedMemory(create=True, size=self.nslots * self.slot_bytes)
        # the workers come from a forkserver (a fresh interpreter that never touches HIP), so they
        # are safe to start whatever GPU state this process is in; they never use the GPU
        self.pool = ProcessPoolExecutor(self.workers, mp_context=mp.get_context("forkserver"),
                                        initializer=_attach,
                                        initargs=(self.shm.name, self.slot_bytes, self.meta_cap))
        # start every worker now (not on demand inside the decode loop): each holds a task until
        # all have started
        list(self.pool.map(_hold, [0.3] * self.workers))
        self.base = C.addressof(C.c_char.from_buffer(self.shm.buf))
        rc = self.lib.color_host_register(C.c_void_p(self.base), self.nslots * self.slot_bytes)
        if rc != 0:
            self.close()
            raise _lib.KnnError(f"color_host_register failed: {self.lib.color_hist_last_error().decode()}")
        self._registered = True
        dev = torch.cuda.current_device() if device is None else device
        self.device = torch.device("cuda", dev)
        self.stream = torch.cuda.Stream(device=self.device)
        pix_cap = _pix_cap(self.slot_bytes, self.meta_cap)
        self.dev_pix = [torch.empty(pix_cap, dtype=torch.uint8, device=self.device) for _ in range(2)]
        self.dev_meta = [torch.empty(2 * self.meta_cap, dtype=torch.int64, device=self.device)
                         for _ in range(2)]

    # ------------------------------------------------------------------------------------------
    def histograms(self, paths, return_counts: bool = False):
        torch = self.torch
        paths = [str(p) for p in paths]
        n = len(paths)
        nb = 3 * self.bins
        out = torch.empty((max(n, 1), nb), dtype=torch.float32, device=self.device)
        counts = torch.empty((max(n, 1), nb), dtype=torch.int32, device=self.device) \
            if return_counts else None
        row = np.full(n, -1, dtype=np.int64)          # output row of each input (-1: None)
        spills = {}
        chunks = [list(range(i, min(i + self.chunk, n))) for i in range(0, n, self.chunk)]
        free = list(range(self.nslots))
        busy = {}                                     # slot -> event of its upload
        pending = {}                                  # future -> chunk index
        next_chunk, next_row, buf_i = 0, 0, 0
        from concurrent.futures import FIRST_COMPLETED, wait

        def reclaim(block: bool):
            for s in list(busy):
                if block or busy[s].query():
                    if block:
                        busy[s].synchronize()
                    del busy[s]
                    free.append(s)

        while next_chunk < len(chunks) or pending:
            while next_chunk < len(chunks):
                if not free:
                    reclaim(block=not pending)
                    if not free:
                        break
                s = free.pop()
                f = self.pool.submit(_decode_chunk, (s, [paths[i] for i in chunks[next_chunk]]))
                pending[f] = next_chunk
                next_chunk += 1
            if not pending:
                continue
            done, _ = wait(list(pending), return_when=FIRST_COMPLETED)
            for f in done:
                ci = pending.pop(f)
                slot, status, used, nimg, spill = f.result()
                idx = chunks[ci]
                for j, st in enumerate(status):
                    if st >= 0:
                        row[idx[j]] = next_row + st
                    elif st == -2:
                        spills[idx[j]] = spill[j]
                if nimg == 0:
                    free.append(slot)
                    continue
                b = buf_i
                buf_i ^= 1
                # device buffer b was last used two uploads ago, earlier on the same stream
                base = self.base + slot * self.slot_bytes
                meta_host = base + self.slot_bytes - 16 * self.meta_cap
                # (the two device buffers alternate on one stream: stream order protects them)
                rc = self.lib.color_hist_batch_async(
                    C.c_void_p(base), int(used), C.c_void_p(meta_host), int(nimg), self.bins,
                    C.c_void_p(self.dev_pix[b].data_ptr()), C.c_void_p(self.dev_meta[b].data_ptr()),
                    C.c_void_p(out[next_row].data_ptr()),
                    C.c_void_p(counts[next_row].data_ptr()) if counts is not None else None,
                    C.c_void_p(self.stream.cuda_stream))
                if rc != 0:
                    raise _lib.KnnError(f"color_hist_batch_async failed ({rc}): "
                                        f"{self.lib.color_hist_last_error().decode()}")
                ev = torch.cuda.Event()
                ev.record(self.stream)
                busy[slot] = ev
                next_row += nimg
            reclaim(block=False)
        self.stream.synchronize()
        reclaim(block=True)
        vecs = out[:next_row].cpu().numpy()
        cnts = counts[:next_row].cpu().numpy() if counts is not None else None
        res, res_c = [None] * n, [None] * n
        for i in range(n):
            if row[i] >= 0:
                res[i] = vecs[row[i]]
                if cnts is not None:
                    res_c[i] = cnts[row[i]].astype(np.uint32)
        if spills:                                   # images larger than a slot: one host batch
            from .create_color_vector import color_histograms
            keys = sorted(spills)
            h, c = color_histograms([spills[i] for i in keys], bins=self.bins, return_counts=True)
            for j, i in enumerate(keys):
                res[i] = h[j]
                res_c[i] = c[j]
        return (res, res_c) if return_counts else res

    # ------------------------------------------------------------------------------------------
    def close(self):
        pool = getattr(self, "pool", None)
        if pool is not None:
            pool.shutdown(wait=True)
            self.pool = None
        if getattr(self, "_registered", False):
            self.torch.cuda.synchronize(self.device)
            self.lib.color_host_unregister(C.c_void_p(self.base))
            self._registered = False
        shm = getattr(self, "shm", None)
        if shm is not None:
            self.base = None
            for attr in ("dev_pix", "dev_meta"):
                setattr(self, attr, None)
            shm.close()
            shm.unlink()
            self.shm = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def write_synthetic_images(directory, n: int, size: int = 256, seed: int = 5, fmt: str = "jpg",
                           workers: int | None = None):
    """Write n synthetic RGB images (smooth gradients + noise, like bench_pipeline's) as files;
    returns their paths.  Test and benchmark input only."""
    directory = Path(directory)
    directory.mkdir(parents=True, exist_ok=True)
    paths = [directory / f"img_{i:06d}.{fmt}" for i in range(n)]
    args = [(str(p), size, seed * 1_000_003 + i) for i, p in enumerate(paths)]
    with ProcessPoolExecutor(workers or min(16, os.cpu_count() or 1),
                             mp_context=mp.get_context("fork")) as ex:
        list(ex.map(_write_one, args, chunksize=64))
    return paths


def _write_one(args):
    from PIL import Image
    path, size, seed = args
    rng = np.random.default_rng(seed)
    a, b, c = rng.random(3), rng.random(3), rng.random(3)
    yy = np.linspace(0, 1, size)[:, None, None]
    xx = np.linspace(0, 1, size)[None, :, None]
    img = (a * yy + b * xx) * 0.7 + 0.3 * c + 0.08 * rng.standard_normal((size, size, 3))
    arr = (np.clip(img, 0, 1) * 255).astype(np.uint8)
    kw = {"quality": 92} if path.endswith(".jpg") else {}
    Image.fromarray(arr, "RGB").save(path, **kw)
