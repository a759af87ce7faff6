"""Colour-histogram features on the MI355X — drop-in for vector_scripts/create_color_vector.py.

The reference (/root/reference/vector_scripts/create_color_vector.py:12-78) decodes every image
with OpenCV in a ProcessPoolExecutor and runs cv2.calcHist (16 bins per channel, R|G|B, then L2
normalisation) per image.  Here a batch of decoded images is packed into one byte buffer and the
HIP kernel ``color_hist_device`` (csrc/color_hist.hip) computes all histograms in one launch.
``compute_vectors`` (the indexer's batch path, reference :54-78) streams files through
``decode_pipeline.ColorDecodePipeline``: worker processes decode into a page-locked shared-memory
ring, batches are DMA'd to the GPU and histogrammed while later files decode.  Output: one
(3*bins,) float32 vector per image, None for unreadable images, exactly like ``compute_vectors``
of the reference.
"""
from __future__ import annotations

import ctypes as C
import os
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path
from typing import Sequence

import numpy as np

from .. import _lib
from .create_vector_base import BaseVectorIndexer, load_image


def color_histograms(images: Sequence[np.ndarray], bins: int = 16, device: int = -1,
                     return_counts: bool = False):
    """HIP colour histograms of HxWx3 uint8 RGB images -> (n, 3*bins) float32 (L2-normalised)."""
    n = len(images)
    nb = 3 * bins
    out = np.zeros((n, nb), np.float32)
    counts = np.zeros((n, nb), np.uint32) if return_counts else None
    if n == 0:
        return (out, counts) if return_counts else out
    arrs = []
    for im in images:
        a = np.asarray(im)
        if a.ndim != 3 or a.shape[2] != 3 or a.dtype != np.uint8:
            raise ValueError(f"expected HxWx3 uint8 images, got {a.shape} {a.dtype}")
        arrs.append(np.ascontiguousarray(a))
    npix = np.array([a.shape[0] * a.shape[1] for a in arrs], np.int64)
    offsets = np.zeros(n, np.int64)
    np.cumsum(3 * npix[:-1], out=offsets[1:])
    buf = np.concatenate([a.reshape(-1) for a in arrs])
    lib = _lib.load()
    rc = lib.color_hist_host(buf.ctypes.data, int(buf.nbytes), offsets.ctypes.data,
                             npix.ctypes.data, n, int(bins), int(device), out.ctypes.data,
                             counts.ctypes.data if counts is not None else None)
    if rc != 0:
        raise _lib.KnnError(f"color_hist_host failed ({rc}): "
                            f"{lib.color_hist_last_error().decode()}")
    return (out, counts) if return_counts else out


def color_histograms_device(pixels, offsets, npix, bins: int = 16):
    """Device-resident variant (torch tensors on one HIP device): uint8 pixels (total bytes),
    int64 offsets/npix (n) -> (n, 3*bins) float32 tensor, on the current torch stream."""
    import torch
    n = int(offsets.numel())
    out = torch.empty((n, 3 * bins), dtype=torch.float32, device=pixels.device)
    lib = _lib.load()
    rc = lib.color_hist_device(C.c_void_p(pixels.data_ptr()), C.c_void_p(offsets.data_ptr()),
                               C.c_void_p(npix.data_ptr()), n, int(bins),
                               C.c_void_p(out.data_ptr()), None,
                               C.c_void_p(torch.cuda.current_stream(pixels.device).cuda_stream or None))
    if rc != 0:
        raise _lib.KnnError(f"color_hist_device failed ({rc}): "
                            f"{lib.color_hist_last_error().decode()}")
    return out


class ColorVectorIndexer(BaseVectorIndexer):
    table_name = "color_vectors"
    vector_column = "color_vector_blob"
    id_column = "image_id"
    bins = 16

    @classmethod
    def compute_paths(cls, paths, images_dir, bins=None, workers=None):
        bins = bins or cls.bins
        images_dir = Path(images_dir)

        def decode(p):
            p = Path(p)
            return load_image(p if p.is_absolute() else images_dir / p, normalize=False,
                              as_array=True)

        with ThreadPoolExecutor(max_workers=workers or min(16, os.cpu_count() or 1)) as ex:
            imgs = list(ex.map(decode, paths))
        ok = [i for i, im in enumerate(imgs)
              if im is not None and im.ndim == 3 and im.shape[2] == 3]
        ok_set = set(ok)
        results = [None] * len(paths)
        for i in range(len(paths)):
            if i not in ok_set:
                print(f"Image unreadable or wrong shape: {paths[i]}")
        if ok:
            hist = color_histograms([imgs[i] for i in ok], bins=bins)
            for j, i in enumerate(ok):
                results[i] = hist[j]
        return results

    def compute_vectors(self, paths: list[str], chunksize=16):
        from .decode_pipeline import ColorDecodePipeline
        if getattr(self, "_pipeline", None) is None:
            self._pipeline = ColorDecodePipeline(bins=self.bins)
        full = [p if Path(p).is_absolute() else self.base_dir / p for p in paths]
        res = self._pipeline.histograms(full)
        for p, v in zip(paths, res):
            if v is None:
                print(f"Image unreadable or wrong shape: {p}")
        return res

    def run(self):
        try:
            super().run()
        finally:
            if getattr(self, "_pipeline", None) is not None:
                self._pipeline.close()
                self._pipeline = None


if __name__ == "__main__":
    ColorVectorIndexer("images.db", Path().cwd(), log_file="color_indexer.log",
                       batch_size=16384).run()
