#!/usr/bin/env python3
"""Colour feature from image files: images/s of the decode pipeline
(vector_scripts/decode_pipeline.py) against the reference's CPU structure, on the same files.

  pipeline   worker processes decode (PIL) into a page-locked shared-memory ring; batches are
             DMA'd to the GPU and histogrammed (color_hist_fixed_kernel) while later files decode
  cpu        the reference's shape (/root/reference/vector_scripts/create_color_vector.py:18-78):
             a ProcessPoolExecutor of the same worker count, each worker decodes and histograms
             one image (numpy bincount = oracle/color_hist.py, cv2.calcHist being absent here)
  decode     the workers decoding only (no histogram anywhere): the decode ceiling

The files are written first (synthetic 256 x 256 JPEGs, q 92, like bench_pipeline's images).
Prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time
from concurrent.futures import ProcessPoolExecutor
import multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _cpu_one(p):
    from image_recommender_amd.vector_scripts.create_vector_base import load_image
    from oracle.color_hist import color_hist_reference
    img = load_image(p, normalize=False, as_array=True)
    return None if img is None else color_hist_reference(img, 16)


def _decode_only(p):
    from image_recommender_amd.vector_scripts.create_vector_base import load_image
    img = load_image(p, normalize=False, as_array=True)
    return 0 if img is None else img.shape[0]


def main():
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--images", type=int, default=8192)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--workers", type=int, default=16)
    ap.add_argument("--chunk", type=int, default=64)
    ap.add_argument("--fmt", default="jpg")
    a = ap.parse_args()
    tmp = tempfile.mkdtemp(prefix="imgrec_decode_")
    from image_recommender_amd.vector_scripts.decode_pipeline import (ColorDecodePipeline,
                                                                      write_synthetic_images)
    t0 = time.perf_counter()
    paths = [str(p) for p in write_synthetic_images(tmp, a.images, a.size, fmt=a.fmt,
                                                     workers=a.workers)]
    t_write = time.perf_counter() - t0
    ctx = mp.get_context("fork")
    # CPU-only measurements first (their pools fork before this process touches the GPU)
    with ProcessPoolExecutor(a.workers, mp_context=ctx) as ex:
        list(ex.map(_decode_only, paths[:256], chunksize=16))          # warm the page cache
        t0 = time.perf_counter()
        list(ex.map(_decode_only, paths, chunksize=16))
        t_dec = time.perf_counter() - t0
        t0 = time.perf_counter()
        ref = list(ex.map(_cpu_one, paths, chunksize=16))
        t_cpu = time.perf_counter() - t0
    import numpy as np
    import torch
    torch.cuda.init()
    with ColorDecodePipeline(workers=a.workers, chunk=a.chunk) as pipe:
        pipe.histograms(paths[:512])
        t0 = time.perf_counter()
        got = pipe.histograms(paths)
        t_pipe = time.perf_counter() - t0
    same = all(np.allclose(g, r, rtol=1e-6, atol=1e-7) for g, r in zip(got, ref))
    n = a.images
    print(json.dumps({
        "metric": "colour feature from image files, images/s (decode + 16-bin RGB histogram)",
        "images": n, "size": a.size, "format": a.fmt, "workers": a.workers, "chunk": a.chunk,
        "pipeline_images_per_s": n / t_pipe, "cpu_reference_shape_images_per_s": n / t_cpu,
        "decode_only_images_per_s": n / t_dec, "pipeline_vs_decode_ceiling": t_dec / t_pipe,
        "pipeline_vs_cpu": t_cpu / t_pipe, "results_equal_cpu": same, "write_s": t_write,
        "data": "synthetic gradient+noise images written as files by this tool",
        "cpu": "same host, same worker count; cv2 absent so the worker histogram is numpy "
               "bincount (oracle/color_hist.py)"}))
    import shutil
    shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
