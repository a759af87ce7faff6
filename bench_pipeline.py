#!/usr/bin/env python3
"""the ingest + search pipeline, images/s per stage.

N synthetic RGB uint8 images (256 x 256: smooth gradients + noise, generated on device from
seed 5 in blocks of 1024 so every sharding sees the same images) go through the stages the
reference runs per image:

  colour    HIP histogram kernel (csrc/color_hist.hip; reference vector_scripts/
            create_color_vector.py:18-52: 16 bins per RGB channel, L2-normalised, 48-d)
  dreamsim  resize 256 -> 224 (bicubic, antialiased: the reference resizes with PIL LANCZOS on
            the CPU) + the DreamSim-architecture ensemble (3 ViT-B/16, 1792-d) on PyTorch-ROCm:
            bf16 GEMMs from weights cast once, fp32 LayerNorm / residual stream, the fused HIP
            passes of include/imgrec_vit.h; RANDOM weights (the pretrained weights cannot be
            downloaded here: throughput only)
  index     concatenate [colour 48 | dreamsim 1792] = 1840-d rows (the SIFT part needs the
            reference's trained VLAD codebook, which is not in the repo) and add them to the
            resident exact index (HBM copy, norms, bf16 copy)
  search    1024 queries (normalised concatenations of the first 1024 images, as
            main/search_from_image.py:305-322 builds them), k = 10

`--gpus N` (torchrun): each rank runs the stages on its contiguous share of the images
(weak in the number of images per rank, no collective until search), the index is row-sharded
and the search merges per-shard results over RCCL.  Prints one JSON line on rank 0; `value` =
end-to-end images/s (colour + dreamsim + index stages, max over ranks), per-stage rates inside.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

IMG = 256
BLOCK = 1024


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--images", type=int, default=100_000, help="total images (all ranks)")
    ap.add_argument("--model-batch", type=int, default=512)
    ap.add_argument("--nq", type=int, default=1024)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--search-reps", type=int, default=10)
    return ap.parse_args(argv)


def gen_images(torch, b0: int, n: int, device):
    """Images b0 .. b0+n-1 (global ids), (n, 256, 256, 3) uint8, block-seeded."""
    out = torch.empty((n, IMG, IMG, 3), dtype=torch.uint8, device=device)
    yy = torch.linspace(0, 1, IMG, device=device).view(1, IMG, 1, 1)
    xx = torch.linspace(0, 1, IMG, device=device).view(1, 1, IMG, 1)
    i = b0
    while i < b0 + n:
        blk = i // BLOCK
        j0, j1 = i - blk * BLOCK, min(BLOCK, b0 + n - blk * BLOCK)
        g = torch.Generator(device=device)
        g.manual_seed(5 * 1_000_003 + blk)
        a = torch.rand((BLOCK, 1, 1, 3), generator=g, device=device)
        b = torch.rand((BLOCK, 1, 1, 3), generator=g, device=device)
        c = torch.rand((BLOCK, 1, 1, 3), generator=g, device=device)
        sl = slice(j0, j1)
        noise = torch.randn((j1 - j0, IMG, IMG, 3), generator=g, device=device) * 0.08
        img = (a[sl] * yy + b[sl] * xx) * 0.7 + 0.3 * c[sl] + noise
        out[i - b0:i - b0 + (j1 - j0)] = (img.clamp(0, 1) * 255).to(torch.uint8)
        i += j1 - j0
    return out


def run(a) -> dict | None:
    """The pipeline on this rank; returns the report on rank 0 (None elsewhere)."""
    import torch
    import torch.distributed as dist
    import torch.nn.functional as F

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # IMGREC_DIST_BACKEND=gloo rehearses the N-rank protocol with every rank on one visible GPU
    # (as bench.py); the measured runs use RCCL ("nccl"), one rank per GPU
    backend = os.environ.get("IMGREC_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if world > 1 and backend == "nccl" and (ndev < world or local >= ndev):
        raise SystemExit(f"[bench_pipeline] rank {rank}: WORLD_SIZE={world} ranks need {world} "
                         f"visible GPUs, this process sees {ndev}")
    if backend != "nccl":
        local = local % max(ndev, 1)
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        from datetime import timedelta
        tmo = timedelta(seconds=float(os.environ.get("IMGREC_DIST_TIMEOUT_S", "300")))
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device, timeout=tmo)
        else:
            dist.init_process_group(backend, timeout=tmo)
        dist.barrier()

    from image_recommender_amd.faiss_compat import METRIC_L2
    from image_recommender_amd.sharded import ShardedIndex, shard_range
    from image_recommender_amd.vector_scripts.create_color_vector import color_histograms_device
    from image_recommender_amd.vector_scripts.create_dreamsim_vector import DreamSimVectorIndexer

    r0, r1 = shard_range(a.images, rank, world)
    n = r1 - r0
    imgs = gen_images(torch, r0, n, device)                  # the data source, not timed
    torch.cuda.synchronize()

    class _Embedder(DreamSimVectorIndexer):                   # model only: no DB, no logs
        def __init__(self):
            self.device = device
            self._log_and_print = lambda *x, **y: None
            self._setup_model(None, allow_random_init=True)

    emb = _Embedder()
    d = 48 + emb.dim
    index = ShardedIndex(d, a.images, METRIC_L2, device=local)

    def colour(x):                                            # (b,256,256,3) u8 -> (b,48)
        b = x.shape[0]
        npix = torch.full((b,), IMG * IMG, dtype=torch.int64, device=device)
        offs = torch.arange(b, dtype=torch.int64, device=device) * (IMG * IMG * 3)
        return color_histograms_device(x.reshape(-1), offs, npix, 16)

    def dreamsim(x):                                          # (b,256,256,3) u8 -> (b,1792)
        t = x.permute(0, 3, 1, 2).float().div_(255.0)
        t = F.interpolate(t, size=(224, 224), mode="bicubic", antialias=True).clamp_(0, 1)
        return emb.embed_tensor(t.contiguous())

    # warm-up (kernels, autotuning, allocator) on the first batch, outside the timings
    wb = imgs[: min(a.model_batch, n)]
    colour(wb)
    dreamsim(wb)
    torch.cuda.synchronize()

    def timed(fn):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        return out, time.perf_counter() - t0

    # one launch over all of this rank's images (per-call tensor set-up on 4096-image chunks cost
    # 40 % of the stage in round 1: 2.73 vs 4.5 TB/s)
    col, t_col = timed(lambda: colour(imgs))
    dsv, t_ds = timed(lambda: torch.cat([dreamsim(imgs[i:i + a.model_batch])
                                          for i in range(0, n, a.model_batch)]))

    def add():
        rows = torch.cat([col, dsv], 1).contiguous()
        index.add_local(rows)
        return rows
    rows, t_add = timed(add)

    # queries: images 0..nq-1 on every rank (regenerated, outside the timings)
    qi = gen_images(torch, 0, a.nq, device)
    qv = torch.cat([colour(qi), dreamsim(qi)], 1)
    qv = qv / qv.norm(dim=1, keepdim=True).clamp_min(1e-30)
    index.search(qv, a.k)
    (Dq, Iq), t_s = timed(lambda: [index.search(qv, a.k) for _ in range(a.search_reps)][-1])

    times = torch.tensor([t_col, t_ds, t_add, t_s], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(times, op=dist.ReduceOp.MAX)
    t_col, t_ds, t_add, t_s = (float(v) for v in times)
    self_hit = float((Iq[:, 0].cpu() == torch.arange(a.nq)).float().mean())
    out = None
    if rank == 0:
        tot = a.images
        out = {
            "metric": "config-5 pipeline images/s (colour hist + DreamSim-arch forward + index add)",
            "value": tot / (t_col + t_ds + t_add),
            "unit": "images/s",
            "n_gpus": world,
            "higher_is_better": True,
            "scaling": "weak" if world > 1 else "n/a",
            "data": "synthetic 256x256 RGB uint8 (gradients + noise, seed 5), generated on device; "
                    "DreamSim weights random (architecture-equivalent, throughput only)",
            "config": {"images": tot, "images_per_gpu": n, "model_batch": a.model_batch,
                       "dim": d, "parts": "color48|dreamsim1792 (no SIFT codebook)",
                       "nq": a.nq, "k": a.k},
            "stages": {
                "colour_hist": {"images_per_s": tot / t_col, "s": t_col,
                                "hbm_gbs_per_gpu": n * IMG * IMG * 3 / t_col / 1e9},
                "dreamsim": {"images_per_s": tot / t_ds, "s": t_ds,
                             "tflops_per_gpu": n / t_ds * 105.5e9 / 1e12,
                             "bf16_mfma_frac": n / t_ds * 105.5e9 / 2516.8e12,
                             "dtype": "bf16 matrix products (weights cast once), fp32 LayerNorm "
                                      "and residual stream, fp32 normalise"},
                "index_add": {"rows_per_s": tot / t_add, "s": t_add},
                "search": {"queries_per_s": a.nq * a.search_reps / t_s,
                           "ms_per_batch": t_s / a.search_reps * 1e3,
                           "self_match_at_rank0": self_hit},
            },
        }
    if world > 1:
        dist.destroy_process_group()
    return out


def main():
    a = parse()
    # --gpus N > 1 without torchrun: start the N ranks here or stop with a non-zero status
    from image_recommender_amd.launch import maybe_spawn
    maybe_spawn(a.gpus, os.path.abspath(__file__), sys.argv[1:])
    out = run(a)
    if out is not None:
        print(json.dumps(out))


if __name__ == "__main__":
    main()
