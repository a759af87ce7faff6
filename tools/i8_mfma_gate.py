#!/usr/bin/env python3
"""Gate for an int8-MFMA candidate pass at large batches (DESIGN.md "int8
MFMA gate").  numpy over a 1M-row corpus of the bench's config-3 distribution (bench.py's
generators on the CPU: the same distribution as the GPU bench, not the same rows), 32 queries.

Variants of the candidate arithmetic, each with its certificate band = the rows whose approximate
key lies within 2 E_a of the k-th approximate key (the K' a first-pass certificate needs):
  bf16      today's path: bf16 rows, bf16 query (reference point)
  i8b64     int8 rows AND int8 query, one fp32 scale per 64-element block on both (one
            v_mfma_i32_16x16x64_i8 per 64-deep k-step, then an fp32 fold of the i32 block sums)
  i8b128    the same with 128-element blocks (one fold per two k-steps)
E_a per query (L2 keys, the certificate's Cauchy-Schwarz form): 2 (|q| R + dq (X + R)), R = max row
residual |x - x~|, dq = |q - q~|, X = max |x|.  CPU only, ~5 min, ~30 GB RAM.
"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, "/root/repo")
import bench  # noqa: E402

torch.set_num_threads(8)
N = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
NQ, K = 32, 10
cfg = bench.CONFIGS[3]
cent = bench.make_centres(torch, cfg, "cpu", 3)
xq = bench.gen_queries(torch, cfg, cent, NQ, "cpu", 3).numpy().astype(np.float64)
D = xq.shape[1]


def quant_blocks(x, B):
    """int8 codes with one scale per B-element block (symmetric, max|x_b| / 127) -> dequantised."""
    n = x.shape[0]
    Dp = (D + B - 1) // B * B
    xp = np.zeros((n, Dp))
    xp[:, :D] = x
    b = xp.reshape(n, Dp // B, B)
    s = np.abs(b).max(-1, keepdims=True) / 127.0
    s[s == 0] = 1
    return (np.rint(b / s).clip(-127, 127) * s).reshape(n, Dp)[:, :D]


def bf16(x):
    x32 = x.astype(np.float32)
    u = x32.view(np.uint32).astype(np.uint64)
    u = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16            # round to nearest even
    return u.astype(np.uint32).view(np.float32).astype(np.float64)


variants = {
    "bf16": lambda x: bf16(x),
    "i8b64": lambda x: quant_blocks(x, 64),
    "i8b128": lambda x: quant_blocks(x, 128),
}
qv = {v: f(xq) for v, f in variants.items()}
dq = {v: np.linalg.norm(xq - qv[v], axis=1) for v in variants}
qn = (xq ** 2).sum(1)
AP = {v: [] for v in variants}
R = {v: 0.0 for v in variants}
EX, X = [], 0.0
t0 = time.time()
for blk in bench.gen_rows(torch, cfg, cent, 0, N, "cpu", 3):
    xb = blk.numpy().astype(np.float64)
    xn = (xb ** 2).sum(1)
    X = max(X, float(np.sqrt(xn.max())))
    EX.append(qn[:, None] + xn[None] - 2 * xq @ xb.T)
    for v, f in variants.items():
        xv = f(xb)
        R[v] = max(R[v], float(np.linalg.norm(xb - xv, axis=1).max()))
        AP[v].append(qn[:, None] + xn[None] - 2 * qv[v] @ xv.T)
print(f"[gate] {N} rows generated and scored in {time.time() - t0:.0f} s")
ex = np.concatenate(EX, 1)
del EX
res = {}
for v in variants:
    ap = np.concatenate(AP[v], 1)
    AP[v] = None
    ak = np.sort(np.partition(ap, K, axis=1)[:, :K + 1], 1)[:, K - 1]
    Ea = 2 * (np.sqrt(qn) * R[v] + dq[v] * (X + R[v]))
    band = (ap <= (ak + 2 * Ea)[:, None]).sum(1)
    # does the true top-k sit inside the band (sanity of the bound)?
    top = np.argsort(ex, 1)[:, :K]
    inside = np.all(np.take_along_axis(ap, top, 1) <= (ak + 2 * Ea)[:, None])
    res[v] = dict(R=R[v], dq_median=float(np.median(dq[v])), Ea_median=float(np.median(Ea)),
                  band_median=float(np.median(band)), band_p90=float(np.percentile(band, 90)),
                  band_p99=float(np.percentile(band, 99)), band_max=int(band.max()),
                  exact_topk_in_band=bool(inside))
    print(f"[gate] {v:7s} R {R[v]:.4f}  dq {res[v]['dq_median']:.4f}  E_a {res[v]['Ea_median']:.4f}  "
          f"band median {res[v]['band_median']:.0f} p90 {res[v]['band_p90']:.0f} "
          f"p99 {res[v]['band_p99']:.0f} max {res[v]['band_max']}  top-k inside: {inside}")
import json  # noqa: E402
print(json.dumps({"rows": N, "queries": NQ, "k": K, "variants": res}))
