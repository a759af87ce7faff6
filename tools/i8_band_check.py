#!/usr/bin/env python3
"""numpy check behind the int8 small-batch path (DESIGN.md "Small batches"): residual norm R of
the block-scaled int8 copy and the number of rows inside the certificate band per query, over the
whole 1M x 1968 bench corpus (bench.py generator on the CPU).  CPU only, ~3 min, ~20 GB RAM.
CFG=2 runs bench config 2 (1M x 768) instead; VARIANTS=blk64 limits the block sizes."""
import os
import numpy as np, torch, sys, time
sys.path.insert(0, '/root/repo')
import bench
torch.set_num_threads(8)
CFGN = int(os.environ.get("CFG", "3"))
cfg = bench.CONFIGS[CFGN]
dev = 'cpu'
cent = bench.make_centres(torch, cfg, dev, CFGN)
N = 1_000_000
xq = bench.gen_queries(torch, cfg, cent, 32, dev, CFGN).numpy().astype(np.float64)
D = xq.shape[1]
res = {}
variants = [v for v in [("blk64", 64), ("blk32", 32)]
            if v[0] in os.environ.get("VARIANTS", "blk64,blk32").split(",")]
EX = []; AP = {v: [] for v, _ in variants}; RR = {v: [] for v, _ in variants}
t0 = time.time()
for blk in bench.gen_rows(torch, cfg, cent, 0, N, dev, CFGN):
    xb = blk.numpy().astype(np.float64)
    n = xb.shape[0]
    EX.append((xq**2).sum(1)[:, None] + (xb**2).sum(1)[None] - 2 * xq @ xb.T)
    for name, B in variants:
        Dp = (D + B - 1)//B*B
        xp = np.zeros((n, Dp)); xp[:, :D] = xb
        b2 = xp.reshape(n, Dp//B, B)
        s = np.abs(b2).max(-1, keepdims=True) / 127.0
        s[s == 0] = 1
        deq = (np.rint(b2 / s).clip(-127, 127) * s).reshape(n, Dp)[:, :D]
        RR[name].append(np.linalg.norm(xb - deq, axis=1))
        AP[name].append((xq**2).sum(1)[:, None] + (xb**2).sum(1)[None] - 2 * xq @ deq.T)
print("gen+keys %.0f s" % (time.time()-t0))
ex = np.concatenate(EX, 1)
k = 10
for name, _ in variants:
    ap = np.concatenate(AP[name], 1); r = np.concatenate(RR[name])
    R = r.max()
    idx = np.argsort(ap, 1)[:, :k]
    T = np.take_along_axis(ap, idx[:, k-1:k], 1)[:, 0]
    bandG = (ap <= T[:, None] + 4 * R).sum(1)
    # per-row: a_i - 2 r_i <= T + 2 max r over the approx top-k
    Emax = 2 * r[idx].max(1)
    bandR = (ap - 2 * r[None] <= (T + Emax)[:, None]).sum(1)
    print(name, "R %.4f mean r %.4f | band global-R median %d p90 %d max %d | per-row median %d p90 %d max %d" % (
        R, r.mean(), np.median(bandG), np.percentile(bandG, 90), bandG.max(), np.median(bandR), np.percentile(bandR, 90), bandR.max()))
