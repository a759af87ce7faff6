"""Large-k search rate (k > KNN_MAX_K: csrc/knn_largek.hip, exact fused kernel lists + certified
radix-select union + exact-scan fallback) on the
bench corpus (config 3, 1M x 1968), nq = 1 and 1024.  Measurement tool; one JSON line per case."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from image_recommender_amd.faiss_compat import METRIC_L2  # noqa: E402
from image_recommender_amd.sharded import ShardedIndex  # noqa: E402

cfg = dict(bench.CONFIGS[3])
dev = torch.device("cuda", 0)
D = int(sum(cfg["parts"]))
centres = bench.make_centres(torch, cfg, dev, 3)
shard = ShardedIndex(D, cfg["rows"], METRIC_L2, device=0)
for blk in bench.gen_rows(torch, cfg, centres, shard.row0, shard.row1, dev, 3):
    shard.add_local(blk)
for nq, k, reps in ((1, 100, 10), (1024, 100, 3), (1024, 1024, 2)):
    q = bench.gen_queries(torch, cfg, centres, nq, dev, 3)
    shard.search(q, k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        shard.search(q, k)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / reps * 1e3
    from image_recommender_amd import _lib
    import ctypes as C
    nf = C.c_int64()
    _lib.load().knn_large_k_fallbacks(shard.index.handle, C.byref(nf))
    print(json.dumps({"rows": cfg["rows"], "d": D, "nq": nq, "k": k, "ms": ms, "qps": nq / ms * 1e3, "fallbacks": nf.value,
                      "fp32_tflops": 2.0 * cfg["rows"] * D * nq / (ms * 1e-3) / 1e12}), flush=True)
