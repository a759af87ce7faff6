"""Latency of small query batches (nq = 1 .. 256) on the bench corpus, per search mode.

Debug/measurement tool: prints one JSON line per (mode, nq) with the mean wall time per search
(device queries, results on device) and the fused-kernel time from the library's HIP events.
"""
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from image_recommender_amd import _lib  # noqa: E402
from image_recommender_amd.faiss_compat import METRIC_L2  # noqa: E402
from image_recommender_amd.sharded import ShardedIndex  # noqa: E402

torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
cfg = dict(bench.CONFIGS[3])
rows = int(os.environ.get("ROWS", cfg["rows"]))
cent = bench.make_centres(torch, cfg, dev, 3)
shard = ShardedIndex(1968, rows, METRIC_L2, device=0)
for blk in bench.gen_rows(torch, cfg, cent, 0, rows, dev, 3):
    shard.add_local(blk)
torch.cuda.synchronize()
lib = _lib.load()
q = bench.gen_queries(torch, cfg, cent, 256, dev, 3)
modes = sys.argv[1].split(",") if len(sys.argv) > 1 else ["exact", "bf16"]
sizes = [int(x) for x in (sys.argv[2].split(",") if len(sys.argv) > 2 else "1,8,32,128,256".split(","))]
for mode in modes:
    shard.index.search_mode = mode
    for nq in sizes:
        qq = q[:nq].contiguous()
        for _ in range(3):
            shard.search(qq, 10)
        torch.cuda.synchronize()
        lib.knn_set_timing(shard.index.handle, 1)
        reps = 30
        t0 = time.perf_counter()
        for _ in range(reps):
            D, I = shard.search(qq, 10)
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / reps
        tot, nl = C.c_double(), C.c_int()
        lib.knn_kernel_time(shard.index.handle, C.byref(tot), C.byref(nl))
        lib.knn_set_timing(shard.index.handle, 0)
        st = shard.index.search_stats()
        print(json.dumps({"mode": mode, "nq": nq, "ms": el * 1e3, "kernel_ms": tot.value / max(nl.value, 1),
                          "qps": nq / el, "path": lib.knn_last_path(shard.index.handle),
                          "cand_queries": st[0], "fallbacks": st[1]}), flush=True)
