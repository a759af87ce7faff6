#!/usr/bin/env python3
"""One-query search time across many distinct queries (bench.py's single_query leg times only the
first query of the batch): the bench workload's index (CFG, default 2), then for each of the first
NQ_SWEEP queries (default 64) REPS back-to-back searches of that one query (bench.py's region:
synchronize on both sides), with the certificate counts of its search (second chance, exact
re-run).  Also the batch's (1024 queries) second-chance and re-run counts.  Measurement tool: one
JSON line per query, then a summary line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from image_recommender_amd.faiss_compat import METRIC_L2  # noqa: E402
from image_recommender_amd.sharded import ShardedIndex  # noqa: E402

cfg_id = int(os.environ.get("CFG", 2))
nsweep = int(os.environ.get("NQ_SWEEP", 64))
reps = int(os.environ.get("REPS", 40))
k = 10
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
cfg = dict(bench.CONFIGS[cfg_id])
D_total = int(sum(cfg["parts"]))
centres = bench.make_centres(torch, cfg, dev, cfg_id)
q = bench.gen_queries(torch, cfg, centres, 1024, dev, cfg_id)
shard = ShardedIndex(D_total, cfg["rows"], METRIC_L2, device=0, query_groups=1)
for blk in bench.gen_rows(torch, cfg, centres, shard.row0, shard.row1, dev, cfg_id):
    shard.add_local(blk)
shard.index.search_mode = os.environ.get("MODE", "auto")
shard.index.set_fence_mode(lazy=True)
for _ in range(3):
    shard.search(q, k)
torch.cuda.synchronize()
st = shard.index.certificate_stats()
print(json.dumps({"cfg": cfg_id, "batch": 1024, **st}), flush=True)

rows = []
for i in range(nsweep):
    q1 = q[i:i + 1].contiguous()
    for _ in range(3):
        shard.search(q1, k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        shard.search(q1, k)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / reps * 1e3
    st = shard.index.certificate_stats()
    rec = {"q": i, "ms": ms, "second_chance": st["second_chance"], "exact_reruns": st["exact_reruns"]}
    rows.append(rec)
    print(json.dumps(rec), flush=True)
ms = np.array([r["ms"] for r in rows])
sc = np.array([r["second_chance"] > 0 or r["exact_reruns"] > 0 for r in rows])
print(json.dumps({"cfg": cfg_id, "queries": nsweep, "mean_ms": float(ms.mean()),
                  "median_ms": float(np.median(ms)), "frac_second_chance": float(sc.mean()),
                  "mean_ms_certified": float(ms[~sc].mean()) if (~sc).any() else None,
                  "mean_ms_second_chance": float(ms[sc].mean()) if sc.any() else None}), flush=True)
