"""Where the int8 single-query search spends its time on config 2 (1M x 768 L2): certificate
counts and per-search time for the int8 and bf16 paths over 32 queries (measurement tool).
FENCE=lazy: the index's lazy fence (Index.set_fence_mode; no event record per search)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from image_recommender_amd.faiss_compat import METRIC_L2  # noqa: E402
from image_recommender_amd.sharded import ShardedIndex  # noqa: E402

cid = int(os.environ.get("CFG", "2"))
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
cfg = dict(bench.CONFIGS[cid])
cent = bench.make_centres(torch, cfg, dev, cid)
d = sum(cfg["parts"])
shard = ShardedIndex(d, cfg["rows"], METRIC_L2, device=0)
for blk in bench.gen_rows(torch, cfg, cent, 0, cfg["rows"], dev, cid):
    shard.add_local(blk)
q = bench.gen_queries(torch, cfg, cent, 32, dev, cid)
idx = shard.index
fence = os.environ.get("FENCE", "eager")
if fence == "lazy":
    idx.set_fence_mode(True)
for mode in ("i8", "bf16"):
    idx.search_mode = mode
    tot = {"second_chance": 0, "exact_reruns": 0}
    ts = []
    for i in range(32):
        qi = q[i:i + 1].contiguous()
        for rep in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            shard.search(qi, 10)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
        ts.append(dt)
        st = idx.certificate_stats()
        tot["second_chance"] += st["second_chance"]
        tot["exact_reruns"] += st["exact_reruns"]
    ts.sort()
    print(json.dumps({"config": cid, "mode": mode, "fence": fence, "median_ms": ts[16] * 1e3, "max_ms": ts[-1] * 1e3,
                      "min_ms": ts[0] * 1e3, **tot}), flush=True)
