"""PCIe-inclusive search rate: host (numpy) queries in, host results out, through knn_search (the
faiss protocol the reference calls, main/search_from_image.py:247), on the bench corpus
(1M x 1968, generated on device).  Measurement tool; prints one JSON line per batch size."""
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

torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
cfg = dict(bench.CONFIGS[3])
rows = int(os.environ.get("ROWS", cfg["rows"]))
cent = bench.make_centres(torch, cfg, dev, 3)
shard = ShardedIndex(1968, rows, METRIC_L2, device=0)
for blk in bench.gen_rows(torch, cfg, cent, 0, rows, dev, 3):
    shard.add_local(blk)
torch.cuda.synchronize()
qd = bench.gen_queries(torch, cfg, cent, 1024, dev, 3)
qh = qd.cpu().numpy()
idx = shard.index
for nq in (1, 2, 1024):
    x = np.ascontiguousarray(qh[:nq])
    for _ in range(3):
        idx.search(x, 10)
    reps = 50 if nq == 1 else 20
    t0 = time.perf_counter()
    for _ in range(reps):
        D, I = idx.search(x, 10)
    el = (time.perf_counter() - t0) / reps
    Dd = torch.empty((nq, 10), dtype=torch.float32, device=dev)
    Id = torch.empty((nq, 10), dtype=torch.int64, device=dev)
    qq = qd[:nq].contiguous()
    st = torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        idx.search_device(qq.data_ptr(), nq, 10, Dd.data_ptr(), Id.data_ptr(), st)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        idx.search_device(qq.data_ptr(), nq, 10, Dd.data_ptr(), Id.data_ptr(), st)
    torch.cuda.synchronize()
    eld = (time.perf_counter() - t0) / reps
    same = bool((Id.cpu().numpy() == I).all())
    print(json.dumps({"nq": nq, "host_ms": el * 1e3, "host_qps": nq / el, "device_ms": eld * 1e3,
                      "device_qps": nq / eld, "pcie_overhead_ms": (el - eld) * 1e3,
                      "same_results": same}), flush=True)
