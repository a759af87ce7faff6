"""IVF-PQ at the reference's default index configuration.

faiss.IndexIVFPQ(IndexHNSWFlat(d, 32), d, nlist=2048, m=48, nbits=12), nprobe = 1
(/root/reference/main/create_index.py:207-234 with find_valid_m(1968) = 48), on the bench corpus
(config 3: 1M x 1968, bench.py's generator).  Prints one JSON line: training / add seconds, search
queries/s at nq = 1024 and nq = 1 (device queries, results copied to the host as the shim
returns them), recall@10 of 128 queries against the exact index, and the table + scan kernel
times from rocprof-free HIP events.  Measurement tool, not the bench.py contract.
Usage: python tools/bench_ivfpq.py [rows] [nprobe]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from image_recommender_amd.faiss_compat import IndexFlatL2  # noqa: E402
from image_recommender_amd.ivfpq import IndexIVFPQ  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
nprobe = int(sys.argv[2]) if len(sys.argv) > 2 else 1
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
cfg = dict(bench.CONFIGS[3])
cent = bench.make_centres(torch, cfg, dev, 3)
xb = torch.cat(list(bench.gen_rows(torch, cfg, cent, 0, rows, dev, 3)))
q = bench.gen_queries(torch, cfg, cent, 1024, dev, 3)
d = xb.shape[1]

t0 = time.perf_counter()
idx = IndexIVFPQ(d, 2048, 48, 12)
idx.train(xb)
torch.cuda.synchronize()
t_train = time.perf_counter() - t0
t0 = time.perf_counter()
idx.add(xb)
torch.cuda.synchronize()
t_add = time.perf_counter() - t0
idx.nprobe = nprobe

idx.search(q, 10)
t0 = time.perf_counter()
reps = 5
for _ in range(reps):
    D, I = idx.search(q, 10)
qps = 1024 * reps / (time.perf_counter() - t0)
q1 = q[:1]
idx.search(q1, 10)
t0 = time.perf_counter()
for _ in range(20):
    idx.search(q1, 10)
lat1 = (time.perf_counter() - t0) / 20

ex = IndexFlatL2(d, device=0)
ex.search_mode = "exact"
xc = xb.contiguous()
ex.add_device(xc.data_ptr(), rows, torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
Dg = torch.empty((128, 10), dtype=torch.float32, device=dev)
Ig = torch.empty((128, 10), dtype=torch.int64, device=dev)
q128 = q[:128].contiguous()
ex.search_device(q128.data_ptr(), 128, 10, Dg.data_ptr(), Ig.data_ptr(), 0)
torch.cuda.synchronize()
gt = Ig.cpu().numpy()
recall = float(np.mean([len(set(a.tolist()) & set(b.tolist())) / 10 for a, b in zip(I[:128], gt)]))
lists = torch.bincount(idx._lists, minlength=idx.nlist).cpu().numpy()
print(json.dumps({
    "workload": f"IVF-PQ nlist 2048, m 48, nbits 12, nprobe {nprobe} on {rows} x {d} (bench cfg3 data)",
    "train_s": t_train, "add_s": t_add, "queries_per_s_nq1024": qps, "ms_per_query_nq1": lat1 * 1e3,
    "recall_at_10_vs_exact": recall, "codes_bytes": int(idx._codes.numel() * 2),
    "fp32_corpus_bytes": rows * d * 4, "list_rows_mean": float(lists.mean()), "list_rows_max": int(lists.max()),
}))
