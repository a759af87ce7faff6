"""Diagnostic: where a one-query second chance spends its time inside the certificate tail kernel
(a build with -DIMGREC_TAIL_STAMPS, lib/libimgrec_tailstamps.so: tools/build_variants.sh
tailstamps -DIMGREC_TAIL_STAMPS).  Config 2 (1M x 768), int8 path, single queries; for each query
whose first certificate failed, s_memrealtime (100 MHz, one clock for the whole chip) per tail
workgroup at: 0 entry, 1 first claim, 2 slice filtered, 3 slice reranked, 4 slice counted,
5 item merged + answered, 6 plan published / seen, 7 exit; and the rerank workgroup's waves at
0 entry, 1 level-1 lists loaded, 2 level-1 selected, 3 level-2 ranked, 4 exit, 5 query row loaded, 6 the
same lists loaded a second time (relative to wave 0's entry).  Prints per-query critical-path times in us and their medians."""
import ctypes as C
import json
import os
import sys

os.environ.setdefault("IMGREC_LIB_NAME", "libimgrec_tailstamps.so")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from image_recommender_amd import _lib  # noqa: E402
from image_recommender_amd.faiss_compat import METRIC_L2  # noqa: E402
from image_recommender_amd.sharded import ShardedIndex  # noqa: E402

cid = int(os.environ.get("CFG", "2"))
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
cfg = dict(bench.CONFIGS[cid])
cent = bench.make_centres(torch, cfg, dev, cid)
shard = ShardedIndex(sum(cfg["parts"]), cfg["rows"], METRIC_L2, device=0)
for blk in bench.gen_rows(torch, cfg, cent, 0, cfg["rows"], dev, cid):
    shard.add_local(blk)
q = bench.gen_queries(torch, cfg, cent, 32, dev, cid)
idx = shard.index
lib = _lib.load()
buf = (C.c_ulonglong * (1024 * 8))()
rbuf = (C.c_ulonglong * 64)()
rows = []
for i in range(32):
    qi = q[i:i + 1].contiguous()
    shard.search(qi, 10)                     # warm
    torch.cuda.synchronize()
    assert lib.knn_tail_stamps_clear() == 0
    shard.search(qi, 10)
    torch.cuda.synchronize()
    st = idx.certificate_stats()
    if st["second_chance"] == 0:
        continue
    assert lib.knn_tail_stamps_read(buf) == 0
    assert lib.knn_rerank_stamps_read(rbuf) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 8).astype(np.int64)
    rr = np.frombuffer(rbuf, dtype=np.uint64).reshape(8, 8).astype(np.int64)
    live = a[:, 0] > 0
    t0 = a[live, 0].min()
    us = lambda v: round(float(v - t0) / 100.0, 2)   # 100 MHz ticks -> us
    r0 = rr[0, 0]
    rerank = [[round(float(v - r0) / 100.0, 2) if v else None for v in rr[w, :7]] for w in range(8)]
    fin = np.where(a[:, 5] > 0)[0]
    if len(fin) != 1:
        continue
    f = int(fin[0])
    slices = a[a[:, 4] > 0]
    rec = {"query": i, "rerank_waves_us": rerank, "rerank_to_tail_us": round(float(t0 - r0) / 100.0, 2),
           "wgs": int(live.sum()), "entry_spread_us": us(a[live, 0].max()),
           "finisher": [us(v) if v else None for v in a[f]],
           "slice_claim_max_us": us(slices[:, 1].max()), "slice_filtered_max_us": us(slices[:, 2].max()),
           "slice_reranked_max_us": us(slices[:, 3][slices[:, 3] > 0].max()) if (slices[:, 3] > 0).any() else None,
           "slice_counted_max_us": us(slices[:, 4].max()),
           "waiters_seen_max_us": us(a[live & (a[:, 6] > 0), 6].max()),
           "exit_max_us": us(a[live & (a[:, 7] > 0), 7].max()) if (live & (a[:, 7] > 0)).any() else None}
    rows.append(rec)
    print(json.dumps(rec), flush=True)
if rows:
    fin = np.array([[v if v is not None else np.nan for v in r["finisher"]] for r in rows])
    print(json.dumps({"median_finisher_us": [round(float(x), 2) for x in np.nanmedian(fin, axis=0)],
                      "median_entry_spread_us": float(np.median([r["entry_spread_us"] for r in rows])),
                      "median_exit_max_us": float(np.median([r["exit_max_us"] for r in rows if r["exit_max_us"]])),
                      "n": len(rows)}), flush=True)
