"""Diagnostic: where the int8 scan's fixed cost goes (a build with -DIMGREC_I8_STAMPS,
lib/libimgrec_i8stamps.so: tools/build_variants.sh i8stamps -DIMGREC_I8_STAMPS).  One-query
searches on bench config CFG (default 2); per scan workgroup s_memrealtime (100 MHz, one clock
for the chip) at 0 entry, 1 query side in LDS, 2 first group processed, 3-6 waves leave the row
loop, 7 lists written.  Prints per-query phase times in us (relative to the first entry) and the
medians over queries, one JSON line each."""
import ctypes as C
import json
import os
import sys

os.environ.setdefault("IMGREC_LIB_NAME", "libimgrec_i8stamps.so")
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
rows = int(os.environ.get("ROWS", cfg["rows"]))
cent = bench.make_centres(torch, cfg, dev, cid)
shard = ShardedIndex(sum(cfg["parts"]), rows, METRIC_L2, device=0)
for blk in bench.gen_rows(torch, cfg, cent, 0, rows, dev, cid):
    shard.add_local(blk)
q = bench.gen_queries(torch, cfg, cent, 16, dev, cid)
lib = _lib.load()
buf = (C.c_ulonglong * (1024 * 8))()
res = []
for i in range(16):
    qi = q[i:i + 1].contiguous()
    for _ in range(3):
        shard.search(qi, 10)                 # warm
    torch.cuda.synchronize()
    assert lib.knn_i8_stamps_clear() == 0
    shard.search(qi, 10)
    torch.cuda.synchronize()
    assert lib.knn_i8_stamps_read(buf) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 8).astype(np.int64)
    live = a[:, 0] > 0
    a = a[live]
    t0 = a[:, 0].min()
    us = (a - t0) / 100.0
    loop_end = us[:, 3:7].max(1)
    r = {"cfg": cid, "rows": rows, "workgroups": int(live.sum()),
         "entry_last": round(float(us[:, 0].max()), 2),
         "prep_median": round(float(np.median(us[:, 1] - us[:, 0])), 2),
         "prep_max_end": round(float(us[:, 1].max()), 2),
         "first_group_median": round(float(np.median(us[:, 2] - us[:, 1])), 2),
         "loop_end_min": round(float(loop_end.min()), 2),
         "loop_end_median": round(float(np.median(loop_end)), 2),
         "loop_end_max": round(float(loop_end.max()), 2),
         "wave_end_spread_median": round(float(np.median(us[:, 3:7].max(1) - us[:, 3:7].min(1))), 2),
         "fold_median": round(float(np.median(us[:, 7] - loop_end)), 2),
         "exit_last": round(float(us[:, 7].max()), 2)}
    wg = np.where(live)[0]
    r["loop_end_by_xcd"] = [round(float(np.median(loop_end[(wg % 8) == x])), 1) for x in range(8)]
    r["loop_end_by_half"] = [round(float(np.median(loop_end[(wg < len(wg) // 2) == h])), 1) for h in (True, False)]
    r["start_by_xcd"] = [round(float(np.median(us[(wg % 8) == x, 1])), 1) for x in range(8)]
    r["loop_end_pct"] = [round(float(np.percentile(loop_end, p)), 1) for p in (0, 5, 25, 50, 75, 95, 100)]
    if os.environ.get("DUMP"):               # per workgroup: id, query side ready, loop end (us)
        np.save(f"{os.environ['DUMP']}_q{i}.npy", np.stack([wg, us[:, 1], loop_end]))
    res.append(r)
    print(json.dumps(r), flush=True)
med = {k: float(np.median([r[k] for r in res])) for k in res[0]
       if k not in ("cfg", "rows", "workgroups") and not isinstance(res[0][k], list)}
print(json.dumps({"median_over_queries": med, "cfg": cid, "rows": rows}), flush=True)
