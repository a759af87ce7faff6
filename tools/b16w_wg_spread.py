"""Diagnostic: when each workgroup of the bf16 candidate kernel starts and ends its tiles
(a build with -DIMGREC_B16_STAMPS, lib/libimgrec_stamps.so: s_memrealtime per workgroup at entry
and after its last tile).  For several searches at the bench's config: the spread of the end
times (us after the first start), by XCD (blockIdx % 8), by query block and by row split — how
much of the kernel is the slowest workgroup's tail.
Usage: python tools/b16w_wg_spread.py [config=3] [searches=5]"""
import ctypes as C
import json
import os
import sys

os.environ.setdefault("IMGREC_LIB_NAME", "libimgrec_stamps.so")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    import bench
    from image_recommender_amd import _lib
    from image_recommender_amd.faiss_compat import METRIC_L2
    from image_recommender_amd.sharded import ShardedIndex
    cid = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    cfg = dict(bench.CONFIGS[cid])
    if os.environ.get("IMGREC_STAMPS_ROWS"):
        cfg["rows"] = int(os.environ["IMGREC_STAMPS_ROWS"])
    dev = torch.device("cuda", 0)
    D = int(sum(cfg["parts"]))
    cen = bench.make_centres(torch, cfg, dev, cid)
    q = bench.gen_queries(torch, cfg, cen, 1024, dev, cid)
    sh = ShardedIndex(D, cfg["rows"], METRIC_L2, device=0)
    for blk in bench.gen_rows(torch, cfg, cen, sh.row0, sh.row1, dev, cid):
        sh.add_local(blk)
    sh.index.search_mode = "bf16"
    lib = _lib.load()
    tr, tq, sp, wg = C.c_int(), C.c_int(), C.c_int(), C.c_int()
    lib.knn_plan(sh.index.handle, 1024, 10, C.byref(tr), C.byref(tq), C.byref(sp), C.byref(wg))
    nwg, nsplit = wg.value, sp.value
    for _ in range(3):
        sh.search(q, 10)
    torch.cuda.synchronize()
    buf = (C.c_ulonglong * 2048)()
    for it in range(n):
        sh.search(q, 10)
        torch.cuda.synchronize()
        assert lib.knn_b16w_wg_read(buf) == 0
        a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 2)[:nwg].astype(np.int64)
        t0 = a[:, 0].min()
        start = (a[:, 0] - t0) / 100.0                 # us (100 MHz)
        end = (a[:, 1] - t0) / 100.0
        b = np.arange(nwg)
        # the kernel's bijective XCD-aware map (knn_b16w.hip): wgid from blockIdx
        xcd, qq, rr = b & 7, nwg >> 3, nwg & 7
        wgid = np.where(xcd < rr, xcd * (qq + 1), rr * (qq + 1) + (xcd - rr) * qq) + (b >> 3)
        G = 4 if (nwg // nsplit) % 4 == 0 else nwg // nsplit
        qbg, rem = wgid // (nsplit * G), wgid % (nsplit * G)
        qb = qbg * G + rem % G
        rec = {"config": cid, "rows": cfg["rows"], "search": it, "workgroups": nwg,
               "start_max_us": round(float(start.max()), 2),
               "end_min_us": round(float(end.min()), 2), "end_median_us": round(float(np.median(end)), 2),
               "end_p90_us": round(float(np.percentile(end, 90)), 2), "end_max_us": round(float(end.max()), 2),
               "tail_us": round(float(end.max() - np.median(end)), 2),
               "end_by_xcd": [round(float(np.median(end[xcd == x])), 1) for x in range(8)],
               "end_max_by_xcd": [round(float(end[xcd == x].max()), 1) for x in range(8)],
               "end_by_qblock": [round(float(np.median(end[qb == x])), 1) for x in range(int(qb.max()) + 1)],
               "slowest_10": [int(v) for v in np.argsort(-end)[:10]]}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
