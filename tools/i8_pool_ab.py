"""A/B of the int8 scan's run-time group pool (IMGREC_I8_POOL / IMGREC_I8_POOL_CH, I8Args::pool)
on the reference CLI's one-query search: per setting a fresh index of the same device rows, then
alternating rounds of `searches` back-to-back one-query searches (wall ms per search, the scan
kernel's event time) and a hash of the answers of 64 queries (must equal the pool-off hash).
Prints one JSON line per (round, setting).
Usage: python tools/i8_pool_ab.py [config=3] [searches=200] [rounds=2] [settings=0:2,4:2,8:2,8:1,8:4,16:2]"""
import ctypes as C
import hashlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import bench
    from image_recommender_amd import _lib
    from image_recommender_amd.faiss_compat import METRIC_L2
    from image_recommender_amd.sharded import ShardedIndex
    cid = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    settings = [tuple(int(v) for v in s.split(":")) for s in
                (sys.argv[4] if len(sys.argv) > 4 else "0:2,4:2,8:2,8:1,8:4,16:2").split(",")]
    cfg = dict(bench.CONFIGS[cid])
    dev = torch.device("cuda", 0)
    cen = bench.make_centres(torch, cfg, dev, cid)
    d = sum(cfg["parts"])
    q = bench.gen_queries(torch, cfg, cen, 64, dev, cid)
    lib = _lib.load()
    idx = {}
    for pool, ch in settings:
        os.environ["IMGREC_I8_POOL"] = str(pool)
        os.environ["IMGREC_I8_POOL_CH"] = str(ch)
        sh = ShardedIndex(d, cfg["rows"], METRIC_L2, device=0)
        for blk in bench.gen_rows(torch, cfg, cen, 0, cfg["rows"], dev, cid):
            sh.add_local(blk)
        h = hashlib.sha256()
        for i in range(64):
            D, I = sh.search(q[i:i + 1].contiguous(), 10)
            h.update(D.cpu().numpy().tobytes())
            h.update(I.cpu().numpy().tobytes())
        idx[(pool, ch)] = (sh, h.hexdigest()[:16], lib.knn_last_path(sh.index.handle))
    torch.cuda.synchronize()
    for r in range(rounds):
        for key, (sh, hx, path) in idx.items():
            hd = sh.index.handle
            for i in range(8):
                sh.search(q[i:i + 1].contiguous(), 10)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(n):
                sh.search(q[i % 64:i % 64 + 1].contiguous(), 10)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) / n * 1e3
            lib.knn_set_timing(hd, 1)
            for i in range(n):
                sh.search(q[i % 64:i % 64 + 1].contiguous(), 10)
            torch.cuda.synchronize()
            tot, nl = C.c_double(), C.c_int()
            _lib.check(lib.knn_kernel_time(hd, C.byref(tot), C.byref(nl)), "timing")
            lib.knn_set_timing(hd, 0)
            print(json.dumps({"config": cid, "round": r, "pool64": key[0], "pool_ch": key[1],
                              "path": path, "ms_per_search": wall,
                              "scan_kernel_ms": tot.value / max(nl.value, 1), "hash": hx}), flush=True)


if __name__ == "__main__":
    main()
