"""A/B of the bf16 candidate kernel's tile pool (IMGREC_B16W_POOL = P tiles per row split,
TileArgs::pool_p) on the bench's batch search (1024 queries, k = 10): per setting a fresh index
of the same device rows, then alternating rounds of `searches` back-to-back batch searches
(wall ms per search, the candidate kernel's event time) and a hash of the answers (must equal the
pool-off hash).  Prints one JSON line per (round, setting).
Usage: python tools/b16_pool_ab.py [config=3] [searches=20] [rounds=3] [settings=0,1,2,3] [rows]"""
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
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    settings = [int(v) for v in (sys.argv[4] if len(sys.argv) > 4 else "0,1,2,3").split(",")]
    cfg = dict(bench.CONFIGS[cid])
    if len(sys.argv) > 5:
        cfg["rows"] = int(sys.argv[5])
    dev = torch.device("cuda", 0)
    cen = bench.make_centres(torch, cfg, dev, cid)
    d = sum(cfg["parts"])
    q = bench.gen_queries(torch, cfg, cen, 1024, dev, cid)
    lib = _lib.load()
    idx = {}
    for pool in settings:
        os.environ["IMGREC_B16W_POOL"] = str(pool)
        sh = ShardedIndex(d, cfg["rows"], METRIC_L2, device=0)
        for blk in bench.gen_rows(torch, cfg, cen, 0, cfg["rows"], dev, cid):
            sh.add_local(blk)
        D, I = sh.search(q, 10)
        h = hashlib.sha256(D.cpu().numpy().tobytes() + I.cpu().numpy().tobytes()).hexdigest()[:16]
        idx[pool] = (sh, h, lib.knn_last_path(sh.index.handle))
    torch.cuda.synchronize()
    for r in range(rounds):
        for pool, (sh, hx, path) in idx.items():
            hd = sh.index.handle
            for _ in range(2):
                sh.search(q, 10)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(n):
                sh.search(q, 10)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) / n * 1e3
            lib.knn_set_timing(hd, 1)
            for _ in range(n):
                D, I = sh.search(q, 10)
            torch.cuda.synchronize()
            tot, nl = C.c_double(), C.c_int()
            _lib.check(lib.knn_kernel_time(hd, C.byref(tot), C.byref(nl)), "timing")
            lib.knn_set_timing(hd, 0)
            h2 = hashlib.sha256(D.cpu().numpy().tobytes() + I.cpu().numpy().tobytes()).hexdigest()[:16]
            print(json.dumps({"config": cid, "rows": cfg["rows"], "round": r, "pool": pool, "path": path,
                              "ms_per_search": wall, "kernel_ms": tot.value / max(nl.value, 1),
                              "hash": hx, "hash_again": h2}), flush=True)


if __name__ == "__main__":
    main()
