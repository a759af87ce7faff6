"""A/B of index-creation knobs (IMGREC_* read when an index is created) on the bench's batch search:
per setting a fresh index of the same device rows, then alternating rounds of `searches`
back-to-back searches of `nq` queries (wall ms per search, candidate-kernel event ms) and a hash
of the answers (must agree across settings).  One JSON line per (round, setting).
Usage: python tools/env_ab.py <config> <rows|0> <nq> <searches> <rounds> "A=1 B=2" "A=0" ..."""
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
    cid, rows, nq, n, rounds = (int(v) for v in sys.argv[1:6])
    settings = sys.argv[6:] or [""]
    cfg = dict(bench.CONFIGS[cid])
    if rows:
        cfg["rows"] = rows
    dev = torch.device("cuda", 0)
    cen = bench.make_centres(torch, cfg, dev, cid)
    d = sum(cfg["parts"])
    q = bench.gen_queries(torch, cfg, cen, nq, dev, cid)
    lib = _lib.load()
    idx = {}
    for st in settings:
        kv = dict(x.split("=", 1) for x in st.split())
        old = {k: os.environ.get(k) for k in kv}
        os.environ.update(kv)
        sh = ShardedIndex(d, cfg["rows"], METRIC_L2, device=0)
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        for blk in bench.gen_rows(torch, cfg, cen, 0, cfg["rows"], dev, cid):
            sh.add_local(blk)
        D, I = sh.search(q, 10)
        idx[st] = (sh, hashlib.sha256(D.cpu().numpy().tobytes() + I.cpu().numpy().tobytes()).hexdigest()[:16])
    torch.cuda.synchronize()
    for r in range(rounds):
        for st, (sh, hx) in idx.items():
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
                sh.search(q, 10)
            torch.cuda.synchronize()
            tot, nl = C.c_double(), C.c_int()
            _lib.check(lib.knn_kernel_time(hd, C.byref(tot), C.byref(nl)), "timing")
            lib.knn_set_timing(hd, 0)
            print(json.dumps({"config": cid, "rows": cfg["rows"], "nq": nq, "round": r, "setting": st,
                              "ms_per_search": wall, "kernel_ms": tot.value / max(nl.value, 1),
                              "post_kernel_ms": wall - tot.value / max(nl.value, 1), "hash": hx}), flush=True)


if __name__ == "__main__":
    main()
