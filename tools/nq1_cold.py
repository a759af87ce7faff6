"""One-query search kernel time warm (back to back) and cold three ways — after a 512 MiB read,
after a 512 MiB copy (dirty lines draining under the scan), alternating with a second resident
index of the same rows (another full scan through the MALL in between) — for the library
IMGREC_LIB_NAME names.  Prints one JSON line.
Usage: python tools/nq1_cold.py [config=3] [searches=64]"""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import bench
    from image_recommender_amd import _lib
    from image_recommender_amd.faiss_compat import METRIC_L2
    from image_recommender_amd.sharded import ShardedIndex
    cid = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    cfg = dict(bench.CONFIGS[cid])
    dev = torch.device("cuda", 0)
    cen = bench.make_centres(torch, cfg, dev, cid)
    d = sum(cfg["parts"])
    sh = ShardedIndex(d, cfg["rows"], METRIC_L2, device=0)
    for blk in bench.gen_rows(torch, cfg, cen, 0, cfg["rows"], dev, cid):
        sh.add_local(blk)
    q = bench.gen_queries(torch, cfg, cen, 64, dev, cid)
    other = ShardedIndex(d, cfg["rows"], METRIC_L2, device=0)       # a second copy of the rows
    for blk in bench.gen_rows(torch, cfg, cen, 0, cfg["rows"], dev, cid):
        other.add_local(blk)
    lib, h = _lib.load(), sh.index.handle
    flush_buf = torch.ones(128 << 20, dtype=torch.int32, device=dev)
    flush_dst = torch.empty_like(flush_buf)
    out = torch.empty((), dtype=torch.int64, device=dev)
    for i in range(4):
        sh.search(q[i:i + 1].contiguous(), 10)
        other.search(q[i:i + 1].contiguous(), 10)
    res = {"lib": os.environ.get("IMGREC_LIB_NAME", "libimgrec.so"), "config": cid}
    for mode in ("warm", "read512", "copy512", "alternate"):
        lib.knn_set_timing(h, 1)
        for i in range(n):
            qi = q[i % 64:i % 64 + 1].contiguous()
            if mode == "read512":
                torch.sum(flush_buf, dim=0, dtype=torch.int64, out=out)
            elif mode == "copy512":
                flush_dst.copy_(flush_buf)
            elif mode == "alternate":
                other.search(qi, 10)
            sh.search(qi, 10)
        torch.cuda.synchronize()
        tot, nl = C.c_double(), C.c_int()
        _lib.check(lib.knn_kernel_time(h, C.byref(tot), C.byref(nl)), "timing")
        lib.knn_set_timing(h, 0)
        res[f"kernel_ms_{mode}"] = tot.value / max(nl.value, 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
