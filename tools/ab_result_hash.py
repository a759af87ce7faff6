"""Hash of one AUTO search's (D, I) on a bench workload, for A/B bit-identity of library variants
(run once per IMGREC_LIB_NAME; equal hashes = identical results).
Usage: IMGREC_LIB_NAME=libimgrec_x.so python tools/ab_result_hash.py [config] [nq]"""
import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import bench
    from image_recommender_amd import faiss_compat as faiss
    cid = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    nq = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    cfg = dict(bench.CONFIGS[cid])
    dev = torch.device("cuda", 0)
    cen = bench.make_centres(torch, cfg, dev, cid)
    d = sum(cfg["parts"])
    idx = faiss.IndexFlatL2(d)
    idx.reserve(cfg["rows"])
    st = torch.cuda.current_stream().cuda_stream
    for blk in bench.gen_rows(torch, cfg, cen, 0, cfg["rows"], dev, cid):
        idx.add_device(blk.data_ptr(), blk.shape[0], st)
    q = bench.gen_queries(torch, cfg, cen, nq, dev, cid)
    D = torch.empty((nq, 10), dtype=torch.float32, device=dev)
    I = torch.empty((nq, 10), dtype=torch.int64, device=dev)
    idx.search_device(q.data_ptr(), nq, 10, D.data_ptr(), I.data_ptr(), st)
    torch.cuda.synchronize()
    h = hashlib.sha256(D.cpu().numpy().tobytes() + I.cpu().numpy().tobytes()).hexdigest()
    print(f"{os.environ.get('IMGREC_LIB_NAME', 'libimgrec.so')} cfg{cid} nq={nq} {h} "
          f"stats={idx.certificate_stats()}")


if __name__ == "__main__":
    main()
