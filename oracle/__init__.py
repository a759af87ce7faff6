"""TEST INFRASTRUCTURE ONLY — CPU restatements of the reference hot path, used as the checker.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this package.  The product (``image_recommender_amd``) never imports it and has no CPU fallback.

Contents
  flat_knn.py     exact flat k-NN (faiss IndexFlatL2 / IndexFlatIP semantics) in float64, the fp32
                  BLAS form of faiss's exhaustive_L2sqr_blas (CPU baseline), the fp32 error bound
                  used by the parity tests.
  plumbing.py     the reference's index/search plumbing: canonical type order, find_valid_m,
                  query assembly (concat -> mean -> normalize_L2), offset bookkeeping.
  color_hist.py   cv2.calcHist-equivalent RGB histogram + L2 normalisation (numpy bincount).
  ivfpq.py        faiss IndexIVFPQ's by-residual ADC search (the opt-in IVF-PQ index).
  c/              plain-C restatements (flat L2/IP search in double, colour histogram counts)
                  built by oracle/c/Makefile into oracle/_build/liboracle.so (git-ignored);
                  tests/test_oracle_c_cpu.py holds them against flat_knn.py / color_hist.py, and
                  the full-size cfg2 GPU test uses the C search as its second, independent checker.

Parity status: the arithmetic of the path lives in faiss-cpu 1.10.0 and
opencv-python 4.11.0.86, neither installed nor vendored, so it is "parity unpinned" against the
libraries themselves.  The plumbing restatement is pinned against fixtures captured by running the
reference's own modules (main/create_index.py, main/search_from_image.py) under import stubs in the
build container (tests/golden/make_golden.py); the arithmetic is pinned by float64 ground truth.
"""
