#!/bin/bash
# Host-pointer search (the faiss call the reference makes) with page-locked staging for small
# batches: its tests, then the PCIe-inclusive rate at nq = 1, 2, 1024 against the device entry.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r03q}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_knn_gpu.py tests/test_i8_gpu.py tests/test_dropin_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python tools/host_search_rate.py > $OUT/host_search_rate.jsonl 2> $OUT/host.err || { tail $OUT/host.err; exit 2; }
cat $OUT/host_search_rate.jsonl
