#!/bin/bash
# A/B: non-temporal corpus DMA in one-query-block launches (default lib) vs without (nont)
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/ab_nt; mkdir -p $OUT
timeout -k 10 300 python -m pytest tests/test_bf16_gpu.py tests/test_knn_gpu.py -x -q > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
  for v in libimgrec.so libimgrec_nont.so; do
    IMGREC_LIB_NAME=$v timeout -k 10 200 python tools/small_batch.py bf16,exact 1,8,32 > $OUT/${v}_$rep.jsonl 2> $OUT/${v}_$rep.err || { tail -20 $OUT/${v}_$rep.err; exit 2; }
    echo "== $v rep $rep"; cat $OUT/${v}_$rep.jsonl
  done
done
