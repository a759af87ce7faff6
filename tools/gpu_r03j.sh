#!/bin/bash
# Group-interleaved row splits of the narrow (nq <= 32) bf16 tile: the GPU suite, then the nq = 1
# kernel against whole tile rounds (tools/gpu_r03i.sh) and at 1M rows.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r03j}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
bash tools/gpu_r03i.sh ${1:-r03j} || exit 2
for i in 1 2; do timeout -k 10 120 python bench.py --nq 1 --profile-only --steps 300 --warmup 100 >> $OUT/nq1.jsonl 2>>$OUT/nq1.err || exit 3; done
cat $OUT/nq1.jsonl
