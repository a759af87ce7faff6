#!/bin/bash
# epilogue breakdown of the bf16 256x256 kernel (IMGREC_B16_PROF build) at three corpus sizes
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/b16prof; mkdir -p $OUT
for r in 125000 1000000 4000000; do
  timeout -k 10 300 python tools/prof_b16.py $r > $OUT/rows_$r.txt 2>&1 || { tail -20 $OUT/rows_$r.txt; exit 1; }
  echo "== rows $r"; grep -v "^\[" $OUT/rows_$r.txt | tail -9
done
