#!/bin/bash
# nq = 1 kernel: balanced vs unbalanced tile counts per row split (512 splits of 256-row tiles):
# 1,000,000 rows = 3907 tiles (7.63 per split), 1,048,576 = 8 per split, 917,504 = 7 per split.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r03g}; mkdir -p $OUT
for r in 1000000 1048576 917504 1000000; do
  timeout -k 10 120 python bench.py --rows $r --nq 1 --profile-only --steps 300 --warmup 100 >> $OUT/nq1_rows.jsonl 2>>$OUT/nq1_rows.err || exit 1
done
cat $OUT/nq1_rows.jsonl
