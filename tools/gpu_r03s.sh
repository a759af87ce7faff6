#!/bin/bash
# config 2 (1M x 768 L2) single-query and batch steps, int8 vs bf16 at nq = 1.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r03s}; mkdir -p $OUT
for args in "--nq 1" "--nq 1 --mode bf16" "--nq 2" "--nq 1024"; do
  echo "{\"config\": 2, \"args\": \"$args\"}" >> $OUT/cfg2.jsonl
  timeout -k 10 200 python bench.py --config 2 $args --profile-only --steps 200 --warmup 50 >> $OUT/cfg2.jsonl 2>> $OUT/err.log || { tail $OUT/err.log; exit 1; }
done
cat $OUT/cfg2.jsonl
