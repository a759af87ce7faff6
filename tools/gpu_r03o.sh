#!/bin/bash
# int8 small-batch path: per-search step at nq = 1..4 (AUTO forced to the int8 path with --mode i8)
# for two workgroups-per-CU plans, against the bf16 path at the same nq.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r03o}; mkdir -p $OUT
for w in 2 3; do for nq in 1 2 3 4; do
  echo "{\"wgpcu\": $w, \"nq\": $nq, \"mode\": \"i8\"}" >> $OUT/sweep.jsonl
  IMGREC_I8_WGPCU=$w timeout -k 10 120 python bench.py --nq $nq --mode i8 --profile-only --steps 300 --warmup 100 >> $OUT/sweep.jsonl 2>>$OUT/err.log || exit 1
done; done
for nq in 2 4 8; do
  echo "{\"nq\": $nq, \"mode\": \"bf16\"}" >> $OUT/sweep.jsonl
  timeout -k 10 120 python bench.py --nq $nq --mode bf16 --profile-only --steps 300 --warmup 100 >> $OUT/sweep.jsonl 2>>$OUT/err.log || exit 2
done
cat $OUT/sweep.jsonl
