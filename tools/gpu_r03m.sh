#!/bin/bash
# Candidate merge change: the whole GPU suite, then per-search steps on the int8 path (nq 1, 8)
# and the bf16 path (nq 1), with IMGREC_MERGE_K1 as given (default: k1 = 16).
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r03m}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for m in "1 i8" "8 i8" "1 bf16"; do
  set -- $m
  timeout -k 10 120 python bench.py --nq $1 --mode $2 --profile-only --steps 300 --warmup 100 > $OUT/nq$1_$2.json 2>>$OUT/err.log || exit 2
  echo "nq $1 $2 $(cat $OUT/nq$1_$2.json)"
done
CFG=2 timeout -k 10 300 python tools/i8_cfg2_probe.py > $OUT/probe_cfg2.jsonl 2>> $OUT/err.log || exit 3
cat $OUT/probe_cfg2.jsonl
