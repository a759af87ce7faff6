#!/bin/bash
# Remainder-balanced narrow bf16 tile: the GPU suite, then nq = 1 kernel time at whole-round and
# 1M corpora with two workgroups per CU (2-slot ring) and one (4-slot ring).
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r03k}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for w in 2 1; do for r in 131072 524288 1048576 1000000 1000000; do
  IMGREC_B16_NARROW_WGPCU=$w timeout -k 10 120 python bench.py --rows $r --nq 1 --profile-only --steps 400 --warmup 100 > $OUT/tmp.json 2>>$OUT/nq1_rows.err || exit 2
  python3 -c "import json,sys; d=json.loads(open('$OUT/tmp.json').read().strip().splitlines()[-1]); d['rows']=$r; d['wgpcu']=$w; print(json.dumps(d))" >> $OUT/nq1_rows.jsonl
done; done
cat $OUT/nq1_rows.jsonl
