#!/bin/bash
# nq = 1 kernel time against whole rounds of 512 x 256-row tiles (1, 2, 4, 8 tiles per split):
# slope = one round, intercept = the fixed part of the launch.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r03i}; mkdir -p $OUT
for r in 131072 262144 524288 1048576 786432; do
  timeout -k 10 120 python bench.py --rows $r --nq 1 --profile-only --steps 400 --warmup 100 > $OUT/tmp.json 2>>$OUT/nq1_rows.err || exit 1
  python3 -c "import json,sys; d=json.loads(open('$OUT/tmp.json').read().strip().splitlines()[-1]); d['rows']=$r; print(json.dumps(d))" >> $OUT/nq1_rows.jsonl
done
cat $OUT/nq1_rows.jsonl
