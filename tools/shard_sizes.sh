#!/bin/bash
# per-rank cost of the strong-scaling shards (1M / N rows on one GPU): step time vs kernel time,
# plus a kernel trace of the 125k-row (N = 8) shard to read the fixed per-step costs
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-shards}; mkdir -p $OUT
for r in 125000 250000 500000; do
  timeout -k 10 300 python bench.py --rows $r --steps 50 --warmup 5 --profile-only > $OUT/rows_$r.json 2> $OUT/rows_$r.err || { tail -20 $OUT/rows_$r.err; exit 1; }
  echo "$r $(cat $OUT/rows_$r.json)"
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof -o run --output-format csv -- python3 bench.py --rows 125000 --steps 30 --warmup 3 --profile-only > $OUT/prof.log 2>&1 || { echo "rocprof failed"; exit 3; }
echo done
