#!/bin/bash
# cfg4's whole 10M x 1968 corpus resident on ONE MI355X (fp32 + bf16 + split copies, ~200 GB)
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/cfg4_1gpu; mkdir -p $OUT
( while sleep 30; do date >> $OUT/alive.txt; done ) & HB=$!
timeout -k 10 700 python -u bench.py --config 4 --no-cpu-baseline --steps 5 --warmup 1 --single-query-steps 10 > $OUT/bench.json 2> $OUT/bench.err
rc=$?
kill $HB
cat $OUT/bench.json; tail -5 $OUT/bench.err
exit $rc
