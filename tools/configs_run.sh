#!/bin/bash
# Bench lines for the other BASELINE configs on one GPU: cfg2 (1M x 768, L2) and the per-GPU shard
# of cfg4 (10M x 1968 over 8 GPUs = 1.25M rows per GPU)
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/configs; mkdir -p $OUT
timeout -k 10 400 python bench.py --config 2 > $OUT/cfg2.json 2> $OUT/cfg2.err || { tail -20 $OUT/cfg2.err; exit 1; }
cat $OUT/cfg2.json
timeout -k 10 400 python bench.py --config 4 --rows 1250000 --no-cpu-baseline > $OUT/cfg4_shard.json 2> $OUT/cfg4_shard.err || { tail -20 $OUT/cfg4_shard.err; exit 2; }
cat $OUT/cfg4_shard.json
