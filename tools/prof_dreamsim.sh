#!/bin/bash
# DreamSim-architecture forward: variant timings and a rocprofv3 kernel summary of the config-5
# dreamsim stage (bench_pipeline on 4096 images).  Writes under gpurun_out/$1.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-dreamsim}; mkdir -p $OUT
timeout -k 10 400 python tools/dreamsim_variants.py ${VARIANT_ARGS:-} > $OUT/variants.jsonl 2> $OUT/variants.err || { tail $OUT/variants.err; exit 1; }
cat $OUT/variants.jsonl
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench_pipeline.py --images 4096 --model-batch ${MB:-256} --nq 256 --search-reps 2 > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 2; }
tail -1 $OUT/prof.log
