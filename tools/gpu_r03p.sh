#!/bin/bash
# config-5 pipeline with the HIP attention kernel in the DreamSim stage: 20k and 100k images.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r03p}; mkdir -p $OUT
timeout -k 10 400 python bench_pipeline.py --images 20000 > $OUT/pipeline_20k.json 2> $OUT/pipeline_20k.err || { tail $OUT/pipeline_20k.err; exit 1; }
cat $OUT/pipeline_20k.json
timeout -k 10 500 python bench_pipeline.py --images 100000 > $OUT/pipeline_100k.json 2> $OUT/pipeline_100k.err || { tail $OUT/pipeline_100k.err; exit 2; }
cat $OUT/pipeline_100k.json
