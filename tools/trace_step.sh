#!/bin/bash
# Kernel timeline of one search step (rocprofv3 --kernel-trace): each kernel's duration and the
# gap before it, over the last step of `bench.py --profile-only` with the given arguments.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-trace}; shift; mkdir -p $OUT
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/t -o run -- python3 bench.py --profile-only --no-phases "$@" > $OUT/bench.json 2> $OUT/err.log || { tail -5 $OUT/err.log; exit 2; }
python3 tools/trace_summary.py $(ls $OUT/t/*/run_kernel_trace.csv $OUT/t/run_kernel_trace.csv 2>/dev/null | head -1) | tee $OUT/timeline.txt
