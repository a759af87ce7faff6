#!/bin/bash
# DreamSim-architecture forward at batch 512 with PyTorch TunableOp: every GEMM shape of the
# forward benchmarked over the hipBLASLt / rocBLAS solutions once (results file), then replayed
# from the file with tuning off.  Baseline first, same process settings otherwise.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r03h}; mkdir -p $OUT
V=${VARIANTS:-fused_gelu_lt,fused_gelu_lt@efficient}
timeout -k 10 300 python tools/dreamsim_variants.py --batches 512 --variants $V --iters 6 > $OUT/base.jsonl 2> $OUT/base.err || { tail $OUT/base.err; exit 1; }
cat $OUT/base.jsonl
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 PYTORCH_TUNABLEOP_FILENAME=$OUT/tunableop_results.csv \
  timeout -k 10 600 python tools/dreamsim_variants.py --batches 512 --variants $V --iters 6 > $OUT/tune.jsonl 2> $OUT/tune.err || { tail $OUT/tune.err; exit 2; }
cat $OUT/tune.jsonl
ls $OUT
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$OUT/tunableop_results.csv \
  timeout -k 10 300 python tools/dreamsim_variants.py --batches 512 --variants $V --iters 6 > $OUT/replay.jsonl 2> $OUT/replay.err || { tail $OUT/replay.err; exit 3; }
cat $OUT/replay.jsonl
