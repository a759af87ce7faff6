#!/bin/bash
# A/B of two builds of the library on one box: per-search steps at the given nq list on the
# int8 path, alternating libimgrec.so (A) and $ALT (B) twice.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-ab}; mkdir -p $OUT
for rep in 1 2; do
  for lib in libimgrec.so $ALT; do
    for nq in ${NQS:-1 8}; do
      IMGREC_LIB_NAME=$lib timeout -k 10 120 python bench.py --nq $nq --mode ${MODE:-i8} --profile-only --steps 300 --warmup 100 > $OUT/r$rep.$lib.nq$nq.json 2>>$OUT/err.log || exit 2
      python3 -c "import json;d=json.load(open('$OUT/r$rep.$lib.nq$nq.json'));print('$rep $lib nq $nq', round(d['ms_per_step'],4), round(d['kernel_ms'],4))"
    done
  done
done
