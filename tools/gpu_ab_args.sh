#!/bin/bash
# A/B of two builds of the library on one box: bench.py --profile-only steps for each argument
# set in CASES (";"-separated), alternating libimgrec.so (A) and $ALT (B) twice.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-ab}; mkdir -p $OUT
IFS=';' read -ra CS <<< "${CASES:---nq 1;--rows 125000}"
for rep in 1 2; do
  for lib in libimgrec.so $ALT; do
    n=0
    for c in "${CS[@]}"; do
      n=$((n+1))
      IMGREC_LIB_NAME=$lib timeout -k 10 120 python bench.py $c --profile-only --steps 200 --warmup 60 > $OUT/r$rep.$lib.c$n.json 2>>$OUT/err.log || exit 2
      python3 -c "import json;d=json.load(open('$OUT/r$rep.$lib.c$n.json'));print('$rep $lib [$c]', round(d['ms_per_step'],4), round(d['kernel_ms'],4))"
    done
  done
done
