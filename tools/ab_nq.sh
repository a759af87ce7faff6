#!/bin/bash
# A/B of lib/libimgrec.so against lib/$2 at nq = $NQ (default 1) on configs 2 and 3, twice alternating -> gpurun_out/$1/ab.txt
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$1; mkdir -p $OUT
for rep in 1 2; do
  for lib in libimgrec.so $2; do
    for c in 2 3; do
      IMGREC_LIB_NAME=$lib timeout -k 10 200 python bench.py --config $c --nq ${NQ:-1} --profile-only --steps 300 --warmup 100 > $OUT/ab.json 2>> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
      python3 -c "import json;d=json.load(open('$OUT/ab.json'));print('$rep $lib cfg$c nq ${NQ:-1} step', round(d['ms_per_step'],4), 'kernel', round(d['kernel_ms'],4))" | tee -a $OUT/ab.txt
    done
  done
done
