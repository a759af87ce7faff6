#!/bin/bash
# bench.py --profile-only per (config, nq, mode): tools/ab_modes_nq.sh TAG "2 3" "4 5 8" "bf16 i8"
# -> gpurun_out/TAG/modes_nq.txt
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$1; mkdir -p $OUT
for c in $2; do
  for nq in $3; do
    for m in $4; do
      timeout -k 10 200 python bench.py --config $c --nq $nq --mode $m --profile-only --no-phases --steps 100 --warmup 30 > $OUT/m.json 2>> $OUT/m.err || { tail -5 $OUT/m.err; exit 1; }
      python3 -c "import json;d=json.load(open('$OUT/m.json'));print('cfg$c nq $nq $m step', round(d['ms_per_step'],4), 'kernel', round(d['kernel_ms'],4))" | tee -a $OUT/modes_nq.txt
    done
  done
done
