#!/bin/bash
# int8 single-query scan: workgroups per CU (IMGREC_I8_WGPCU, the split count = CUs x this) on
# configs 2 and 3, bench --nq $NQ (default 1) --profile-only, twice alternating.  Writes
# gpurun_out/$1/.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-i8_wgpcu}; mkdir -p $OUT
for rep in 1 2; do
  for w in ${WGPCU_LIST:-2 3 4 6}; do
    for c in 2 3; do
      IMGREC_I8_WGPCU=$w timeout -k 10 200 python bench.py --config $c --nq ${NQ:-1} --profile-only --steps 300 --warmup 100 \
        > $OUT/w${w}_cfg$c.json 2>> $OUT/err.log || { tail -5 $OUT/err.log; exit 1; }
      python3 -c "import json;d=json.load(open('$OUT/w${w}_cfg$c.json'));print('$rep nq ${NQ:-1} wgpcu $w cfg$c step', round(d['ms_per_step'],4), 'kernel', round(d['kernel_ms'],4))" | tee -a $OUT/sweep.txt
    done
  done
done
