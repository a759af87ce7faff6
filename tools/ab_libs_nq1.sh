#!/bin/bash
# One-query search on configs 2 and 3 for several library builds, twice alternating:
# tools/ab_libs_nq1.sh TAG libimgrec.so libimgrec_X.so ... -> gpurun_out/TAG/ab_nq1.txt
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$1; shift; mkdir -p $OUT
for rep in 1 2; do
  for lib in "$@"; do
    for c in 2 3; do
      IMGREC_LIB_NAME=$lib timeout -k 10 200 python bench.py --config $c --nq 1 --profile-only --no-phases --steps 300 --warmup 100 > $OUT/a.json 2>> $OUT/a.err || { tail -5 $OUT/a.err; exit 1; }
      python3 -c "import json;d=json.load(open('$OUT/a.json'));print('$rep $lib cfg$c step', round(d['ms_per_step'],4), 'kernel', round(d['kernel_ms'],4))" | tee -a $OUT/ab_nq1.txt
    done
  done
done
