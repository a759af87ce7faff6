#!/bin/bash
# One-query search and int8 scan kernel time against the corpus size (a line fit separates the
# scan's fixed cost from its streaming rate): bench.py --nq 1 --profile-only at --rows R for
# configs $CFGS (default "2 3") -> gpurun_out/TAG/scan_rows.txt
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$1; mkdir -p $OUT
for c in ${CFGS:-2 3}; do
  for r in 125000 250000 500000 1000000; do
    timeout -k 10 200 python bench.py --config $c --rows $r --nq 1 --profile-only --no-phases --steps 200 --warmup 50 > $OUT/s.json 2>> $OUT/s.err || { tail -5 $OUT/s.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/s.json'));print('cfg$c rows $r step', round(d['ms_per_step'],4), 'kernel', round(d['kernel_ms'],4))" | tee -a $OUT/scan_rows.txt
  done
done
