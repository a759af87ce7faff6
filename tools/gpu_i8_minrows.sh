#!/bin/bash
# Where the candidate paths overtake the exact fp32 kernel on small corpora: per-search steps at
# several corpus sizes (ROWS), batch NQ (default 1), search modes MODES (default exact i8 auto).
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-i8_minrows}; mkdir -p $OUT
for rows in ${ROWS:-16384 32768 65536 131072}; do
  for mode in ${MODES:-exact i8 auto}; do
    timeout -k 10 120 python bench.py --rows $rows --nq ${NQ:-1} --mode $mode --profile-only --steps 300 --warmup 100 > $OUT/q${NQ:-1}.r$rows.$mode.json 2>>$OUT/err.log || exit 2
    python3 -c "import json;d=json.load(open('$OUT/q${NQ:-1}.r$rows.$mode.json'));print('nq ${NQ:-1}', $rows, '$mode', round(d['ms_per_step'],4), round(d['kernel_ms'],4))"
  done
done
