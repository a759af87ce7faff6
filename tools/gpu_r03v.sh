#!/bin/bash
# Sliced second chance: tail-kernel time vs the slice count (config 2, int8 single queries).
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r03v}; mkdir -p $OUT
for S in ${SLICES:-8 16 32 64}; do
  IMGREC_SC_SLICES=$S CFG=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$S -o run --output-format csv -- python3 tools/i8_cfg2_probe.py > $OUT/prof_$S.log 2>&1 || { tail $OUT/prof_$S.log; exit 1; }
  grep '"mode": "i8"' $OUT/prof_$S.log | sed "s/^/S=$S /"
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/prof_$S/run_kernel_stats.csv')):
    if 'cert_tail' in r['Name']: print('S=$S tail', r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg', round(float(r['MaxNs'])/1e3,1), 'max')"
done
