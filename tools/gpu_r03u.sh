#!/bin/bash
# Kernel durations of config-2 single-query searches on the int8 path (second chance active).
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r03u}; mkdir -p $OUT
CFG=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 tools/i8_cfg2_probe.py > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 1; }
python3 -c "
import csv
for r in list(csv.DictReader(open('$OUT/prof/run_kernel_stats.csv')))[:14]:
    print(r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg', round(float(r['MaxNs'])/1e3,1), 'max', r['Name'][:80])"
