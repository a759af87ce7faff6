#!/bin/bash
# Round-2 measurements of the device-side certificate path: the cfg2 bench line (1M x 768, L2),
# the N = 8 shard shape (125k rows) per-step time, and a kernel trace of that shape (what runs
# outside the candidate kernel).  Each GPU step under its own timeout; stop at the first failure.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r02_over}; mkdir -p $OUT
timeout -k 10 300 python bench.py --config 2 --no-cpu-baseline > $OUT/cfg2.json 2> $OUT/cfg2.err || { tail $OUT/cfg2.err; exit 1; }
cat $OUT/cfg2.json
for R in 125000 1000000; do
  timeout -k 10 300 python bench.py --rows $R --profile-only --steps 50 --warmup 5 > $OUT/rows_$R.json 2>> $OUT/err.log || exit 2
  cat $OUT/rows_$R.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof125k -o run --output-format csv -- python3 bench.py --rows 125000 --profile-only --steps 50 --warmup 5 > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 3; }
cut -d, -f1-8 $OUT/prof125k/run_kernel_stats.csv | head -20
