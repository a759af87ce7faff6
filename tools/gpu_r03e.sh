#!/bin/bash
# Round-3 records: the default bench command under rocprofv3 --kernel-trace --stats (its events vs
# the trace), the r03 PMC traffic / clock records of the candidate kernel (one counter set per
# pass), per-rank steps at the N = 2 / 4 shard sizes, and the config-5 pipeline at 20k images.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r03e}; mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_bench -o run --output-format csv -- python3 bench.py > $OUT/bench_under_rocprof.json 2> $OUT/bench_under_rocprof.err || { tail $OUT/bench_under_rocprof.err; exit 1; }
python3 -c "
import json,csv; d=json.loads(open('$OUT/bench_under_rocprof.json').read().strip().splitlines()[-1]); print('events kernel_ms', d['roofline']['kernel_ms'], 'value', d['value'])
for r in csv.DictReader(open('$OUT/prof_bench/run_kernel_stats.csv')):
    if 'b16w' in r['Name']: print('rocprof avg ms', float(r['AverageNs'])/1e6, 'calls', r['Calls'])"
BENCH_ARGS="" timeout -k 10 300 bash tools/pmc_traffic.sh r03_v1 > $OUT/traffic.log 2>&1 || { tail $OUT/traffic.log; exit 2; }
tail -12 $OUT/traffic.log
timeout -k 10 200 bash tools/pmc_clock.sh pmcclk_r03 > $OUT/clock.log 2>&1 || { tail $OUT/clock.log; exit 3; }
tail -2 $OUT/clock.log
for r in 500000 250000; do timeout -k 10 200 python bench.py --rows $r --profile-only --steps 100 --warmup 30 >> $OUT/shards.jsonl 2>>$OUT/shards.err || exit 4; done
cat $OUT/shards.jsonl
timeout -k 10 400 python bench_pipeline.py --images 20000 > $OUT/pipeline_20k.json 2> $OUT/pipeline_20k.err || { tail $OUT/pipeline_20k.err; exit 5; }
cut -c1-700 $OUT/pipeline_20k.json
IMGREC_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench_pipeline.py --gpus 2 --images 4096 --model-batch 256 --nq 256 --search-reps 2 > $OUT/pipeline_gloo_n2.json 2> $OUT/pipeline_gloo_n2.err || { tail -20 $OUT/pipeline_gloo_n2.err; exit 6; }
cut -c1-600 $OUT/pipeline_gloo_n2.json
