#!/bin/bash
# bench lines of the exact fp32 and split paths on the default workload (the AUTO default is bf16)
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/modes; mkdir -p $OUT
for m in exact split; do
  timeout -k 10 400 python bench.py --mode $m --steps 10 --warmup 2 --no-cpu-baseline > $OUT/$m.json 2> $OUT/$m.err || { tail -20 $OUT/$m.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$m.json')); r=d['roofline']; print('$m', round(d['value']), r['kernel'], round(r['kernel_ms'],3), round(r['frac'],3), r['peak_basis'], d['recall_at_10'])"
done
