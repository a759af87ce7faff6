#!/bin/bash
# Round-3 check after the merge-select and DreamSim prologue changes: every GPU test, smoke, the
# bench line, the 125k-row (N = 8 per-rank) and nq = 1 steps, the DreamSim variants at batch 512.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r03d}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $OUT/pytest.log | head; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 2; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json')); print('value', d['value'], 'ms', d['ms_per_step'], 'kernel', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac']); print('single', d['single_query'])"
for i in 1 2; do timeout -k 10 120 python bench.py --rows 125000 --profile-only --steps 200 --warmup 50 >> $OUT/rows125k.jsonl 2>>$OUT/rows125k.err || exit 3; done
cat $OUT/rows125k.jsonl
for i in 1 2; do timeout -k 10 120 python bench.py --nq 1 --profile-only --steps 300 --warmup 50 >> $OUT/nq1.jsonl 2>>$OUT/nq1.err || exit 4; done
cat $OUT/nq1.jsonl
timeout -k 10 300 python tools/dreamsim_variants.py --batches 512 --variants fused_gelu_lt,fused_gelu_lt@efficient,fused --iters 8 > $OUT/variants.jsonl 2> $OUT/variants.err || { tail $OUT/variants.err; exit 5; }
cat $OUT/variants.jsonl
timeout -k 10 400 bash tools/rehearse_ranks.sh 8 > $OUT/rehearse_n8.log 2>&1 || { echo "rehearsal failed"; tail -30 $OUT/rehearse_n8.log; exit 6; }
cp gpurun_out/rehearse/n8.json $OUT/rehearse_gloo_n8.json && cut -c1-400 $OUT/rehearse_gloo_n8.json
