#!/bin/bash
# Round-3 check after the lazy fence / event-free value region / lazy split copy / large-k
# workspace changes: every GPU test (incl. the new cfg2 1M and cfg4 10M whole-corpus tests),
# smoke, the bench line, the 125k-row shard step (N = 8 per-rank shape) and its kernel timeline.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r03b}; mkdir -p $OUT
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" $OUT/pytest.log | head -20; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
grep -E "cfg2:|cfg4 10M:" $OUT/pytest.log || true
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
fi
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 2; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json')); print('value', d['value'], 'ms', d['ms_per_step'], 'kernel', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac']); print('single', d['single_query']); print('cpu', d['cpu_baseline'])"
for i in 1 2; do timeout -k 10 120 python bench.py --rows 125000 --profile-only --steps 50 --warmup 5 >> $OUT/rows125k.jsonl 2>>$OUT/rows125k.err || exit 3; done
cat $OUT/rows125k.jsonl
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/prof125k -o run --output-format csv -- python3 bench.py --rows 125000 --profile-only --steps 50 --warmup 5 > $OUT/prof125k.log 2>&1 || { tail $OUT/prof125k.log; exit 4; }
grep elapsed $OUT/prof125k.log
timeout -k 10 600 python tools/bench_ingest.py --rows ${INGEST_ROWS:-1000000} > $OUT/ingest.json 2> $OUT/ingest.err || { echo "ingest failed"; tail -5 $OUT/ingest.err; exit 5; }
cut -c1-600 $OUT/ingest.json
