#!/bin/bash
# Round-2 GPU run: the config-shaped parity tests, the whole -m gpu suite, the bench line and a
# kernel-stats profile.  Every GPU step under its own timeout; stop at the first failure.
#   TESTS=tests/test_configs_gpu.py (default: all)   SKIP_BENCH=1   SKIP_PROF=1
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
TAG=${1:-r02}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -x -v -m gpu --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
grep -E "passed|failed" $OUT/pytest.log | tail -2
grep -E "^cfg3:|^8 shards:" $OUT/pytest.log || true
[ -n "${SKIP_BENCH:-}" ] && exit 0
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 2; }
cat $OUT/bench.json
[ -n "${SKIP_PROF:-}" ] && exit 0
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/prof.log 2>&1 || { echo "rocprof failed"; exit 3; }
head -8 $OUT/prof/run_kernel_stats.csv | cut -c1-200
