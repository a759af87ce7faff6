#!/bin/bash
# Round-3 first GPU call: HEAD's GPU tests + smoke, the default bench line, the hipBLASLt bf16 GEMM
# ceiling at the candidate kernel's shape (events + rocprofv3 kernel stats + one --pmc clock/busy
# pass, the same counters as tools/pmc_clock.sh on the fused kernel in the same call), and the
# 125k-row shard step under rocprofv3.  Each GPU step under its own timeout, stop at first failure.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r03a}; mkdir -p $OUT
CTR="GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA"
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
fi
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 2; }
cut -c1-400 $OUT/bench.json
timeout -k 10 180 python tools/gemm_ceiling.py > $OUT/gemm.jsonl 2> $OUT/gemm.err || { tail $OUT/gemm.err; exit 3; }
cat $OUT/gemm.jsonl
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/gemm_prof -o run --output-format csv -- python3 tools/gemm_ceiling.py --profile-only > $OUT/gemm_prof.log 2>&1 || { tail $OUT/gemm_prof.log; exit 4; }
head -5 $OUT/gemm_prof/run_kernel_stats.csv | cut -c1-220
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $CTR -d $OUT/gemm_pmc -o run --output-format csv -- python3 tools/gemm_ceiling.py --profile-only --steps 5 --warmup 1 > $OUT/gemm_pmc.log 2>&1 || { tail $OUT/gemm_pmc.log; exit 5; }
python3 tools/pmc_clock_summary.py $OUT/gemm_pmc $OUT/gemm_clock.json | grep -v -E "^(elementwise|distribution|.*normal)" || true
timeout -s KILL 90 rocprofv3 --kernel-trace --kernel-include-regex knn_b16 --pmc $CTR -d $OUT/knn_pmc -o run --output-format csv -- python3 bench.py --profile-only --steps 5 --warmup 1 > $OUT/knn_pmc.log 2>&1 || { tail $OUT/knn_pmc.log; exit 6; }
python3 tools/pmc_clock_summary.py $OUT/knn_pmc $OUT/knn_clock.json
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/prof125k -o run --output-format csv -- python3 bench.py --rows 125000 --profile-only --steps 50 --warmup 5 > $OUT/prof125k.log 2>&1 || { tail $OUT/prof125k.log; exit 7; }
cut -d, -f1-5 $OUT/prof125k/run_kernel_stats.csv | cut -c1-160
tail -1 $OUT/prof125k.log
