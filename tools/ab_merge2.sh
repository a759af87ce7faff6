#!/bin/bash
# level-2 candidate merge A/B (LIBS), with the merge kernels' durations from rocprofv3 per library
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/ab_merge2; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_bf16_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for v in ${LIBS:-libimgrec.so}; do
  IMGREC_LIB_NAME=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$v -o run --output-format csv -- python3 tools/small_batch.py bf16 1,8,64 > $OUT/$v.jsonl 2> $OUT/$v.err || { tail -20 $OUT/$v.err; exit 2; }
  echo "== $v"; cut -c1-110 $OUT/$v.jsonl; grep -i "merge_lds\|merge_rank" $OUT/prof_$v/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-40,100-200
done
