#!/bin/bash
# Round-2 checks after the colour (register SWAR) and rerank (two-phase prefix) changes: their
# parity tests, the colour rate against the per-byte-atomic build, and a kernel trace of the
# 125k-row shard step (rerank time).  Each GPU step under its own timeout.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r02b}; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_dropin_gpu.py tests/test_decode_pipeline_gpu.py tests/test_bf16_gpu.py tests/test_split_gpu.py tests/test_certificate_multi_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2; do for v in ${COLOR_LIBS:-libimgrec_colorlds.so libimgrec.so}; do IMGREC_LIB_NAME=$v timeout -k 10 120 python3 tools/color_hist_rate.py | head -1 || exit 2; done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof125k -o run --output-format csv -- python3 bench.py --rows 125000 --profile-only --steps 50 --warmup 5 > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 3; }
grep -E "rerank|b16w" $OUT/prof125k/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-60,200-
tail -1 $OUT/prof.log
