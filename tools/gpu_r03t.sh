#!/bin/bash
# Sliced second chance: the certificate suites, then the config-2 single-query probe.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r03t}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_i8_gpu.py tests/test_bf16_gpu.py tests/test_certificate_multi_gpu.py tests/test_split_gpu.py tests/test_sweep_gpu.py tests/test_configs_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
CFG=2 timeout -k 10 300 python tools/i8_cfg2_probe.py > $OUT/probe_cfg2.jsonl 2>> $OUT/err.log || { tail $OUT/err.log; exit 2; }
cat $OUT/probe_cfg2.jsonl
