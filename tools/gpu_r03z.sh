#!/bin/bash
# int8 path with integer dot4 products and a two-level int8 query: its tests + sweep, then the
# per-search step at nq = 1..4 (forced i8) and the config-2 probe.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r03z}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_i8_gpu.py tests/test_sweep_gpu.py -k "i8" -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for nq in ${NQS:-1 2 3 4 5 8}; do
  timeout -k 10 120 python bench.py --nq $nq --mode i8 --profile-only --steps 300 --warmup 100 > $OUT/nq$nq.json 2>>$OUT/err.log || exit 2
  echo "nq $nq $(cat $OUT/nq$nq.json)"
done
CFG=2 timeout -k 10 300 python tools/i8_cfg2_probe.py > $OUT/probe_cfg2.jsonl 2>> $OUT/err.log || exit 3
cat $OUT/probe_cfg2.jsonl
