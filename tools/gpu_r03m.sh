#!/bin/bash
# HIP attention kernel (vit_attention_bf16): its tests, then the DreamSim forward with it vs SDPA
# and a rocprofv3 kernel split of the new default forward.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r03m}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_vit_fused_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python tools/dreamsim_variants.py --batches 512 --variants fused_gelu_lt,fused_gelu_lt_sdpa,fused_gelu_lt --iters 6 > $OUT/variants.jsonl 2> $OUT/variants.err || { tail $OUT/variants.err; exit 2; }
cat $OUT/variants.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 tools/dreamsim_variants.py --batches 512 --variants fused_gelu_lt --iters 4 > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 3; }
python3 - $OUT/prof/run_kernel_stats.csv <<'PY'
import csv, sys
r = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(x["TotalDurationNs"]) for x in r)
for x in r[:12]:
    print(x["Calls"], round(float(x["AverageNs"]) / 1e3, 1), "us", round(float(x["TotalDurationNs"]) / tot * 100, 1), "%", x["Name"][:80])
PY
