#!/bin/bash
# Per-kernel averages (rocprofv3 --stats) of the search's non-candidate kernels for library
# variants (LIBS) at one shard size (ROWS); the bf16 parity tests on TEST_LIBS first.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-abpost}; mkdir -p $OUT
for v in ${TEST_LIBS:-}; do IMGREC_LIB_NAME=$v timeout -k 10 400 python -u -m pytest tests/test_bf16_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_$v.log 2>&1 || { tail -30 $OUT/pytest_$v.log; exit 1; }; echo "$v $(tail -1 $OUT/pytest_$v.log)"; done
for r in 1 2; do for v in $LIBS; do
  IMGREC_LIB_NAME=$v timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $OUT/$v.$r -o run --output-format csv -- python3 bench.py --rows ${ROWS:-125000} --profile-only --steps 30 --warmup 3 > $OUT/$v.$r.log 2>&1 || exit 3
  python3 - $OUT/$v.$r/run_kernel_stats.csv $v <<'PY'
import csv, sys
keep = ("rerank", "cand_merge", "second", "fallback", "query_prep", "knn_merge", "b16w")
row = {r["Name"].split("(")[0].split("::")[-1][:22]: float(r["AverageNs"]) / 1000 for r in csv.DictReader(open(sys.argv[1])) if any(k in r["Name"] for k in keep)}
print(sys.argv[2], " ".join(f"{k}={v:.1f}" for k, v in sorted(row.items())))
PY
done; done
