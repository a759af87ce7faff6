#!/bin/bash
# Instruction-cache and wait counters of the bf16 kernel (production vs stage-loop-only build)
set -o pipefail
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out/r06/icache; mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1
grep -o "SQC_[A-Z_0-9]*\|SQ_IFETCH[A-Z_0-9]*\|SQ_WAIT[A-Z_0-9]*\|SQ_INSTS_[A-Z_0-9]*" $O/avail.txt | sort -u > $O/names.txt
cat $O/names.txt | tr '\n' ' '; echo
R="--kernel-trace --kernel-include-regex knn_b16 --output-format csv"
for v in libimgrec.so libimgrec_noepi.so; do
  for pass in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE"; do
    tag=$(echo $pass | cut -c1-12 | tr ' ' '_')
    IMGREC_LIB_NAME=$v timeout -s KILL 120 rocprofv3 $R --pmc $pass -d $O/${v}_$tag -o run -- python3 bench.py --profile-only --steps 3 --warmup 1 --no-phases --config 2 > $O/${v}_$tag.log 2>&1 || { echo "$v $tag failed"; tail -3 $O/${v}_$tag.log; }
  done
done
python3 - $O <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
for d in sorted(glob.glob(o + "/*/")):
    f = glob.glob(d + "**/*counter_collection.csv", recursive=True)
    if not f: continue
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(d.split("/")[-2], {k: "%.4g" % (sum(v) / len(v)) for k, v in agg.items()})
PY
