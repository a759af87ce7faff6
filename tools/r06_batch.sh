#!/bin/bash
# Round-6 GPU batch: the large-k / sweep / sharded tests, the cfg2 / cfg3 epilogue split, the
# default bench (with its live PMC passes), and the config-5 pipeline's 2-rank gloo rehearsal.
# Every GPU step has its own time limit; the first failure ends the batch.
set -o pipefail
O=gpurun_out/r06
mkdir -p $O
step() { echo "[batch] $1" >&2; }
step tests
timeout -k 10 900 python -u -m pytest tests/test_largek_gpu.py tests/test_sweep_gpu.py tests/test_sharded_gpu.py \
    tests/test_certificate_multi_gpu.py tests/test_i8_gpu.py tests/test_vit_gemm_gpu.py -x -v --timeout 300 \
    --timeout-method thread -s > $O/largek.log 2>&1 || { tail -30 $O/largek.log; exit 1; }
tail -2 $O/largek.log
step epi
bash tools/b16w_epi_split.sh $O/epi_cfg2 --config 2 || exit 2
bash tools/b16w_epi_split.sh $O/epi_cfg3 --config 3 || exit 3
step bench
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 4; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['frac'], d['roofline']['traffic'], d['roofline']['pmc_live'], d['single_query'])"
step pipeline
IMGREC_DIST_BACKEND=gloo timeout -k 10 600 python bench_pipeline.py --gpus 2 --images 8192 --model-batch 256 \
    --nq 256 --search-reps 2 > $O/pipe_gloo2.json 2> $O/pipe_gloo2.err || { tail -20 $O/pipe_gloo2.err; exit 5; }
cat $O/pipe_gloo2.json
