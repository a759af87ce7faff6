#!/bin/bash
# One GPU lease, several named stages run in order; each GPU step under its own timeout, the
# script stops at the first failure (gpurun rules: no retries, nothing after a fault).
#   tools/gpu_stages.sh TAG stage [stage ...]
# stages:
#   tests[=FILES]   pytest -m gpu (all, or the listed test files, comma-separated)
#   smoke           __graft_entry__.smoke()
#   bench           bench.py (default workload, CPU baseline included) -> bench.json
#   bench2          bench.py --config 2 (1M x 768) -> bench_cfg2.json
#   rows125k        bench.py --rows 125000 --profile-only (the N = 8 per-rank step) -> rows125k.json
#   nq1             bench.py --nq 1 --profile-only, cfg3 and cfg2 -> nq1_cfg{3,2}.json
#   rocprof         rocprofv3 --kernel-trace --stats of a bench run -> prof/
#   rehearse=N      gloo N-rank rehearsal of bench.py on this one GPU -> rehearse_nN.json
#   rehearse_pipe=N gloo N-rank rehearsal of bench_pipeline.py (config 5) on this one GPU -> pipe_nN.json
#   pipe            bench_pipeline.py, 100k images on this GPU -> pipe.json
#   pmc[=ARGS]      clock/MFMA-busy and HBM-traffic passes of the candidate kernel (bench args,
#                   comma-separated: pmc=--config,2)
#   vit             vit_gemm_rate.py (the forward's GEMM shapes, HIP vs hipBLASLt) + dreamsim_variants.py
#                   at batch 512 (hipBLASLt forward vs HIP-GEMM forward) -> vit_gemm_rate.jsonl, ds_variants.jsonl
#   trace=ARGS      kernel timeline of one search step (tools/trace_step.sh, bench args comma-separated)
#   probe=CFG       tools/i8_cfg2_probe.py: 32 single queries, certificate counts and times -> probe_cfgN.jsonl
#   stamps=CFG[:LIB] per-tile stage-loop / epilogue cycles of the 256 x 256 bf16 kernel on bench
#                   config CFG (lib/LIB, default libimgrec_stamps.so: tools/build_variants.sh stamps
#                   -DIMGREC_B16_STAMPS)
#   tailstamps=CFG  tools/tail_stamps.py: certificate-tail workgroup timestamps of one-query second
#                   chances (lib/libimgrec_tailstamps.so: build_variants.sh tailstamps -DIMGREC_TAIL_STAMPS)
#   ab=LIB          A/B of lib/libimgrec.so and lib/LIB: per-step and kernel ms on cfg2, cfg3 and
#                   the 125k-row shard
#                   (profile-only, twice alternating) -> ab_LIB.txt
# Extra bench arguments for every bench stage: BENCH_ARGS.
set -u
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
BA=${BENCH_ARGS:-}
fail() { echo "stage $1 failed"; tail -30 "$2"; exit 1; }
for st in "$@"; do
  name=${st%%=*}; arg=${st#*=}; [ "$arg" = "$st" ] && arg=""
  echo "== $st $(date +%T)"
  case $name in
    tests)
      files=tests; [ -n "$arg" ] && files=$(echo "$arg" | tr ',' ' ')
      timeout -k 10 1000 python -u -m pytest $files -x -v -s -m gpu --timeout 300 --timeout-method thread \
        > $OUT/pytest_$(echo "$arg" | tr ',/' '__' | cut -c1-40).log 2>&1 || fail tests $OUT/pytest_*.log
      tail -2 $OUT/pytest_*.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || fail smoke $OUT/smoke.log
      tail -2 $OUT/smoke.log ;;
    bench)
      timeout -k 10 500 python bench.py $BA > $OUT/bench.json 2> $OUT/bench.err || fail bench $OUT/bench.err
      cat $OUT/bench.json ;;
    bench2)
      timeout -k 10 500 python bench.py --config 2 --no-cpu-baseline $BA > $OUT/bench_cfg2.json 2> $OUT/bench_cfg2.err || fail bench2 $OUT/bench_cfg2.err
      cat $OUT/bench_cfg2.json ;;
    rows125k)
      timeout -k 10 300 python bench.py --rows 125000 --profile-only --steps 200 --warmup 50 $BA > $OUT/rows125k.json 2> $OUT/rows125k.err || fail rows125k $OUT/rows125k.err
      cat $OUT/rows125k.json ;;
    nq1)
      for c in 3 2; do
        timeout -k 10 300 python bench.py --config $c --nq 1 --profile-only --steps 300 --warmup 100 $BA > $OUT/nq1_cfg$c.json 2> $OUT/nq1_cfg$c.err || fail nq1 $OUT/nq1_cfg$c.err
        cat $OUT/nq1_cfg$c.json
      done ;;
    rocprof)
      timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline $BA > $OUT/prof.log 2>&1 || fail rocprof $OUT/prof.log
      head -8 $OUT/prof/run_kernel_stats.csv | cut -c1-220 ;;
    rehearse)
      n=${arg:-8}
      IMGREC_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
        --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus $n --steps 3 --warmup 1 --single-query-steps 3 $BA \
        > $OUT/rehearse_n$n.json 2> $OUT/rehearse_n$n.err || fail rehearse $OUT/rehearse_n$n.err
      cat $OUT/rehearse_n$n.json ;;
    rehearse_pipe)
      n=${arg:-8}
      IMGREC_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
        --master-addr 127.0.0.1 --master-port 29534 bench_pipeline.py --gpus $n --images 16384 --model-batch 256 --search-reps 2 \
        > $OUT/pipe_n$n.json 2> $OUT/pipe_n$n.err || fail rehearse_pipe $OUT/pipe_n$n.err
      cat $OUT/pipe_n$n.json ;;
    pipe)
      timeout -k 10 400 python bench_pipeline.py > $OUT/pipe.json 2> $OUT/pipe.err || fail pipe $OUT/pipe.err
      cat $OUT/pipe.json ;;
    pmc)
      arg=${arg//,/ }                       # pmc=--config,2 -> "--config 2"
      BENCH_ARGS="$arg" bash tools/pmc_clock.sh $TAG/pmcclk > $OUT/pmc_clock.log 2>&1 || fail pmc $OUT/pmc_clock.log
      cat $OUT/pmc_clock.log
      BENCH_ARGS="$arg" bash tools/pmc_traffic.sh $TAG > $OUT/pmc_traffic.log 2>&1 || fail pmc $OUT/pmc_traffic.log
      tail -12 $OUT/pmc_traffic.log ;;
    vit)
      timeout -k 10 300 python tools/vit_gemm_rate.py > $OUT/vit_gemm_rate.jsonl 2> $OUT/vit_gemm_rate.err || fail vit $OUT/vit_gemm_rate.err
      cat $OUT/vit_gemm_rate.jsonl
      timeout -k 10 400 python tools/dreamsim_variants.py --batches 512 --iters 6 --variants fused_gelu_lt,hip_gemm,hip_gemm_tanh,fused_gelu_lt,hip_gemm,hip_gemm_tanh \
        > $OUT/ds_variants.jsonl 2> $OUT/ds_variants.err || fail vit $OUT/ds_variants.err
      cat $OUT/ds_variants.jsonl ;;
    trace)
      arg=${arg//,/ }
      bash tools/trace_step.sh $TAG/trace_$(echo "$arg" | tr ' -' '__') $arg > $OUT/trace.log 2>&1 || fail trace $OUT/trace.log
      cat $OUT/trace.log ;;
    probe)
      CFG=${arg:-2} FENCE=${FENCE:-eager} timeout -k 10 300 python tools/i8_cfg2_probe.py > $OUT/probe_cfg${arg:-2}.jsonl 2> $OUT/probe_cfg${arg:-2}.err || fail probe $OUT/probe_cfg${arg:-2}.err
      cat $OUT/probe_cfg${arg:-2}.jsonl ;;
    stamps)
      c=${arg%%:*}; c=${c:-3}; lib=libimgrec_stamps.so; [ "${arg#*:}" != "$arg" ] && lib=${arg#*:}
      IMGREC_LIB_NAME=$lib IMGREC_STAMPS_CFG=$c IMGREC_STAMPS_FN=knn_b16w_stamps_read timeout -k 10 300 python tools/b16_stamps.py \
        > $OUT/stamps_cfg${c}_$lib.json 2> $OUT/stamps_cfg${c}_$lib.err || fail stamps $OUT/stamps_cfg${c}_$lib.err
      cat $OUT/stamps_cfg${c}_$lib.err ;;
    tailstamps)
      CFG=${arg:-2} timeout -k 10 300 python tools/tail_stamps.py > $OUT/tail_stamps_cfg${arg:-2}.jsonl 2> $OUT/tail_stamps.err || fail tailstamps $OUT/tail_stamps.err
      tail -3 $OUT/tail_stamps_cfg${arg:-2}.jsonl ;;
    ab)
      for rep in 1 2; do
        for lib in libimgrec.so $arg; do
          for c in 2 3 r125k; do
            ca="--config $c"; [ $c = r125k ] && ca="--rows 125000"
            IMGREC_LIB_NAME=$lib timeout -k 10 200 python bench.py $ca --profile-only --no-phases --steps 60 --warmup 20 \
              > $OUT/ab.json 2>> $OUT/ab.err || fail ab $OUT/ab.err
            python3 -c "import json;d=json.load(open('$OUT/ab.json'));print('$rep $lib cfg$c step', round(d['ms_per_step'],4), 'kernel', round(d['kernel_ms'],4))" | tee -a $OUT/ab_$arg.txt
          done
        done
      done ;;
    *) echo "unknown stage $st"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
