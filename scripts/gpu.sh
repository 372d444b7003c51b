#!/bin/bash
# One parameterised driver for GPU-box sessions (gpurun): each argument names a
# step, run in order under its own time limit, output in gpurun_out/<step>.log.
# The session stops at the first failing step (a GPU fault, abort, timeout or
# test failure), so nothing else touches the GPU after trouble.
#
#   gpurun --timeout 900 -- bash scripts/gpu.sh smoke persist same_gpu bench20
#
# Steps:
#   native        load the in-tree _C (fails loudly if it is missing / stale)
#   smoke         __graft_entry__.smoke()
#   pytest_gpu    every GPU test (tests -m gpu)
#   persist       persistent-engine numerics tests (1 GPU)
#   same_gpu      multi-rank exchange tests, 2-8 ranks sharing cuda:0
#   exchange8     only the W = 5..8 same-GPU exchange tests
#   bench20       bench.py at the driver's setting (--steps 20 --warmup 5), 3 runs
#   bench5500     bench.py defaults (10 epochs of 550 steps)
#   bench2        bench.py --gpus 2 as the driver launches it, both ranks on cuda:0
#   phases        per-phase device stamps of the fp32 engine (scripts/prof_persist_f32.py)
#   phase_sweep   the same under each "DBG:GATHER" pair of $PHASE_SWEEP (DTF_PERSIST_DBG /
#                 DTF_GATHER_MODE kernel knobs; default "0:3 1:3 0:0 0:1")
#   prof_bench    rocprofv3 kernel trace + stats of bench.py --steps 5500
#   lowering      compat-graph lowering tests + bench_graph_step
#   models        BERT-base / ResNet-50 / sparse benches (scripts/bench_models.py)
#   bert_prof     rocprofv3 kernel stats of BERT-base B=128
#   gemm          gemm_big numerics / race-screen tests, then in-tree GEMM vs
#                 hipBLASLt (scripts/bench_gemm.py)
#   gemm_sweep    gemm_big schedules vs hipBLASLt over K (fixed vs per-K-tile cost)
#   sparse        sparse LR / Wide&Deep / sparse-optimizer GPU tests + benches
#   ipc           IPC data-plane tests: collectives with 2-4 ranks on cuda:0, the
#                 compat example as 1 ps + 2 / 4 sync workers, then the per-run time
#                 of 1 ps + 2 workers (scripts/bench_graph_step.py --workers 2)
#   tests         the GPU tests named in $TESTS (pytest node ids / files)
# Env: STEP_ARGS_<step> adds arguments to that step's main command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
PYT="python -u -m pytest -v --timeout 240 --timeout-method thread"

run() {  # name timeout cmd... ; a failing step ends the session
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"
  tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}

for step in "$@"; do
  extra_var="STEP_ARGS_$step"
  extra=${!extra_var:-}
  case $step in
    native) run native 300 python -c "from distributed_tensorflow_example_amd import _native as n; C = n.load(); print('native', C.ARCH, getattr(C, 'SRC_HASH', '?'))" ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    pytest_gpu) run pytest_gpu 1100 $PYT tests -m gpu $extra ;;
    persist) run persist 600 $PYT -x tests/test_mlp_persist_gpu.py -k "not same_gpu and not two_ranks" $extra ;;
    same_gpu) run same_gpu 900 $PYT -x tests/test_mlp_persist_gpu.py tests/test_ipc_gpu.py -k "same_gpu or two_ranks" $extra ;;
    exchange8) run exchange8 700 $PYT -x tests/test_mlp_persist_gpu.py -k "eight_ranks or five_six" $extra ;;
    bench20)
      for i in 1 2 3; do
        run bench20_$i 180 python bench.py --gpus 1 --steps 20 --warmup 5 $extra
      done ;;
    bench5500) run bench5500 300 python bench.py --gpus 1 $extra ;;
    bench2)
      PORT=$((20000 + RANDOM % 20000))
      DTF_BENCH_SAME_GPU=1 run bench2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
        --master-addr=127.0.0.1 --master-port=$PORT bench.py --gpus 2 --steps 20 --warmup 5 $extra ;;
    phases) run phases 300 python scripts/prof_persist_f32.py fp32 $extra ;;
    phase_sweep)
      for pair in ${PHASE_SWEEP:-0:3 1:3 0:0 0:1}; do
        DTF_PERSIST_DBG=${pair%%:*} DTF_GATHER_MODE=${pair##*:} run phases_${pair%%:*}_${pair##*:} 300 \
          python scripts/prof_persist_f32.py fp32 $extra
      done ;;
    prof_bench)
      rm -rf $OUT/prof_bench
      run prof_bench 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_bench -o run -- \
        python3 bench.py --gpus 1 --steps 5500 --warmup 550 $extra ;;
    lowering)
      run lowering_tests 500 $PYT -x tests/test_lowering_gpu.py tests/test_lowering_cpu.py $extra
      run bench_graph 300 python scripts/bench_graph_step.py 2000
      rm -rf $OUT/prof_graph
      run prof_graph 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_graph -o run -- \
        python3 scripts/bench_graph_step.py 500 ;;
    models)
      run bench_resnet50 400 python scripts/bench_models.py --model resnet50 --steps 30 --warmup 5
      run bench_bert_b128 400 python scripts/bench_models.py --model bert_base --batch 128 --steps 20 --warmup 5 $extra ;;
    bert_prof)
      rm -rf $OUT/prof_bert
      run bert_prof 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_bert -o run -- \
        python3 scripts/bench_models.py --model bert_base --batch 128 --steps 10 --warmup 3 $extra
      python3 scripts/prof_summary.py $OUT/prof_bert/run_kernel_trace.csv --steps 13 --top 40 > $OUT/prof_bert_summary.txt ;;
    gemm_sweep) run gemm_sweep 300 python scripts/probes/gemm_k_sweep.py $extra ;;
    gemm)
      run gemm_tests 500 $PYT -x tests/test_gemm_big_gpu.py
      run gemm 400 python scripts/bench_gemm.py $extra ;;
    sparse)
      run sparse_tests 500 $PYT -x tests/test_models_gpu.py tests/test_async_ps_gpu.py tests/test_sparse_optim_gpu.py $extra
      run bench_lr2 300 python scripts/bench_models.py --model sparse_lr --graph
      run bench_wd 300 python scripts/bench_models.py --model wide_deep --graph ;;
    ipc)
      run ipc_tests 700 $PYT -x tests/test_ipc_coll_gpu.py tests/test_compat_ipc_gpu.py $extra
      run bench_workers2 400 python scripts/bench_graph_step.py --workers 2 1000 ;;
    tests) run tests 900 $PYT -x $TESTS $extra ;;
    *) echo "unknown step: $step"; exit 2 ;;
  esac
done
exit 0
