#!/bin/bash
# One gpurun session: GPU tests, a short bench, and a rocprofv3 kernel profile.
# Stops at the first GPU fault / abort / timeout (exit codes other than 0/1
# from pytest, anything non-zero from the others).
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
STEPS=${STEPS:-2000}

fatal() { rc=$1; [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; }

python -c "import distributed_tensorflow_example_amd._native as n; n.load(); print('native ok')" > $OUT/native.log 2>&1 || exit 3

if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-420} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
  rc=$?
  tail -5 $OUT/pytest_gpu.log
  if fatal $rc; then echo "pytest fatal rc=$rc"; exit $rc; fi
fi

timeout -k 10 300 python bench.py --steps $STEPS --warmup 500 > $OUT/bench.log 2>&1
rc=$?; cat $OUT/bench.log | tail -3
[ $rc -ne 0 ] && { echo "bench rc=$rc"; exit $rc; }

timeout -k 10 300 python bench.py --steps $STEPS --warmup 500 --eager > $OUT/bench_eager.log 2>&1
rc=$?; tail -1 $OUT/bench_eager.log
[ $rc -ne 0 ] && { echo "bench eager rc=$rc"; exit $rc; }

if [ "${MODEL_BENCH:-0}" = "1" ]; then
  for m in ${MODELS:-sparse_lr wide_deep bert_base resnet50}; do
    timeout -k 10 300 python scripts/bench_models.py --model $m --steps ${MODEL_STEPS:-50} --warmup 10 > $OUT/bench_$m.log 2>&1
    rc=$?; tail -1 $OUT/bench_$m.log
    [ $rc -ne 0 ] && { echo "bench $m rc=$rc"; exit $rc; }
  done
fi

if [ "${SKIP_PROF:-0}" != "1" ]; then
  rm -rf $OUT/prof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv rocpd -d $OUT/prof -o run -- python3 bench.py --steps 1000 --warmup 200 > $OUT/prof.log 2>&1
  rc=$?; tail -2 $OUT/prof.log
  [ $rc -ne 0 ] && { echo "prof rc=$rc"; exit $rc; }
  find $OUT/prof -name "*stats*" | head
fi
exit 0
