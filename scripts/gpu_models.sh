#!/bin/bash
# Dense-model benches + a kernel profile of BERT (one gpurun call).
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  tail -1 $OUT/$name.log
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -5 $OUT/$name.log; exit $rc; fi
}
run bench_resnet50 300 python scripts/bench_models.py --model resnet50 --steps 30 --warmup 5
run bench_bert_b64 300 python scripts/bench_models.py --model bert_base --batch 64 --steps 30 --warmup 5
run bench_bert_b128 300 python scripts/bench_models.py --model bert_base --batch 128 --steps 20 --warmup 5
if [ "${PROF:-1}" = "1" ]; then
  rm -rf $OUT/prof_bert
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_bert -o run -- python3 scripts/bench_models.py --model bert_base --batch 64 --steps 10 --warmup 3 > $OUT/prof_bert.log 2>&1 || { echo "prof rc=$?"; exit 1; }
  rm -rf $OUT/prof_resnet
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_resnet -o run -- python3 scripts/bench_models.py --model resnet50 --steps 10 --warmup 3 > $OUT/prof_resnet.log 2>&1 || { echo "prof rc=$?"; exit 1; }
  find $OUT/prof_bert $OUT/prof_resnet -name "*kernel_stats*"
fi
