#!/bin/bash
# ResNet-50 bench + kernel profile (one gpurun call).
set -u
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python scripts/bench_models.py --model resnet50 --steps 30 --warmup 5 "$@" > $OUT/resnet.log 2>&1 || { tail $OUT/resnet.log; exit 1; }
tail -1 $OUT/resnet.log
rm -rf $OUT/prof_resnet
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_resnet -o run -- python3 scripts/bench_models.py --model resnet50 --steps 10 --warmup 3 "$@" > $OUT/prof_resnet.log 2>&1 || { echo prof fail; tail $OUT/prof_resnet.log; exit 1; }
find $OUT/prof_resnet -name "*kernel_stats*"
