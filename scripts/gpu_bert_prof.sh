#!/bin/bash
# BERT-base bench + steady-state kernel profile (one gpurun call).
set -u
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
B=${B:-128}
timeout -k 10 600 python scripts/bench_models.py --model bert_base --batch $B --steps 20 --warmup 5 "$@" > $OUT/bert.log 2>&1 || { tail $OUT/bert.log; exit 1; }
tail -1 $OUT/bert.log
rm -rf $OUT/prof_bert
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_bert -o run -- python3 scripts/bench_models.py --model bert_base --batch $B --steps 10 --warmup 3 "$@" > $OUT/prof_bert.log 2>&1 || { echo prof fail; tail $OUT/prof_bert.log; exit 1; }
python3 scripts/prof_summary.py $OUT/prof_bert/run_kernel_trace.csv --steps 13 --top 40 > $OUT/prof_bert_summary.txt
