#!/bin/bash
# round 6, session x: BERT-base kernel trace after the tied word gradient (zeros fill + add gone?)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out; mkdir -p $OUT
rm -rf /tmp/prof_bert7
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/prof_bert7 -o run -- python3 scripts/bench_models.py --model bert_base --batch 128 --steps 10 --warmup 5 > $OUT/x_bert_prof.json 2> $OUT/x_bert_prof.err || exit 1
db=$(find /tmp/prof_bert7 -name "*_results.db" | head -n 1); python scripts/rocpd_steps.py $db --steps 8 --top 60 > $OUT/x_bert_steps.txt 2>&1
python scripts/kernel_shares.py $OUT/x_bert_steps.txt > $OUT/x_bert_shares.txt 2>&1
head -3 $OUT/x_bert_steps.txt; cat $OUT/x_bert_shares.txt
grep -n "Fill\|CUDAFunctor_add" $OUT/x_bert_steps.txt || true
