#!/bin/bash
# round 6, session ah: ResNet-50 and BERT-base kernel traces at the final round-6 build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out; mkdir -p $OUT
rm -rf /tmp/prof_resnet7
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/prof_resnet7 -o run -- python3 scripts/bench_models.py --model resnet50 --steps 10 --warmup 5 > $OUT/ah_resnet_prof.json 2> $OUT/ah_resnet_prof.err || exit 1
db=$(find /tmp/prof_resnet7 -name "*_results.db" | head -n 1); python scripts/rocpd_steps.py $db --steps 8 --top 60 > $OUT/ah_resnet_steps.txt 2>&1
python scripts/kernel_shares.py $OUT/ah_resnet_steps.txt > $OUT/ah_resnet_shares.txt 2>&1
head -3 $OUT/ah_resnet_steps.txt; cat $OUT/ah_resnet_shares.txt
rm -rf /tmp/prof_bert8
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/prof_bert8 -o run -- python3 scripts/bench_models.py --model bert_base --batch 128 --steps 10 --warmup 5 > $OUT/ah_bert_prof.json 2> $OUT/ah_bert_prof.err || exit 1
db=$(find /tmp/prof_bert8 -name "*_results.db" | head -n 1); python scripts/rocpd_steps.py $db --steps 8 --top 60 > $OUT/ah_bert_steps.txt 2>&1
python scripts/kernel_shares.py $OUT/ah_bert_steps.txt > $OUT/ah_bert_shares.txt 2>&1
head -3 $OUT/ah_bert_steps.txt; cat $OUT/ah_bert_shares.txt
