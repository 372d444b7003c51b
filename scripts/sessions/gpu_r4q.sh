set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_rn5 -o run -- python3 scripts/bench_models.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/rn_p5.json 2> gpurun_out/rn_p5.err || exit 1
db=$(find /tmp/prof_rn5 -name "*_results.db"); python scripts/rocpd_steps.py $db --steps 8 --top 60 > gpurun_out/rn5_steps.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_bert5 -o run -- python3 scripts/bench_models.py --model bert_base --batch 128 --steps 10 --warmup 5 > gpurun_out/bert_p5.json 2> gpurun_out/bert_p5.err || exit 1
db=$(find /tmp/prof_bert5 -name "*_results.db"); python scripts/rocpd_steps.py $db --steps 8 --top 60 > gpurun_out/bert5_steps.txt 2>&1
timeout -k 10 300 python -u scripts/bench_models.py --model resnet50 --steps 30 --warmup 10 > gpurun_out/rn_final.json 2> gpurun_out/rn_final.err || exit 1
timeout -k 10 300 python -u scripts/bench_models.py --model bert_base --batch 128 --steps 30 --warmup 10 > gpurun_out/bert_final.json 2> gpurun_out/bert_final.err || exit 1
