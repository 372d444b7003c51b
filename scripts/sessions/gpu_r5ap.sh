set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python scripts/bench_models.py --model bert_base --batch 128 --steps 30 --warmup 10 > gpurun_out/r5ap_bert.json 2> gpurun_out/r5ap_bert.err || { tail -n 20 gpurun_out/r5ap_bert.err; exit 1; }
tail -n 1 gpurun_out/r5ap_bert.json | cut -c1-120
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_bert6 -o run -- python3 scripts/bench_models.py --model bert_base --batch 128 --steps 10 --warmup 5 > gpurun_out/r5ap_bert_prof.json 2> gpurun_out/r5ap_bert_prof.err || exit 1
db=$(find /tmp/prof_bert6 -name "*_results.db"); python scripts/rocpd_steps.py $db --steps 8 --top 40 > gpurun_out/r5ap_bert_steps.txt 2>&1
python scripts/kernel_shares.py gpurun_out/r5ap_bert_steps.txt
grep -h "slab\|colsum" gpurun_out/r5ap_bert_steps.txt | cut -c1-100
echo done
