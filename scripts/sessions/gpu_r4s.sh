set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python -u scripts/bench_models.py --model bert_base --batch 128 --steps 30 --warmup 10"
for i in 1 2; do
timeout -k 10 300 $B > gpurun_out/bert_auto$i.json 2> gpurun_out/bert_auto$i.err || exit 1
DTF_BIG_GEMM=always timeout -k 10 300 $B > gpurun_out/bert_always$i.json 2> gpurun_out/bert_always$i.err || exit 1
done
