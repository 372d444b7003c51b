set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u scripts/bench_models.py --model bert_base --batch 128 --steps 30 --warmup 10 > gpurun_out/bert128.json 2> gpurun_out/bert128.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_bert128 -o run -- python3 scripts/bench_models.py --model bert_base --batch 128 --steps 10 --warmup 5 > gpurun_out/bert128_p.json 2> gpurun_out/bert128_p.err
