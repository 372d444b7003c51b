set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u scripts/bench_models.py --model resnet50 --steps 30 --warmup 10 > gpurun_out/rn.json 2> gpurun_out/rn.err || exit 1
timeout -k 10 300 python -u scripts/bench_models.py --model bert_base --steps 30 --warmup 10 > gpurun_out/bert.json 2> gpurun_out/bert.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_rn -o run -- python3 scripts/bench_models.py --model resnet50 --steps 10 --warmup 5 --trace-marker > gpurun_out/rn_p.json 2> gpurun_out/rn_p.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_bert -o run -- python3 scripts/bench_models.py --model bert_base --steps 10 --warmup 5 --trace-marker > gpurun_out/bert_p.json 2> gpurun_out/bert_p.err
