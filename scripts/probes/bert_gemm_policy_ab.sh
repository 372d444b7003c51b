set -u
cd "${GRAFT_REPO_ROOT:-.}"
for pol in never auto always; do
  DTF_BIG_GEMM=$pol timeout -k 10 400 python scripts/bench_models.py --model bert_base --batch 128 --steps 20 --warmup 5 > gpurun_out/bert_$pol.log 2>&1
  rc=$?; echo "[bert_$pol] rc=$rc"; tail -1 gpurun_out/bert_$pol.log | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
done
