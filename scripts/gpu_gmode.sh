cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_ipc_gpu.py tests/test_mlp_persist_gpu.py -k "same_gpu" > gpurun_out/t_ipc.log 2>&1; echo "ipc tests rc=$?"; tail -3 gpurun_out/t_ipc.log
for prec in fp32 fp32-mfma fp32-split7; do for gm in 0 1 3; do
  DTF_GATHER_MODE=$gm timeout -k 10 120 python bench.py --steps 2200 --warmup 550 --precision $prec > gpurun_out/gm_${prec}_$gm.log 2>&1 || exit 1
  echo "$prec gmode=$gm $(python -c "import json,sys;d=json.loads(open('gpurun_out/gm_${prec}_$gm.log').read().strip().splitlines()[-1]);print(d['step_time_p50_ms'], d['value'])")"
done; done
