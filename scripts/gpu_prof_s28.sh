cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python scripts/prof_persist_f32.py fp32-s28 > gpurun_out/prof_s28.log 2>&1
