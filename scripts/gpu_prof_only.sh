cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python scripts/prof_persist_f32.py > gpurun_out/prof_f32.log 2>&1; rc=$?; echo "prof rc=$rc"; exit $rc
