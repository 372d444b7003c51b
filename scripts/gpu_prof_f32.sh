cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { name=$1; shift; t=$1; shift; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; tail -40 gpurun_out/$name.log; [ $rc -le 1 ]; }
run prof_f32 200 python scripts/prof_persist_f32.py &&
run rocprof_b20 200 rocprofv3 --kernel-trace --stats -d gpurun_out/rp_b20 -o rp -- python bench.py --steps 20 --warmup 5
