set -u
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_bn_gpu.py -q -x > $OUT/bn_tests.log 2>&1 || { tail -30 $OUT/bn_tests.log; exit 1; }
tail -1 $OUT/bn_tests.log
timeout -k 10 300 python scripts/bench_models.py --model resnet50 --steps 30 --warmup 5 > $OUT/resnet_fused.log 2>&1 || { tail $OUT/resnet_fused.log; exit 1; }
tail -1 $OUT/resnet_fused.log
DTF_FUSED_BN=0 timeout -k 10 300 python scripts/bench_models.py --model resnet50 --steps 30 --warmup 5 > $OUT/resnet_miopen.log 2>&1 || { tail $OUT/resnet_miopen.log; exit 1; }
tail -1 $OUT/resnet_miopen.log
rm -rf $OUT/prof_resnet_bn
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_resnet_bn -o run -- python3 scripts/bench_models.py --model resnet50 --steps 10 --warmup 3 > $OUT/prof_resnet_bn.log 2>&1 || { echo prof fail; exit 1; }
find $OUT/prof_resnet_bn -name "*kernel_stats*"
