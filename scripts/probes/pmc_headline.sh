# PMC pass over the headline engine (one counter pass, its own run; tuning / evidence)
set -e
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_headline
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc_headline -o run -- python3 bench.py --gpus 1 --steps 1100 --warmup 550 > gpurun_out/pmc_headline.log 2>&1
echo pmc ok
