set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_encode_gpu.py tests/test_mirror.py -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for d in 0 3; do
LSM_SST_DBG=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sst_d$d -o run -- python bench.py --config sst --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_sst_d$d.log 2>&1 || exit 1
echo "dbg=$d"; grep -E "regions|bloom" gpurun_out/prof_sst_d$d/run_kernel_stats.csv | cut -d, -f1,4 | sed 's/lsm::(anonymous namespace):://; s/(lsm[^"]*//'
done
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM --output-format csv -d gpurun_out/pmc_sstB -o run -- python bench.py --config sst --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_sstB.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_sstC -o run -- python bench.py --config sst --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_sstC.log 2>&1 && echo pmc_ok
