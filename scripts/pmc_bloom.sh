set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
export LSM_SST_DBG=3
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d gpurun_out/pmc_bl1 -o run -- python bench.py --config sst --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_bl1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SMEM SQ_CYCLES SQ_WAVES --output-format csv -d gpurun_out/pmc_bl2 -o run -- python bench.py --config sst --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_bl2.log 2>&1 && echo ok
