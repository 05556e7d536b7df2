set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc1
export TMPDIR=/tmp LSM_LANE_BLOCKS=3
i=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc1/p$i -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/pmc1/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc1/p$i.log; }
done
ls gpurun_out/pmc1/*/
