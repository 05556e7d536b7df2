set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc2/fetch -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/pmc2/f.log 2>&1 || { tail gpurun_out/pmc2/f.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc2/write -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/pmc2/w.log 2>&1 || { tail gpurun_out/pmc2/w.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d gpurun_out/pmc2/p1 -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/pmc2/p1.log 2>&1 || { tail gpurun_out/pmc2/p1.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/pmc2/p2 -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/pmc2/p2.log 2>&1 || { tail gpurun_out/pmc2/p2.log; exit 1; }
python scripts/pmc_summary.py gpurun_out/pmc2/fetch gpurun_out/pmc2/write decode_spec_kernel decode4k:100000:desc gpurun_out/pmc2/summary.json
