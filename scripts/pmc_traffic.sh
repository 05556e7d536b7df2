# HBM traffic (FETCH_SIZE, WRITE_SIZE in separate passes) of one decode config.
set -o pipefail
export TMPDIR=/tmp
CFG=${CFG:-decode64k}; TAG=${TAG:-x}
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmct_${TAG}_$c -o run -- python bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmct_${TAG}_$c.log 2>&1 || { tail -5 gpurun_out/pmct_${TAG}_$c.log; exit 1; }
done
python scripts/pmc_summary.py gpurun_out/pmct_${TAG}_FETCH_SIZE gpurun_out/pmct_${TAG}_WRITE_SIZE ${KSUB:-decode_v2_kernel} $CFG gpurun_out/pmct_${TAG}.json
