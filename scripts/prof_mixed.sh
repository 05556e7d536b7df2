set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mixed -o run -- python bench.py --config mixed --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_mixed.log 2>&1 || { tail -20 gpurun_out/prof_mixed.log; exit 1; }
find gpurun_out/prof_mixed -name "*stats*"
cat $(find gpurun_out/prof_mixed -name "*kernel_stats.csv" | head -1) | cut -c1-250
