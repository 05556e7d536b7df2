set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_r03b.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_r03b.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_r03b.log
timeout -k 10 300 python bench.py --config compact > gpurun_out/bench_r03b_compact.json 2> gpurun_out/bench_r03b_compact.err || { tail -20 gpurun_out/bench_r03b_compact.err; exit 1; }
cut -c1-400 gpurun_out/bench_r03b_compact.json
