set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out


timeout -k 10 300 python bench.py --e2e > gpurun_out/bench_e2e.json 2>gpurun_out/bench_e2e.err || { tail -20 gpurun_out/bench_e2e.err; exit 1; }
cat gpurun_out/bench_e2e.json
timeout -k 10 300 python bench.py --e2e --chunk 25000 > gpurun_out/bench_e2e2.json 2>gpurun_out/bench_e2e2.err || { tail -20 gpurun_out/bench_e2e2.err; exit 1; }
cat gpurun_out/bench_e2e2.json
