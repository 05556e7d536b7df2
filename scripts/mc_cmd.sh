#!/bin/bash
# may_contain: parity tests, probe bench, kernel stats.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_may_contain_gpu.py > gpurun_out/mc_tests.log 2>&1 || { tail -40 gpurun_out/mc_tests.log; exit 1; }
tail -2 gpurun_out/mc_tests.log
timeout -k 10 300 python bench.py --config probe > gpurun_out/bench_probe.json 2>gpurun_out/bench_probe.err \
    || { tail -20 gpurun_out/bench_probe.err; exit 1; }
cat gpurun_out/bench_probe.json
rm -rf gpurun_out/prof_probe
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_probe -o run -- \
    python bench.py --config probe --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_probe.log 2>&1 \
    || { tail -20 gpurun_out/prof_probe.log; exit 1; }
