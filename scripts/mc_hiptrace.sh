#!/bin/bash
# Host-side HIP API durations of the probe bench (runtime trace; no counters).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof_mchip
timeout -k 10 300 rocprofv3 --hip-trace --stats --output-format csv -d gpurun_out/prof_mchip -o run -- \
    python bench.py --config probe --steps 50 --warmup 2 --no-cpu-baseline > gpurun_out/prof_mchip.log 2>&1 \
    || { tail -20 gpurun_out/prof_mchip.log; exit 1; }
