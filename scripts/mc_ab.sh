#!/bin/bash
# may_contain diagnostics: kernel stats with LSM_MC_DBG = 0, 1 (fill only), 2 (no L2 tail reads).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for d in ${DBGS:-0 1 2}; do
  rm -rf gpurun_out/prof_mc$d
  LSM_MC_DBG=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mc$d -o run -- \
      python bench.py --config probe --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/prof_mc$d.log 2>&1 \
      || { tail -20 gpurun_out/prof_mc$d.log; exit 1; }
done
