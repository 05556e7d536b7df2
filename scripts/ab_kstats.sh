#!/bin/bash
# Kernel stats per library variant: for each ab/<v>.so in $VARIANTS (prod = the
# product library), rocprofv3 --kernel-trace --stats over bench.py $ARGS; prints
# the lsm kernels' average durations (us).  Diagnostic only.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in $VARIANTS; do
  lib=ab/$v.so; [ $v = prod ] && lib=go-lsm_amd/liblsm_gpu.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ks_$v -o run \
    -- python scripts/ab_lib.py $lib $ARGS --steps 20 --warmup 3 > gpurun_out/ks_$v.log 2>&1 || { tail -5 gpurun_out/ks_$v.log; exit 1; }
  python3 - $v <<'PY'
import csv, sys, glob
v = sys.argv[1]
f = glob.glob(f"gpurun_out/ks_{v}/**/*kernel_stats.csv", recursive=True)[0]
tot = 0
for r in csv.DictReader(open(f)):
    if "lsm::" in r["Name"]:
        us = float(r["AverageNs"]) / 1000
        print(v, r["Name"].split("(")[0].split("::")[-1][:40], r["Calls"], round(us, 1))
PY
done
