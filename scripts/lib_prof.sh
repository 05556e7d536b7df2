#!/bin/bash
# Kernel stats per library variant (build_var/liblsm_gpu_<v>.so swapped in):
# rocprofv3 --kernel-trace --stats over bench.py $ARGS; prints lsm kernels' averages.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
orig=$(mktemp); cp go-lsm_amd/liblsm_gpu.so $orig
trap 'cp $orig go-lsm_amd/liblsm_gpu.so' EXIT
for v in $VARIANTS; do
  cp build_var/liblsm_gpu_$v.so go-lsm_amd/liblsm_gpu.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lprof_$v -o run \
    -- python bench.py $ARGS --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/lprof_$v.log 2>&1 || { tail -5 gpurun_out/lprof_$v.log; exit 1; }
  python3 - $v <<'PY'
import csv, sys, glob
v = sys.argv[1]
f = glob.glob(f"gpurun_out/lprof_{v}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "lsm::" in r["Name"]:
        print(v, r["Name"].split("(")[0][-40:], r["Calls"], round(float(r["AverageNs"]) / 1000, 1))
PY
done
