#!/bin/bash
# A/B of library builds on bench lines: for each line in $LINES, run
# ab/<variant>.so for each variant in $VARIANTS, interleaved $REPS times.
# Prints "variant line value kernel_ms frac" per run.  Diagnostic only.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do
for line in ${LINES:-decode4k}; do
  case $line in
    cfg4) args="--global-blocks 1000000" ;;
    g[0-9]*) args="--global-blocks ${line#g}000" ;;
    arena) args="--arena" ;;
    *) args="--config $line" ;;
  esac
  for v in $VARIANTS; do
    lib=ab/$v.so; [ $v = prod ] && lib=go-lsm_amd/liblsm_gpu.so
    timeout -k 10 240 python scripts/ab_lib.py $lib $args --steps ${STEPS:-100} --warmup 10 > gpurun_out/abp_$v.json 2> gpurun_out/abp_$v.err || { tail -5 gpurun_out/abp_$v.err; exit 1; }
    python3 -c "import json,sys; j=json.load(open('gpurun_out/abp_$v.json')); r=j['roofline']; print('$v', '$line', j['value'], j['ms_per_step'], r['kernel_ms'], r.get('kernel_ms_median'), r['frac'], 'cold', (j.get('cold_input') or {}).get('value'))"
  done
done
done
