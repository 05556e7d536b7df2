#!/bin/bash
# Library A/B within one box: build_var/liblsm_gpu_<v>.so (variant builds,
# e.g. -D switches) swapped in as the product library per run; parity (GPU
# tests selected by $K) under each, then alternating bench runs of $CFG.
set -o pipefail
mkdir -p gpurun_out
orig=$(mktemp); cp go-lsm_amd/liblsm_gpu.so $orig
trap 'cp $orig go-lsm_amd/liblsm_gpu.so' EXIT
for v in $VARIANTS; do
  [ -z "$K" ] && break  # K empty: timing-only variants, no parity
  cp build_var/liblsm_gpu_$v.so go-lsm_amd/liblsm_gpu.so
  timeout -k 10 300 python -u -m pytest tests -m gpu -q -k "$K" --timeout 120 --timeout-method thread \
      -p no:cacheprovider > gpurun_out/libab_test_$v.log 2>&1 || { tail -30 gpurun_out/libab_test_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/libab_test_$v.log)"
done
for r in 1 2; do
  for v in $VARIANTS; do
    cp build_var/liblsm_gpu_$v.so go-lsm_amd/liblsm_gpu.so
    timeout -k 10 300 python bench.py --config $CFG --no-cpu-baseline > gpurun_out/libab_${v}_$r.json 2> gpurun_out/libab_$v.err \
      || { tail -20 gpurun_out/libab_$v.err; exit 1; }
    echo "$v run $r: $(python -c "import json; d=json.load(open('gpurun_out/libab_${v}_$r.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])")"
  done
done
