#!/bin/bash
# Decode ring-size A/B on one box: decode parity under each variant, then
# alternating bench runs of the decode configs (LSM_DECODE_KERNEL=<v>; "v2" =
# the default 8 KiB ring).
set -o pipefail
mkdir -p gpurun_out
for v in ${VARIANTS:-v2 v2r6}; do
  e=$v; [ "$v" = v2 ] && e=
  LSM_DECODE_KERNEL=$e timeout -k 10 300 python -u -m pytest tests -m gpu -q -k "decode" --timeout 120 \
      --timeout-method thread -p no:cacheprovider > gpurun_out/ring_test_$v.log 2>&1 || { tail -30 gpurun_out/ring_test_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/ring_test_$v.log)"
done
for r in 1 2; do
  for c in ${CONFIGS:-decode4k decode64k mixed}; do
    for v in ${VARIANTS:-v2 v2r6}; do
      e=$v; [ "$v" = v2 ] && e=
      LSM_DECODE_KERNEL=$e timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > gpurun_out/ring_${c}_${v}_$r.json 2> gpurun_out/ring_$v.err \
        || { tail -20 gpurun_out/ring_$v.err; exit 1; }
      echo "$c $v run $r: $(python -c "import json; d=json.load(open('gpurun_out/ring_${c}_${v}_$r.json')); print(d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'])")"
    done
  done
done
