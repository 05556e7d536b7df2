#!/bin/bash
# WAL replay A/B within one box: parity under each seg-kernel variant, then
# alternating bench runs (LSM_WAL_KERNEL = default, stage1k, ...).
set -o pipefail
mkdir -p gpurun_out
for v in ${VARIANTS:-default stage4k}; do
  LSM_WAL_KERNEL=$v timeout -k 10 300 python -u -m pytest tests -m gpu -q -k wal --timeout 120 --timeout-method thread \
      -p no:cacheprovider > gpurun_out/wal_ab_test_$v.log 2>&1 || { tail -30 gpurun_out/wal_ab_test_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/wal_ab_test_$v.log)"
done
for r in 1 2; do
  for v in ${VARIANTS:-default stage4k}; do
    LSM_WAL_KERNEL=$v timeout -k 10 300 python bench.py --config wal --no-cpu-baseline > gpurun_out/wal_ab_${v}_$r.json 2> gpurun_out/wal_ab_$v.err \
      || { tail -20 gpurun_out/wal_ab_$v.err; exit 1; }
    echo "$v run $r: $(python -c "import json,sys; d=json.load(open('gpurun_out/wal_ab_${v}_$r.json')); print(d['value'], d['ms_per_step'])")"
  done
done
