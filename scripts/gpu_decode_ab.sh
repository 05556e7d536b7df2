#!/bin/bash
# Decode parity + decode bench lines, with optional kernel-variant A/B (one GPU call).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; TAG=${TAG:-ab}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_decode_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_decode_$TAG.log 2>&1 \
  || { tail -40 $OUT/pytest_decode_$TAG.log; exit 1; }
tail -1 $OUT/pytest_decode_$TAG.log
for v in ${VARIANTS:-default}; do
  for cfg in ${CONFIGS:-decode4k decode64k mixed}; do
    if [ "$v" = default ]; then unset LSM_DECODE_KERNEL; else export LSM_DECODE_KERNEL=$v; fi
    timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline > $OUT/bench_${TAG}_${v}_$cfg.json 2> $OUT/bench_${TAG}_${v}_$cfg.err \
      || { tail -30 $OUT/bench_${TAG}_${v}_$cfg.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/bench_${TAG}_${v}_$cfg.json'));print('$v $cfg', d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'])"
  done
done
