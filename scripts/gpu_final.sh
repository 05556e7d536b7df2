#!/bin/bash
# Round-end evidence session: parity, smoke, every bench line, kernel stats,
# HBM traffic (PMC, separate passes) and the nt-load counter calibration.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; TAG=${TAG:-r01}
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name" >&2; timeout -k 10 $lim "$@"; }
PHASE=${PHASE:-all}  # 1: tests + bench lines, 2: profiles + PMC
if [ "$PHASE" != 2 ]; then
step pytest 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu_$TAG.log 2>&1 \
  || { tail -60 $OUT/pytest_gpu_$TAG.log; exit 1; }
tail -1 $OUT/pytest_gpu_$TAG.log
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke_$TAG.log 2>&1 \
  || { tail -30 $OUT/smoke_$TAG.log; exit 1; }
for cfg in ${CONFIGS:-decode4k decode64k mixed sst sstdec sstdec1 wal probe compact}; do
  step bench_$cfg 600 python bench.py --config $cfg > $OUT/bench_${TAG}_$cfg.json 2> $OUT/bench_${TAG}_$cfg.err \
    || { tail -30 $OUT/bench_${TAG}_$cfg.err; exit 1; }
  cut -c1-300 $OUT/bench_${TAG}_$cfg.json
done
step bench_e2e 600 python bench.py --e2e > $OUT/bench_${TAG}_e2e.json 2> $OUT/bench_${TAG}_e2e.err || exit 1
fi
[ "$PHASE" = 1 ] && { echo "== done"; exit 0; }
for cfg in ${PROF:-decode4k decode64k mixed sst sstdec wal probe compact}; do
  step prof_$cfg 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_${TAG}_$cfg -o run \
    -- python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline > $OUT/prof_${TAG}_$cfg.log 2>&1 || exit 1
done
for cfg in ${PMC:-decode4k decode64k mixed}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    step pmc_${cfg}_$c 300 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_${TAG}_${cfg}_$c -o run \
      -- python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline > $OUT/pmc_${TAG}_${cfg}_$c.log 2>&1 || exit 1
  done
done
for c in FETCH_SIZE WRITE_SIZE; do
  step pmcprobe_$c 300 rocprofv3 --pmc $c --output-format csv -d $OUT/pmcprobe_${TAG}_$c -o run \
    -- python tools/block_probe.py > $OUT/pmcprobe_${TAG}_$c.log 2>&1 || exit 1
done
echo "== done"
