#!/bin/bash
# Full GPU session: parity tests (incl. the C++ mirror), smoke, every bench
# config, and rocprofv3 kernel stats of the default bench.  Each GPU step has
# its own limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
TAG=${TAG:-r01}
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name" >&2; timeout -k 10 $lim "$@"; }

step pytest 900 python -m pytest tests -m gpu -q -p no:cacheprovider > $OUT/pytest_gpu_$TAG.log 2>&1 \
  || { tail -60 $OUT/pytest_gpu_$TAG.log; exit 1; }
tail -2 $OUT/pytest_gpu_$TAG.log
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke_$TAG.log 2>&1 \
  || { tail -30 $OUT/smoke_$TAG.log; exit 1; }
tail -1 $OUT/smoke_$TAG.log
for cfg in ${CONFIGS:-decode4k decode64k mixed sst}; do
  step bench_$cfg 600 python bench.py --config $cfg > $OUT/bench_${TAG}_$cfg.json 2> $OUT/bench_${TAG}_$cfg.err \
    || { tail -30 $OUT/bench_${TAG}_$cfg.err; exit 1; }
  cat $OUT/bench_${TAG}_$cfg.json
done
if [[ -z $NOPROF ]]; then
  step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run \
    -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline > $OUT/prof_$TAG.log 2>&1 \
    || { tail -30 $OUT/prof_$TAG.log; exit 1; }
  find $OUT/prof_$TAG -name "*kernel_stats*"
fi
echo "== done"
