#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
TAG=${TAG:-r01}
STEPS=${STEPS:-tests,smoke,bench,prof}

run() { echo "== $1"; shift; "$@"; }

if [[ $STEPS == *tests* ]]; then
  run pytest timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider \
      ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1 || { tail -50 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
fi
if [[ $STEPS == *smoke* ]]; then
  run smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" \
      > $OUT/smoke.log 2>&1 || { tail -30 $OUT/smoke.log; exit 1; }
  tail -2 $OUT/smoke.log
fi
if [[ $STEPS == *bench* ]]; then
  run bench timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err \
      || { tail -30 $OUT/bench_$TAG.err; exit 1; }
  cat $OUT/bench_$TAG.json
fi
if [[ $STEPS == *prof* ]]; then
  export TMPDIR=/tmp
  run rocprof timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $OUT/prof_$TAG -o run -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} \
      > $OUT/prof_$TAG.log 2>&1 || { tail -30 $OUT/prof_$TAG.log; exit 1; }
  find $OUT/prof_$TAG -name "*stats*" | head
fi
if [[ $STEPS == *pmc* ]]; then
  export TMPDIR=/tmp
  run pmc_fetch timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv \
      -d $OUT/pmc_fetch_$TAG -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} \
      > $OUT/pmc_fetch_$TAG.log 2>&1 || { tail -30 $OUT/pmc_fetch_$TAG.log; exit 1; }
  run pmc_write timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv \
      -d $OUT/pmc_write_$TAG -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} \
      > $OUT/pmc_write_$TAG.log 2>&1 || { tail -30 $OUT/pmc_write_$TAG.log; exit 1; }
fi
echo "== done"
