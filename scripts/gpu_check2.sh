#!/bin/bash
# Round-2 check: GPU parity suite, smoke, the default bench line, config 4 at
# N=1 (1M blocks), and the self-launching N=2 path rehearsed on one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; TAG=${TAG:-r02}
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name" >&2; timeout -k 10 $lim "$@"; }
step pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest_gpu_$TAG.log 2>&1 \
  || { tail -60 $OUT/pytest_gpu_$TAG.log; exit 1; }
tail -1 $OUT/pytest_gpu_$TAG.log
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 \
  || { tail -30 $OUT/smoke_$TAG.log; exit 1; }
tail -1 $OUT/smoke_$TAG.log
step bench 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_${TAG}.json 2> $OUT/bench_${TAG}.err \
  || { tail -30 $OUT/bench_${TAG}.err; exit 1; }
cut -c1-400 $OUT/bench_${TAG}.json
[ -n "$QUICK" ] && exit 0
step bench_cfg4 600 python bench.py --global-blocks 1000000 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_${TAG}_cfg4.json 2> $OUT/bench_${TAG}_cfg4.err \
  || { tail -30 $OUT/bench_${TAG}_cfg4.err; exit 1; }
cut -c1-400 $OUT/bench_${TAG}_cfg4.json
step bench_n2 600 env LSM_BENCH_REHEARSE=1 python bench.py --gpus 2 --steps 20 --warmup 5 > $OUT/bench_${TAG}_n2.json 2> $OUT/bench_${TAG}_n2.err \
  || { tail -30 $OUT/bench_${TAG}_n2.err; exit 1; }
cut -c1-400 $OUT/bench_${TAG}_n2.json
echo "== done"
