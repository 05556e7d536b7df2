# Ad-hoc GPU step: optional test files (TESTS), then kernel stats of one bench line (CFG).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-compact}; TAG=${TAG:-r03b}
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_quick.log 2>&1 \
    || { tail -40 gpurun_out/pytest_quick.log; exit 1; }
  tail -1 gpurun_out/pytest_quick.log
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_$CFG -o run \
  -- python bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline --no-cold > gpurun_out/prof_${TAG}_$CFG.log 2>&1 \
  || { tail -20 gpurun_out/prof_${TAG}_$CFG.log; exit 1; }
cut -c1-300 gpurun_out/prof_${TAG}_$CFG.log | tail -2
