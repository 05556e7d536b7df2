# Ad-hoc GPU step (one gpurun call): optional test files ($TESTS), then
# either A/B lines ($LINES, scripts/ab_pair.sh with $VARIANTS, default the
# product library) or rocprofv3 kernel stats of one bench line ($CFG).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03x}
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_quick.log 2>&1 \
    || { tail -30 gpurun_out/pytest_quick.log; exit 1; }
  tail -1 gpurun_out/pytest_quick.log
fi
if [ -n "$LINES" ]; then
  VARIANTS="${VARIANTS:-prod}" REPS=${REPS:-2} STEPS=${STEPS:-50} bash scripts/ab_pair.sh || exit 1
fi
if [ -n "$CFG" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_$CFG -o run \
    -- python bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline --no-cold > gpurun_out/prof_${TAG}_$CFG.log 2>&1 \
    || { tail -20 gpurun_out/prof_${TAG}_$CFG.log; exit 1; }
  python scripts/kstats.py gpurun_out/prof_${TAG}_$CFG/run_kernel_stats.csv 63 | head -12 || true
fi
