# Ad-hoc GPU step: test files ($TESTS), then A/B lines ($LINES) with the product library.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_quick.log 2>&1 || { tail -30 gpurun_out/pytest_quick.log; exit 1; }
tail -1 gpurun_out/pytest_quick.log
VARIANTS="${VARIANTS:-prod}" REPS=${REPS:-2} STEPS=${STEPS:-50} bash scripts/ab_pair.sh
