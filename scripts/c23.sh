# round-5 GPU step 23: merge statistics with the next pair's descriptors prefetched: parity, A/B, kernel stats
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_merge_gpu.py -m gpu -q -x --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/c23_pytest.log 2>&1 || { tail -40 gpurun_out/c23_pytest.log; exit 1; }
tail -1 gpurun_out/c23_pytest.log
LINES="compact" VARIANTS="old prod" REPS=4 STEPS=20 bash scripts/ab_pair.sh || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/c23prof -o compact -- python3 $GRAFT_REPO_ROOT/bench.py --config compact --steps 20 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/c23_prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/c23_prof.log; exit 1; }
grep -h merge_stats $(find $GRAFT_REPO_ROOT/gpurun_out/c23prof -name '*kernel_stats.csv') | cut -c1-160
