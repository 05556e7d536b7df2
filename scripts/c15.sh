# round-5 GPU step 15: merge flags with the predecessor key by shuffle, windowed run ranks: parity, A/B, kernel stats
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_merge_gpu.py tests/test_mirror.py -m gpu -q -x --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/c15_pytest.log 2>&1 || { tail -40 gpurun_out/c15_pytest.log; exit 1; }
tail -1 gpurun_out/c15_pytest.log
LINES="compact" VARIANTS="old prod" REPS=3 STEPS=20 bash scripts/ab_pair.sh || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/c15prof -o compact -- python3 $GRAFT_REPO_ROOT/bench.py --config compact --steps 20 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/c15_prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/c15_prof.log; exit 1; }
echo prof ok
