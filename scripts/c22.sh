# round-5 GPU step 22: the level search's filter test by slices (two 100 KiB halves per table, nothing read past LDS, may cleared by either): parity, A/B, traffic, kernel stats
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_level_search_gpu.py tests/test_level_get_gpu.py tests/test_may_contain_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/c22_pytest.log 2>&1 || { tail -40 gpurun_out/c22_pytest.log; exit 1; }
tail -1 gpurun_out/c22_pytest.log
LINES="level get" VARIANTS="old prod" REPS=3 STEPS=100 bash scripts/ab_pair.sh || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/c22pmc_$c -o run -- python bench.py --config level --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/c22pmc_$c.log 2>&1 || { tail -5 gpurun_out/c22pmc_$c.log; exit 1; }
done
python scripts/pmc_multi.py gpurun_out/c22pmc_FETCH_SIZE gpurun_out/c22pmc_WRITE_SIZE lv_classify_kernel,lv_test_kernel lv_classify_kernel level:208:1048576 gpurun_out/c22pmc_level.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/c22prof -o level -- python3 $GRAFT_REPO_ROOT/bench.py --config level --steps 50 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/c22_prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/c22_prof.log; exit 1; }
for f in $(find $GRAFT_REPO_ROOT/gpurun_out/c22prof -name '*kernel_stats.csv'); do cut -c1-110 "$f" | head -5; done
