# round-5 GPU step 19: WAL scratch entries by rows (coalesced), compact re-orders through LDS; level-search classify stages its slots in LDS (coalesced stores): parity, A/B, kernel stats, traffic
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_wal_gpu.py tests/test_level_search_gpu.py tests/test_level_get_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/c19_pytest.log 2>&1 || { tail -40 gpurun_out/c19_pytest.log; exit 1; }
tail -1 gpurun_out/c19_pytest.log
LINES="wal level" VARIANTS="old prod" REPS=3 STEPS=100 bash scripts/ab_pair.sh || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/c19pmc_$c -o run -- python bench.py --config wal --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/c19pmc_$c.log 2>&1 || { tail -5 gpurun_out/c19pmc_$c.log; exit 1; }
done
python scripts/pmc_multi.py gpurun_out/c19pmc_FETCH_SIZE gpurun_out/c19pmc_WRITE_SIZE wal_seg_lanes_kernel,wal_stitch_kernel,wal_compact_kernel wal_stitch_kernel wal:64:desc gpurun_out/c19pmc_wal.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/c19prof -o wal -- python3 $GRAFT_REPO_ROOT/bench.py --config wal --steps 50 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/c19_prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/c19_prof.log; exit 1; }
for f in $(find $GRAFT_REPO_ROOT/gpurun_out/c19prof -name '*kernel_stats.csv'); do cut -c1-120 "$f" | head -5; done
