# round-5 GPU step 18: WAL write-phase ablations (timing-only diagnostic libraries, their output is wrong by design) and the streaming filter staging (lvnt): parity, A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in waltnr waltns; do
  timeout -k 10 300 python scripts/ab_lib.py ab/$v.so --config wal --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c18_$v.out 2> gpurun_out/c18_$v.err
  echo "$v rc=$?"; grep WALT gpurun_out/c18_$v.out | tail -3 || true
done
timeout -k 10 600 python -u scripts/ab_pytest.py ab/lvnt.so tests/test_level_search_gpu.py tests/test_may_contain_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/c18_pytest_lvnt.log 2>&1 || { tail -40 gpurun_out/c18_pytest_lvnt.log; exit 1; }
echo "lvnt: $(tail -1 gpurun_out/c18_pytest_lvnt.log)"
LINES="level probe" VARIANTS="prod lvnt" REPS=3 STEPS=100 bash scripts/ab_pair.sh || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/c18pmc_lvnt_$c -o run -- python scripts/ab_lib.py ab/lvnt.so --config level --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/c18pmc_$c.log 2>&1 || { tail -5 gpurun_out/c18pmc_$c.log; exit 1; }
done
python scripts/pmc_multi.py gpurun_out/c18pmc_lvnt_FETCH_SIZE gpurun_out/c18pmc_lvnt_WRITE_SIZE lv_classify_kernel,lv_test_kernel lv_classify_kernel level:208:1048576 gpurun_out/c18pmc_lvnt.json
