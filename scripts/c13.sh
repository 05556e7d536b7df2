# round-5 GPU step 13: occupancy targets (amdgpu_waves_per_eu) for the data-region copy, the IDX-only region writer and the Get kernel: parity, A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in occ8 getw8; do
  timeout -k 10 900 python -u scripts/ab_pytest.py ab/$v.so tests/test_merge_gpu.py tests/test_level_get_gpu.py -m gpu -q -x -k "build or views or get" --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/c13_pytest_$v.log 2>&1 || { tail -40 gpurun_out/c13_pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/c13_pytest_$v.log)"
done
LINES="compact" VARIANTS="prod occ8 occ8v" REPS=3 STEPS=20 bash scripts/ab_pair.sh || exit 1
LINES="get" VARIANTS="prod getw8" REPS=3 STEPS=50 bash scripts/ab_pair.sh || exit 1
