# round-5 GPU step 11: the region writer's data region straight from the values arena (no LDS staging): parity, then A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_encode_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/c11_pytest.log 2>&1 || { tail -40 gpurun_out/c11_pytest.log; exit 1; }
tail -1 gpurun_out/c11_pytest.log
for v in vd4 vd1w8; do
  timeout -k 10 600 python -u scripts/ab_pytest.py ab/$v.so tests/test_encode_gpu.py -m gpu -q -x -k sst --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/c11_pytest_$v.log 2>&1 || { tail -40 gpurun_out/c11_pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/c11_pytest_$v.log)"
done
LINES="sst compact" VARIANTS="old prod vd4 vd1w8" REPS=3 STEPS=50 bash scripts/ab_pair.sh || exit 1
