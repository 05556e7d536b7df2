# round-5 GPU step 16: the split .sst build in file groups (two unequal groups: 85/15 and 93/7 of the files): parity, A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in og85 og93; do
  timeout -k 10 600 python -u scripts/ab_pytest.py ab/$v.so tests/test_encode_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/c16_pytest_$v.log 2>&1 || { tail -40 gpurun_out/c16_pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/c16_pytest_$v.log)"
done
LINES="sst" VARIANTS="prod og85 og93" REPS=3 STEPS=50 bash scripts/ab_pair.sh || exit 1
