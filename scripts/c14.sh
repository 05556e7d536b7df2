# round-5 GPU step 14: the split .sst build in file groups (each group's ORs beside the next groups' regions): parity, A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in og2 og4; do
  timeout -k 10 600 python -u scripts/ab_pytest.py ab/$v.so tests/test_encode_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/c14_pytest_$v.log 2>&1 || { tail -40 gpurun_out/c14_pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/c14_pytest_$v.log)"
done
LINES="sst" VARIANTS="prod og2 og4" REPS=3 STEPS=50 bash scripts/ab_pair.sh || exit 1
