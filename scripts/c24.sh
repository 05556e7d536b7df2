# round-5 GPU step 24: WAL segment kernel's scratch entries collected in LDS and stored by 16-byte rows (walent512 / walent256): parity, A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in walent512 walent256; do
  timeout -k 10 600 python -u scripts/ab_pytest.py ab/$v.so tests/test_wal_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/c24_pytest_$v.log 2>&1 || { tail -40 gpurun_out/c24_pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/c24_pytest_$v.log)"
done
LINES="wal" VARIANTS="prod walent512 walent256" REPS=3 STEPS=100 bash scripts/ab_pair.sh || exit 1
