# round-5 GPU step 6: WAL variants (records kept in registers; 16 KiB LDS per segment) -- parity, then A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in walrec wal10; do
  timeout -k 10 300 python scripts/ab_pytest.py ab/$v.so tests/test_wal_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/c6_t_$v.log 2>&1 || { tail -30 gpurun_out/c6_t_$v.log; exit 1; }
  echo "$v tests: $(tail -1 gpurun_out/c6_t_$v.log)"
done
LINES="wal" VARIANTS="prod walrec wal10" REPS=3 STEPS=100 bash scripts/ab_pair.sh || exit 1
