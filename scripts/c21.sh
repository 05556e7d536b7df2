# round-5 GPU step 21: in-build key copy queued before the data-region copy (kfirst): parity, A/B against the gather's copy
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u scripts/ab_pytest.py ab/kfirst.so tests/test_merge_gpu.py -m gpu -q -x -k "build" --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/c21_pytest.log 2>&1 || { tail -40 gpurun_out/c21_pytest.log; exit 1; }
echo "kfirst: $(tail -1 gpurun_out/c21_pytest.log)"
for rep in 1 2 3; do
  for j in build gather; do
    timeout -k 10 300 python scripts/ab_lib.py ab/kfirst.so --config compact --gather-keys $j --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/c21_$j.json 2> gpurun_out/c21_$j.err || { tail -20 gpurun_out/c21_$j.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/c21_$j.json')); print('$j', d['value'], d['ms_per_step'], d['config']['stage_ms'])"
  done
done
# and the WAL scratch entries by non-temporal stores (walnt)
timeout -k 10 600 python -u scripts/ab_pytest.py ab/walnt.so tests/test_wal_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/c21_pytest_walnt.log 2>&1 || { tail -40 gpurun_out/c21_pytest_walnt.log; exit 1; }
echo "walnt: $(tail -1 gpurun_out/c21_pytest_walnt.log)"
LINES="wal" VARIANTS="prod walnt" REPS=3 STEPS=100 bash scripts/ab_pair.sh || exit 1
