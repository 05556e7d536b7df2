# round-5 GPU step 7: the one-call join + merge (statistics beside the join): parity, then A/B against the two calls
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_merge_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/c7_pytest.log 2>&1 || { tail -40 gpurun_out/c7_pytest.log; exit 1; }
tail -1 gpurun_out/c7_pytest.log
for rep in 1 2 3; do
  for j in fused separate; do
    timeout -k 10 300 python bench.py --config compact --join $j --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/c7_$j.json 2> gpurun_out/c7_$j.err || { tail -20 gpurun_out/c7_$j.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/c7_$j.json')); print('$j', d['value'], d['ms_per_step'], d['config']['stage_ms'])"
  done
done
