# round-5 GPU step 12: IDX-only region writer LDS for the views build + the gather's dense value views: parity, A/B, kernel stats
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_merge_gpu.py tests/test_encode_gpu.py -m gpu -q -x --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/c12_pytest.log 2>&1 || { tail -40 gpurun_out/c12_pytest.log; exit 1; }
tail -1 gpurun_out/c12_pytest.log
for rep in 1 2 3; do
  for j in on off; do
    timeout -k 10 300 python bench.py --config compact --views $j --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/c12_$j.json 2> gpurun_out/c12_$j.err || { tail -20 gpurun_out/c12_$j.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/c12_$j.json')); print('$j', d['value'], d['ms_per_step'], d['config']['stage_ms'])"
  done
done
timeout -k 10 300 python bench.py --config sst --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/c12_sst.json 2> gpurun_out/c12_sst.err || { tail -20 gpurun_out/c12_sst.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/c12_sst.json')); print('sst', d['value'], d['ms_per_step'], d['roofline']['frac'])"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/c12prof -o compact -- python3 $GRAFT_REPO_ROOT/bench.py --config compact --steps 20 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/c12_prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/c12_prof.log; exit 1; }
for f in $(find $GRAFT_REPO_ROOT/gpurun_out/c12prof -name '*kernel_stats.csv'); do cut -c1-130 "$f" | head -24; done
