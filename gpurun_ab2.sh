set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_decode_gpu.py tests/test_encode_gpu.py -q -p no:cacheprovider > gpurun_out/pytest_dec.log 2>&1 || { tail -40 gpurun_out/pytest_dec.log; exit 1; }
tail -1 gpurun_out/pytest_dec.log
for B in 3 4 7; do
  LSM_LANE_BLOCKS=$B timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/ab_B$B.json 2>gpurun_out/ab_B$B.err || { tail gpurun_out/ab_B$B.err; exit 1; }
  python -c "import json;j=json.load(open('gpurun_out/ab_B$B.json'));print('B=$B', j['value'], j['roofline']['kernel_ms'], j['roofline']['frac'])"
done
