set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for R in 1 2; do
for V in spec spec_w1 spec_w2; do
  LSM_DECODE_KERNEL=$V timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/ab_$V.json 2>gpurun_out/ab_$V.err || { tail gpurun_out/ab_$V.err; exit 1; }
  python -c "import json;j=json.load(open('gpurun_out/ab_$V.json'));print('$V', j['value'], j['roofline']['kernel_ms'], j['roofline']['frac'])"
done
done
LSM_DECODE_KERNEL=spec_w1 timeout -k 10 600 python -m pytest tests/test_decode_gpu.py -q -p no:cacheprovider -x > gpurun_out/pytest_w1.log 2>&1 || { echo "FAIL"; tail -40 gpurun_out/pytest_w1.log; exit 1; }
echo "w1 $(tail -1 gpurun_out/pytest_w1.log)"
