set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for V in group64 group32 group16; do
  LSM_DECODE_KERNEL=$V timeout -k 10 600 python -m pytest tests/test_decode_gpu.py -q -p no:cacheprovider -x > gpurun_out/pytest_$V.log 2>&1 || { echo "FAIL $V"; tail -40 gpurun_out/pytest_$V.log; exit 1; }
  echo "$V $(tail -1 gpurun_out/pytest_$V.log)"
done
for V in spec group64 group32 group16; do
  LSM_DECODE_KERNEL=$V timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/ab_$V.json 2>gpurun_out/ab_$V.err || { tail gpurun_out/ab_$V.err; exit 1; }
  python -c "import json;j=json.load(open('gpurun_out/ab_$V.json'));print('$V', j['value'], j['roofline']['kernel_ms'], j['roofline']['frac'])"
done
