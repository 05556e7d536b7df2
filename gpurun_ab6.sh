set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_decode_gpu.py -q -p no:cacheprovider -x > gpurun_out/pytest_pipe.log 2>&1 || { echo "FAIL pipe"; tail -40 gpurun_out/pytest_pipe.log; exit 1; }
echo "pipe $(tail -1 gpurun_out/pytest_pipe.log)"
for V in pipe spec; do
  LSM_DECODE_KERNEL=$V timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/ab_$V.json 2>gpurun_out/ab_$V.err || { tail gpurun_out/ab_$V.err; exit 1; }
  python -c "import json;j=json.load(open('gpurun_out/ab_$V.json'));print('$V', j['value'], j['roofline']['kernel_ms'], j['roofline']['frac'])"
done
timeout -k 10 300 python bench.py --config decode64k --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/ab_64k.json 2>gpurun_out/ab_64k.err || { tail gpurun_out/ab_64k.err; exit 1; }
python -c "import json;j=json.load(open('gpurun_out/ab_64k.json'));print('64k', j['value'], j['roofline']['kernel_ms'], j['roofline']['frac'])"
