set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_decode_gpu.py -q -p no:cacheprovider -x > gpurun_out/pytest_dec.log 2>&1 || { tail -60 gpurun_out/pytest_dec.log; exit 1; }
tail -1 gpurun_out/pytest_dec.log
for V in spec spec1 spec2 spec8 spec16; do
  LSM_DECODE_KERNEL=$V timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/ab_$V.json 2>gpurun_out/ab_$V.err || { tail gpurun_out/ab_$V.err; exit 1; }
  python -c "import json;j=json.load(open('gpurun_out/ab_$V.json'));print('$V', j['value'], j['roofline']['kernel_ms'], j['roofline']['frac'])"
done
for C in decode64k; do
  timeout -k 10 300 python bench.py --config $C --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/ab_$C.json 2>gpurun_out/ab_$C.err || { tail gpurun_out/ab_$C.err; exit 1; }
  python -c "import json;j=json.load(open('gpurun_out/ab_$C.json'));print('$C', j['value'], j['roofline']['kernel_ms'], j['roofline']['frac'])"
done
timeout -k 10 600 python bench.py --config mixed --blocks 268435456 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_mixed.json 2>gpurun_out/ab_mixed.err || { tail gpurun_out/ab_mixed.err; exit 1; }
python -c "import json;j=json.load(open('gpurun_out/ab_mixed.json'));print('mixed', j['value'], j['roofline']['kernel_ms'], j['roofline']['frac'], j['config']['records_per_gpu'])"
