set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for v in ${VARIANTS:-spec spec_w1 spec_w2 pipe spec2 group64 stream32x32 lanes}; do
LSM_DECODE_KERNEL=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 300 > gpurun_out/ab_$v.json 2>gpurun_out/ab_$v.err || { tail gpurun_out/ab_$v.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print('$v', d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'])"
done
for c in ${CONFIGS:-sst}; do
timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > gpurun_out/ab_$c.json 2>gpurun_out/ab_$c.err || { tail gpurun_out/ab_$c.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/ab_$c.json'));print('$c', d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'])"
done
