set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for c in decode4k sst; do
timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > gpurun_out/bench_$c.json 2>gpurun_out/bench_$c.err || { tail gpurun_out/bench_$c.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_$c.json'));print('$c', d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'])"
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sst -o run -- python bench.py --config sst --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_sst.log 2>&1 && \
cut -c1-150 gpurun_out/prof_sst/run_kernel_stats.csv | head -6
