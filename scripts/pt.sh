set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_stream_build_gpu.py tests/test_merge_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06d_pytest.log 2>&1 || { tail -30 gpurun_out/r06d_pytest.log; exit 1; }
tail -1 gpurun_out/r06d_pytest.log
for i in 1 2; do timeout -k 10 300 python scripts/ab_lib.py go-lsm_amd/liblsm_gpu.so --config sst --steps 200 | python3 -c "import json,sys; j=json.load(sys.stdin); print(j['value'], j['ms_per_step'], j['roofline']['kernel_ms'], j['roofline']['frac'])"; done
TESTS= LINES= CFG=sst TAG=r06d bash scripts/gpu_quick.sh > /dev/null 2>&1; python3 scripts/kstats.py gpurun_out/prof_r06d_sst/run_kernel_stats.csv 63 2>/dev/null | grep -i "plan\|regions\|bloom_or"
timeout -k 10 300 python bench.py --config compact --tie goheap --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r06d_bench_goheap.json 2> gpurun_out/r06d_goheap.err || { tail -5 gpurun_out/r06d_goheap.err; exit 1; }
python3 -c "import json; j=json.load(open('gpurun_out/r06d_bench_goheap.json')); print(j['ms_per_step'], j.get('goheap'))"
