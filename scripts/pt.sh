set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_level_get_gpu.py tests/test_level_search_gpu.py tests/test_level0_get_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06e_pytest.log 2>&1 || { tail -30 gpurun_out/r06e_pytest.log; exit 1; }
tail -1 gpurun_out/r06e_pytest.log
for i in 1 2; do timeout -k 10 300 python scripts/ab_lib.py go-lsm_amd/liblsm_gpu.so --config get --steps 200 | python3 -c "import json,sys; j=json.load(sys.stdin); print(j['value'], j['ms_per_step'], j['roofline']['kernel_ms'], j['roofline']['frac'])"; done
TESTS= LINES= CFG=get TAG=r06e bash scripts/gpu_quick.sh > /dev/null 2>&1; python3 scripts/kstats.py gpurun_out/prof_r06e_get/run_kernel_stats.csv 63 2>/dev/null | grep -i "lv_\|level"
