export TMPDIR=/tmp
t() { v=$1; shift; timeout -k 10 200 python scripts/ab_pytest.py ab/$v.so "$@" -x -q --timeout 120 --timeout-method thread > gpurun_out/abt_$v.log 2>&1 || { tail -30 gpurun_out/abt_$v.log; exit 1; }; echo "$v tests: $(tail -1 gpurun_out/abt_$v.log)"; }
t vs2 tests/test_merge_gpu.py tests/test_encode_gpu.py || exit 1
t vs4 tests/test_merge_gpu.py || exit 1
LINES="compact" VARIANTS="prod vs2 vs4" REPS=3 bash scripts/ab_pair.sh || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/pv_vs2 -o run -- python scripts/ab_lib.py ab/vs2.so --config compact --steps 10 --warmup 3 > gpurun_out/pv_vs2.log 2>&1 || exit 1
