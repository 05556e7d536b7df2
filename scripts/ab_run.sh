export TMPDIR=/tmp
t() { v=$1; shift; timeout -k 10 200 python scripts/ab_pytest.py ab/$v.so "$@" -x -q --timeout 120 --timeout-method thread > gpurun_out/abt_$v.log 2>&1 || { tail -30 gpurun_out/abt_$v.log; exit 1; }; echo "$v tests: $(tail -1 gpurun_out/abt_$v.log)"; }
t spin tests/test_merge_gpu.py || exit 1
LINES="compact" VARIANTS="prod spin" REPS=3 bash scripts/ab_pair.sh || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/pv_spin -o run -- python scripts/ab_lib.py ab/spin.so --config compact --steps 10 --warmup 3 > gpurun_out/pv_spin.log 2>&1 || exit 1
TAG=r04y PHASE=1 bash scripts/gpu_evidence.sh || exit 1
