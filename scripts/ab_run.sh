export TMPDIR=/tmp
t() { v=$1; shift; timeout -k 10 200 python scripts/ab_pytest.py ab/$v.so "$@" -x -q --timeout 120 --timeout-method thread > gpurun_out/abt_$v.log 2>&1 || { tail -30 gpurun_out/abt_$v.log; exit 1; }; echo "$v tests: $(tail -1 gpurun_out/abt_$v.log)"; }
timeout -k 10 300 python -u -m pytest tests/test_merge_gpu.py tests/test_encode_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_merge.log 2>&1 || { tail -30 gpurun_out/pt_merge.log; exit 1; }
echo "prod tests: $(tail -1 gpurun_out/pt_merge.log)"
t ixplain tests/test_sst_decode_gpu.py tests/test_merge_gpu.py || exit 1
LINES="compact" VARIANTS="base prod ixplain" REPS=3 bash scripts/ab_pair.sh || exit 1
LINES="sstdec" VARIANTS="prod ixplain" REPS=2 bash scripts/ab_pair.sh || exit 1
