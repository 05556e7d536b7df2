export TMPDIR=/tmp
t() { v=$1; shift; timeout -k 10 200 python scripts/ab_pytest.py ab/$v.so "$@" -x -q --timeout 120 --timeout-method thread > gpurun_out/abt_$v.log 2>&1 || { tail -30 gpurun_out/abt_$v.log; exit 1; }; echo "$v tests: $(tail -1 gpurun_out/abt_$v.log)"; }
t rc2 tests/test_encode_gpu.py || exit 1
t rc8 tests/test_encode_gpu.py || exit 1
LINES="sst" VARIANTS="prod rc2 rc8" REPS=2 bash scripts/ab_pair.sh || exit 1
