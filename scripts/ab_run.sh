export TMPDIR=/tmp
t() { v=$1; shift; timeout -k 10 200 python scripts/ab_pytest.py ab/$v.so "$@" -x -q --timeout 120 --timeout-method thread > gpurun_out/abt_$v.log 2>&1 || { tail -30 gpurun_out/abt_$v.log; exit 1; }; echo "$v tests: $(tail -1 gpurun_out/abt_$v.log)"; }
TAG=r04x PHASE=1 bash scripts/gpu_evidence.sh || exit 1
t lvp1 tests/test_level_search_gpu.py || exit 1
t mcp1 tests/test_may_contain_gpu.py || exit 1
LINES="level probe" VARIANTS="prod lvp1 mcp1" REPS=2 bash scripts/ab_pair.sh || exit 1
TAG=r04x PHASE=3 LINES="sstdec sstdec1 compact" PROF="sstdec compact" bash scripts/gpu_evidence.sh || exit 1
