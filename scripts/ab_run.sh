export TMPDIR=/tmp
t() { v=$1; shift; timeout -k 10 200 python scripts/ab_pytest.py ab/$v.so "$@" -x -q --timeout 120 --timeout-method thread > gpurun_out/abt_$v.log 2>&1 || { tail -30 gpurun_out/abt_$v.log; exit 1; }; echo "$v tests: $(tail -1 gpurun_out/abt_$v.log)"; }
t fx tests/test_sst_decode_gpu.py tests/test_merge_gpu.py || exit 1
t vrpb tests/test_merge_gpu.py tests/test_encode_gpu.py || exit 1
t or3 tests/test_encode_gpu.py || exit 1
LINES="sstdec compact" VARIANTS="prod fx" REPS=2 bash scripts/ab_pair.sh || exit 1
LINES="compact" VARIANTS="prod vrpb vrnochk" REPS=2 bash scripts/ab_pair.sh || exit 1
LINES="sst" VARIANTS="prod or3" REPS=2 bash scripts/ab_pair.sh || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/pv_or3 -o run -- python scripts/ab_lib.py ab/or3.so --config sst --steps 10 --warmup 3 > gpurun_out/pv_or3.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/pv_fx -o run -- python scripts/ab_lib.py ab/fx.so --config sstdec --steps 10 --warmup 3 > gpurun_out/pv_fx.log 2>&1 || exit 1
