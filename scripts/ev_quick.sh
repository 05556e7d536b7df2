set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${T:-r06b}
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_stream_build_gpu.py} -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest.log 2>&1 || { tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
timeout -k 10 300 python bench.py --config sst --cpu-seconds 3 > gpurun_out/${T}_bench_sst.json 2> gpurun_out/${T}_bench_sst.err || { tail -20 gpurun_out/${T}_bench_sst.err; exit 1; }
cut -c1-1500 gpurun_out/${T}_bench_sst.json
CFG=sst TAG=$T bash scripts/gpu_quick.sh
