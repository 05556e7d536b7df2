# Ad-hoc GPU step: the listed test files, then bench lines ($LINES, default
# sst) and rocprofv3 kernel stats of the first ($PROF, default the same).
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${T:-r06x}
if [ -n "${TESTS-tests/test_stream_build_gpu.py}" ]; then
timeout -k 10 900 python -u -m pytest ${TESTS-tests/test_stream_build_gpu.py} -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest.log 2>&1 || { tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
fi
for L in ${LINES:-sst}; do
timeout -k 10 300 python bench.py --config $L --cpu-seconds ${CPUS:-3} > gpurun_out/${T}_bench_$L.json 2> gpurun_out/${T}_bench_$L.err || { tail -20 gpurun_out/${T}_bench_$L.err; exit 1; }
cut -c1-700 gpurun_out/${T}_bench_$L.json
done
for P in ${PROF-sst}; do
TESTS= LINES= CFG=$P TAG=$T bash scripts/gpu_quick.sh 2>/dev/null
done
