# round-5 GPU step 20: the compaction's key copy inside the build, beside its data-region copy (gather offsets first): parity, A/B, trace
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_merge_gpu.py -m gpu -q -x --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/c20_pytest.log 2>&1 || { tail -40 gpurun_out/c20_pytest.log; exit 1; }
tail -1 gpurun_out/c20_pytest.log
timeout -k 10 900 python -u scripts/ab_pytest.py ab/vmain.so tests/test_merge_gpu.py -m gpu -q -x -k "build" --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/c20_pytest_vmain.log 2>&1 || { tail -40 gpurun_out/c20_pytest_vmain.log; exit 1; }
echo "vmain: $(tail -1 gpurun_out/c20_pytest_vmain.log)"
for rep in 1 2 3; do
  for j in build gather; do
    timeout -k 10 300 python bench.py --config compact --gather-keys $j --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/c20_$j.json 2> gpurun_out/c20_$j.err || { tail -20 gpurun_out/c20_$j.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/c20_$j.json')); print('$j', d['value'], d['ms_per_step'], d['config']['stage_ms'])"
  done
  timeout -k 10 300 python scripts/ab_lib.py ab/vmain.so --config compact --gather-keys build --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/c20_vmain.json 2> gpurun_out/c20_vmain.err || { tail -20 gpurun_out/c20_vmain.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/c20_vmain.json')); print('vmain', d['value'], d['ms_per_step'], d['config']['stage_ms'])"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/c20prof -o compact -- python3 $GRAFT_REPO_ROOT/bench.py --config compact --steps 20 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/c20_prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/c20_prof.log; exit 1; }
echo prof ok
