# round-5 GPU step 9: the blocked Seek tree: parity (with, without, partial), then A/B and kernel stats
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_level_get_gpu.py tests/test_abi.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/c9_pytest.log 2>&1 || { tail -40 gpurun_out/c9_pytest.log; exit 1; }
tail -1 gpurun_out/c9_pytest.log
for rep in 1 2 3; do
  for j in on off; do
    timeout -k 10 300 python bench.py --config get --get-tree $j --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/c9_$j.json 2> gpurun_out/c9_$j.err || { tail -20 gpurun_out/c9_$j.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/c9_$j.json')); r=d['roofline']; print('$j', d['value'], d['ms_per_step'], r['achieved'], r['frac'], d['config'].get('seek_tree'))"
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/c9prof -o get -- python3 $GRAFT_REPO_ROOT/bench.py --config get --steps 50 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/c9_prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/c9_prof.log; exit 1; }
for f in $(find $GRAFT_REPO_ROOT/gpurun_out/c9prof -name '*kernel_stats.csv'); do cut -c1-160 "$f"; done
