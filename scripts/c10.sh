# round-5 GPU step 10: bloom_or_kernel with both slices of a filter on one XCD (orpair): parity, A/B, HBM traffic
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/ab_pytest.py ab/orpair.so tests/test_encode_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/c10_pytest.log 2>&1 || { tail -40 gpurun_out/c10_pytest.log; exit 1; }
tail -1 gpurun_out/c10_pytest.log
LINES=sst VARIANTS="prod orpair" REPS=3 STEPS=50 bash scripts/ab_pair.sh || exit 1
for v in prod orpair; do
  lib=ab/$v.so; [ $v = prod ] && lib=go-lsm_amd/liblsm_gpu.so
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/c10pmc_${v}_$c -o run -- python scripts/ab_lib.py $lib --config sst --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/c10pmc_${v}_$c.log 2>&1 || { tail -5 gpurun_out/c10pmc_${v}_$c.log; exit 1; }
  done
  python scripts/pmc_multi.py gpurun_out/c10pmc_${v}_FETCH_SIZE gpurun_out/c10pmc_${v}_WRITE_SIZE sst_regions_kernel,bloom_or_kernel,sst_meta_kernel sst_regions_kernel sst:208 gpurun_out/c10pmc_$v.json > /dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/c10pmc_$v.json')); print('$v', {k: d[k] for k in d if not isinstance(d[k], (dict, list))})"
done
