# round-5 GPU step: parity of the changed paths, A/B of the encode and level variants, new lines
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_encode_gpu.py tests/test_mirror.py tests/test_level_search_gpu.py tests/test_level_get_gpu.py tests/test_may_contain_gpu.py tests/test_merge_gpu.py tests/test_wal_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/c3_pytest.log 2>&1 || { tail -40 gpurun_out/c3_pytest.log; exit 1; }
tail -1 gpurun_out/c3_pytest.log
LINES="sst" VARIANTS="prod rc2" REPS=3 STEPS=50 bash scripts/ab_pair.sh || exit 1
LINES="level" VARIANTS="prod lv32" REPS=3 STEPS=50 bash scripts/ab_pair.sh || exit 1
LINES="wal" VARIANTS="prod w16" REPS=3 STEPS=50 bash scripts/ab_pair.sh || exit 1
LINES="compact" VARIANTS="prod vrp4 vrp8" REPS=2 STEPS=20 bash scripts/ab_pair.sh || exit 1
timeout -k 10 300 python bench.py --config get --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/c3_get.json 2> gpurun_out/c3_get.err || { tail -20 gpurun_out/c3_get.err; exit 1; }
cut -c1-400 gpurun_out/c3_get.json
timeout -k 10 300 python bench.py --config compact --tie goheap --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/c3_goheap.json 2> gpurun_out/c3_goheap.err || { tail -20 gpurun_out/c3_goheap.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/c3_goheap.json')); print(d['value'], d['ms_per_step'], d['goheap'], d['config']['stage_ms'])"
# instruction-mix / wait counters of the kernels the verdict names (one pass per group)
for spec in "wal:wal_seg,wal_compact" "level:lv_classify,lv_test" "decode64k:decode_v2" "compact:sst_vregion_runs,bloom_or,sst_regions"; do
  cfg=${spec%%:*}; kf=${spec#*:}
  OUTD=gpurun_out/pmcmix_$cfg BENCH_ARGS="--config $cfg" KF=$kf PYARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-cold" \
    bash scripts/pmc_decode.sh > gpurun_out/c3_pmcmix_$cfg.txt 2>&1 || { tail -5 gpurun_out/c3_pmcmix_$cfg.txt; exit 1; }
  echo "== $cfg"; cat gpurun_out/c3_pmcmix_$cfg.txt
done
