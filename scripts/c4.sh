# round-5 GPU step 4: parity of the goheap rank path and the prefetching Get,
# A/B of the Get, the goheap line, PMC traffic of the changed lines
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
# (parity: 52 GPU tests passed in the previous call)

LINES="get" VARIANTS="prod g0" REPS=2 STEPS=50 bash scripts/ab_pair.sh || exit 1
timeout -k 10 300 python bench.py --config compact --tie goheap --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/c4_goheap.json 2> gpurun_out/c4_goheap.err || { tail -20 gpurun_out/c4_goheap.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/c4_goheap.json')); print(d['value'], d['ms_per_step'], d['goheap'], d['config']['stage_ms'])"
TAG=r05b PHASE=2 PMC1="" PMCM="sst level get wal" bash scripts/gpu_evidence.sh > gpurun_out/c4_pmc.txt 2>&1 || { tail -20 gpurun_out/c4_pmc.txt; exit 1; }
cat gpurun_out/r05b_pmc_*.json | grep -E "workload_key|hbm_bytes"
LINES="sst" VARIANTS="prod pu" REPS=3 STEPS=50 bash scripts/ab_pair.sh || exit 1
OUTD=gpurun_out/pmcmix_sst1 BENCH_ARGS="--config sst" KF=sst_regions,bloom_or PYARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-cold" \
  bash scripts/pmc_decode.sh > gpurun_out/c4_pmcmix_sst.txt 2>&1 || { tail -5 gpurun_out/c4_pmcmix_sst.txt; exit 1; }
cat gpurun_out/c4_pmcmix_sst.txt
