# Memory-path counters of one kernel of the compact bench (separate passes).
set -o pipefail
export TMPDIR=/tmp
K=${K:-gather_copy}
i=0
for grp in "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" "TA_DATA_STALLED_BY_TC_CYCLES_sum TA_FLAT_READ_WAVEFRONTS_sum" \
           "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmcg/p$i -o run -- python bench.py --config compact --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmcg/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmcg/p$i.log; exit 1; }
done
K=$K python - <<'PY'
import csv, glob, collections, os
for f in sorted(glob.glob("gpurun_out/pmcg/p*/**/*counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(float); cnt = collections.Counter()
    for r in csv.DictReader(open(f)):
        if os.environ["K"] not in r["Kernel_Name"]: continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"]); cnt[r["Counter_Name"]] += 1
    print({c: round(v / cnt[c], 0) for c, v in agg.items()})
PY
