# PMC passes (one per counter group) over one decode config: instruction mix and waits.
set -o pipefail
export TMPDIR=/tmp
CFG=${CFG:-mixed}
KF=${KF:-decode}
OUTD=${OUTD:-gpurun_out/pmcd}; mkdir -p $OUTD
i=0
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS"
G2="SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
# LDS groups (set PMC_LDS=1): array cycles, conflict kinds
G3="SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES"
set -- "$G1" "$G2"
[ -n "$PMC_LDS" ] && set -- "$G1" "$G2" "$G3"
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUTD/p$i -o run -- python ${PYCMD:-bench.py} ${BENCH_ARGS:---config $CFG} ${PYARGS:---steps 3 --warmup 1 --no-cpu-baseline} > $OUTD/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUTD/p$i.log; exit 1; }
done
OUTD=$OUTD KF=$KF python - <<'PY'
import csv, glob, collections, os
for f in sorted(glob.glob(os.environ["OUTD"] + "/p*/**/*counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:60]
        if not any(x in k for x in os.environ.get("KF", "decode").split(",")): continue
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[(k, r["Counter_Name"])] += 1
    for k, d in agg.items():
        print(k, {c: round(v / cnt[(k, c)], 0) for c, v in d.items()})
PY
