#!/bin/bash
# Round evidence: parity suite, smoke, HBM traffic (PMC, one counter per
# pass) written into profiles/ before the bench lines read it, every bench
# line, and rocprofv3 kernel stats.  Everything lands in gpurun_out/ (the
# PMC summaries also as gpurun_out/<tag>_pmc_*.json, to be committed under
# profiles/).  Each GPU step has its own limit; the chain stops at the first
# failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; TAG=${TAG:-r03}
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)" >&2; timeout -k 10 $lim "$@"; }
PHASE=${PHASE:-all}  # all, or a list of phases: "1 2"
has() { [ "$PHASE" = all ] || [[ " $PHASE " == *" $1 "* ]]; }
if has 1; then
step pytest 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu_$TAG.log 2>&1 \
  || { tail -60 $OUT/pytest_gpu_$TAG.log; exit 1; }
tail -1 $OUT/pytest_gpu_$TAG.log
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 \
  || { tail -30 $OUT/smoke_$TAG.log; exit 1; }
tail -1 $OUT/smoke_$TAG.log
fi
if has 2; then
# single-kernel decode lines: FETCH_SIZE x2 + WRITE_SIZE of decode_v2_kernel
declare -A DA DK
DA[desc]="--config decode4k"; DK[desc]=decode4k:100000:desc
DA[arena]="--config decode4k --arena"; DK[arena]=decode4k:100000:arena
DA[d64]="--config decode64k"; DK[d64]=decode64k:6400:desc
for t in ${PMC1-desc arena d64}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    step pmc_${t}_$c 180 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_${TAG}_${t}_$c -o run \
      -- python bench.py ${DA[$t]} --steps 5 --warmup 2 --no-cpu-baseline --no-cold > $OUT/pmc_${TAG}_${t}_$c.log 2>&1 || exit 1
  done
  python scripts/pmc_summary.py $OUT/pmc_${TAG}_${t}_FETCH_SIZE $OUT/pmc_${TAG}_${t}_WRITE_SIZE decode_v2_kernel \
    ${DK[$t]} $OUT/${TAG}_pmc_$t.json > /dev/null && cp $OUT/${TAG}_pmc_$t.json profiles/ || exit 1
done
# multi-launch lines
declare -A K A W
K[sst]=sst_stream_plan_kernel,sst_regions_kernel,bloom_or_kernel,bloom_file_kernel,sst_meta_kernel; A[sst]=sst_regions_kernel; W[sst]=sst:208
K[get0]=level0_get_kernel; A[get0]=level0_get_kernel; W[get0]=get0:3:1048576
K[compact]=sst_index_kernel,sst_tail_kernel,sst_pairs,merge_,goheap,rocprim,gather_,sst_layout,sst_regions_kernel,sst_vregion,bloom_or_kernel,sst_meta; A[compact]=sst_index_kernel; W[compact]=compact:216
K[mixed]=sched_hist_kernel,sched_scatter_kernel,decode_v2_kernel; A[mixed]=decode_v2_kernel; W[mixed]=mixed:37450:desc
K[sstdec]=sst_index_kernel,sst_tail_kernel; A[sstdec]=sst_tail_kernel; W[sstdec]=sstdec:208
K[probe]=mc_prep_kernel,mc_classify_kernel,lv_test_kernel,may_contain_kernel; A[probe]=mc_prep_kernel; W[probe]=probe:208:1048576
K[wal]=wal_seg_lanes_kernel,wal_stitch_kernel,wal_compact_kernel; A[wal]=wal_stitch_kernel; W[wal]=wal:64:desc
K[level]=lv_classify_kernel,lv_test_kernel; A[level]=lv_classify_kernel; W[level]=level:208:1048576
K[get]=lv_classify_kernel,lv_test_kernel,level_get_kernel; A[get]=lv_classify_kernel; W[get]=get:208:1048576
for cfg in ${PMCM-sst sstdec probe wal}; do
  SK=0; [ $cfg = compact ] && SK=1  # the input images' decode before the steps
  for c in FETCH_SIZE WRITE_SIZE; do
    step pmcm_${cfg}_$c 180 rocprofv3 --pmc $c --output-format csv -d $OUT/pmcm_${TAG}_${cfg}_$c -o run \
      -- python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-cold > $OUT/pmcm_${TAG}_${cfg}_$c.log 2>&1 || exit 1
  done
  SKIP_ANCHORS=$SK python scripts/pmc_multi.py $OUT/pmcm_${TAG}_${cfg}_FETCH_SIZE $OUT/pmcm_${TAG}_${cfg}_WRITE_SIZE "${K[$cfg]}" "${A[$cfg]}" "${W[$cfg]}" \
    profiles/${TAG}_pmc_$cfg.json $OUT/${TAG}_pmc_$cfg.json > /dev/null || exit 1
done
fi
if has 3; then
for line in ${LINES:-decode4k cfg4 decode64k mixed arena sst sstdec sstdec1 wal probe level get get0 compact goheap e2e}; do
  case $line in
    cfg4) args="--global-blocks 1000000 --no-cpu-baseline" ;;
    arena) args="--arena" ;;
    e2e) args="--e2e" ;;
    goheap) args="--config compact --tie goheap --steps 5 --warmup 1" ;;
    *) args="--config $line" ;;
  esac
  step bench_$line 600 python bench.py $args > $OUT/bench_${TAG}_$line.json 2> $OUT/bench_${TAG}_$line.err \
    || { tail -20 $OUT/bench_${TAG}_$line.err; exit 1; }
  cut -c1-200 $OUT/bench_${TAG}_$line.json
done
for p in ${PROF:-decode4k arena decode64k mixed sst sstdec probe level get get0 wal compact}; do
  case $p in arena) args="--arena" ;; *) args="--config $p" ;; esac
  step prof_$p 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_${TAG}_$p -o run \
    -- python bench.py $args --steps 20 --warmup 3 --no-cpu-baseline --no-cold > $OUT/prof_${TAG}_$p.log 2>&1 || exit 1
done
fi
echo "== done $(date +%T)"
