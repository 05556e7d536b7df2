#!/bin/bash
# HBM traffic (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, one counter per pass)
# for the multi-launch secondary bench lines, summed per call by
# pmc_multi.py into profiles/ (read by the benches) and gpurun_out/, then the
# bench lines again so they carry roofline.traffic.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out; TAG=${TAG:-r01}
mkdir -p $OUT
declare -A K A W
K[sst]=sst_regions_kernel,bloom_file_kernel,sst_meta_kernel;                  A[sst]=sst_regions_kernel; W[sst]=sst:208
K[sstdec]=sst_index_kernel,sst_index_fixup_kernel,sst_data_verify_kernel,sst_data_fixup_kernel; A[sstdec]=sst_index_fixup_kernel; W[sstdec]=sstdec:208
K[probe]=mc_prep_kernel,mc_classify_kernel,mc_offsets_kernel,mc_scatter_kernel,mc_test_kernel,may_contain_kernel; A[probe]=mc_prep_kernel; W[probe]=probe:208:1048576
K[wal]=wal_seg_lanes_kernel,wal_stitch_kernel,wal_compact_kernel;             A[wal]=wal_stitch_kernel; W[wal]=wal:64:desc
for cfg in ${CFGS:-sst sstdec probe wal}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    echo "== pmc $cfg $c" >&2
    timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d $OUT/pmcm_${cfg}_$c -o run \
      -- python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline > $OUT/pmcm_${cfg}_$c.log 2>&1 || exit 1
  done
  python scripts/pmc_multi.py $OUT/pmcm_${cfg}_FETCH_SIZE $OUT/pmcm_${cfg}_WRITE_SIZE "${K[$cfg]}" "${A[$cfg]}" "${W[$cfg]}" \
    profiles/${TAG}_pmc_$cfg.json $OUT/${TAG}_pmc_$cfg.json || exit 1
done
for cfg in ${CFGS:-sst sstdec probe wal}; do
  echo "== bench $cfg" >&2
  timeout -k 10 300 python bench.py --config $cfg > $OUT/bench_${TAG}_$cfg.json 2> $OUT/bench_${TAG}_$cfg.err || { tail -20 $OUT/bench_${TAG}_$cfg.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_${TAG}_$cfg.json')); print('$cfg', d['value'], d['roofline'])"
done
