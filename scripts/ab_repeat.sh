# Repeated A/B of decode kernel variants (interleaved, same box): R rounds.
set -o pipefail
export TMPDIR=/tmp
for r in $(seq 1 ${R:-3}); do
  for v in ${VARIANTS:-default v2r8}; do
    for cfg in ${CONFIGS:-decode4k decode64k mixed}; do
      if [ "$v" = default ]; then unset LSM_DECODE_KERNEL; else export LSM_DECODE_KERNEL=$v; fi
      timeout -k 10 200 python bench.py --config $cfg --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/abr.json 2>gpurun_out/abr.err || { tail gpurun_out/abr.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/abr.json'));print('$r $v $cfg', d['value'], d['roofline']['frac'])"
    done
  done
done
