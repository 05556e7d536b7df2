# A/B: each library in $LIBS through `scripts/ab_lib.py` with $ARGS, $REPS rounds
# interleaved; prints value and kernel ms per run into $OUT.
set -o pipefail
OUT=${OUT:-gpurun_out/ab.txt}; mkdir -p $(dirname $OUT); : > $OUT
for r in $(seq 1 ${REPS:-2}); do
  for l in $LIBS; do
    timeout -k 10 ${TMO:-240} python scripts/ab_lib.py ab/$l.so $ARGS > gpurun_out/ab_one.json 2>gpurun_out/ab_err.log || { echo "$l failed" >> $OUT; tail -5 gpurun_out/ab_err.log >> $OUT; exit 1; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/ab_one.json').read().strip().splitlines()[-1]); r=d.get('roofline',{}); print('$l', round(d['value'],1), d['ms_per_step'], r.get('frac'), r.get('kernel_ms_median'))" >> $OUT
  done
done
cat $OUT
