set -o pipefail
export TMPDIR=/tmp
for rep in 1 2; do
for a in "--arena" "--arena --placement plan" "" "--placement plan"; do
  timeout -k 10 240 python bench.py $a --steps 60 --warmup 10 --no-cpu-baseline --no-cold > gpurun_out/pl.json 2> gpurun_out/pl.err || { tail -5 gpurun_out/pl.err; exit 1; }
  python3 -c "import json; j=json.load(open('gpurun_out/pl.json')); r=j['roofline']; print('$a', j['value'], j['ms_per_step'], r['kernel_ms'], r['frac'])"
done; done
