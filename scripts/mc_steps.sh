#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for k in 10 50 200 1000; do
  timeout -k 10 200 python bench.py --config probe --steps $k --warmup 5 --no-cpu-baseline > gpurun_out/mcs_$k.json 2>gpurun_out/mcs_$k.err || { tail gpurun_out/mcs_$k.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/mcs_$k.json'));print($k,d['ms_per_step'],d['roofline']['kernel_ms'])"
done
for k in 10 200; do
  timeout -k 10 200 python bench.py --config sstdec --steps $k --warmup 5 --no-cpu-baseline > gpurun_out/mcd_$k.json 2>gpurun_out/mcd_$k.err || { tail gpurun_out/mcd_$k.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/mcd_$k.json'));print('sstdec',$k,d['ms_per_step'],d['roofline']['kernel_ms'])"
done
