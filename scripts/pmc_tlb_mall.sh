#!/bin/bash
# PMC: translation misses (UTCL1) and fabric reads split by destination
# (TCC_EA0_RDREQ vs its DRAM part) for the headline decode at 100k and 1M
# blocks, and for resident vs rotated (cold) input (tools/cold_probe.py).
# One rocprofv3 --pmc pass per workload; summaries by scripts/pmc_kv.py.
set -o pipefail
export TMPDIR=/tmp
C="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum"
run() { local tag=$1; shift; timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmcx_$tag -o run -- "$@" > gpurun_out/pmcx_$tag.log 2>&1 || { tail -5 gpurun_out/pmcx_$tag.log; exit 1; }; }
run d100k python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-cold
run d1m python bench.py --global-blocks 1000000 --steps 3 --warmup 1 --no-cpu-baseline --no-cold
ONLY=decode K=8 run cold python tools/cold_probe.py
