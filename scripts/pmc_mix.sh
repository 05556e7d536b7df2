# Instruction-mix PMC passes for the given decode lines (default: arena)
set -o pipefail
for t in ${LINES:-arena}; do
  case $t in
    desc) a="--config decode4k" ;; arena) a="--config decode4k --arena" ;;
    d64) a="--config decode64k" ;; mixed) a="--config mixed" ;;
  esac
  OUTD=gpurun_out/pmcmix_$t BENCH_ARGS="$a" KF=decode_v2,sched bash scripts/pmc_decode.sh > gpurun_out/pmcmix_$t.txt 2>&1 || { tail -5 gpurun_out/pmcmix_$t.txt; exit 1; }
  echo "== $t"; cat gpurun_out/pmcmix_$t.txt
done
