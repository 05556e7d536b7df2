set -o pipefail
export TMPDIR=/tmp
for spec in ${SPECS:-"0 default decode64k" "2 default decode64k" "4 default decode64k" "0 v2r8 decode64k" "2 v2r8 decode64k"}; do
  set -- $spec
  if [ "$2" = default ]; then unset LSM_DECODE_KERNEL; else export LSM_DECODE_KERNEL=$2; fi
  LSM_DECODE_DBG=$1 timeout -k 10 200 python bench.py --config $3 --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/dbg.json 2>gpurun_out/dbg.err || { tail gpurun_out/dbg.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/dbg.json'));print('$1 $2 $3', d['value'], d['roofline']['kernel_ms'])"
done
