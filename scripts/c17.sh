# round-5 GPU step 17: where wal_seg_lanes_kernel's time goes (clock64 stamps per section, diagnostic library)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python scripts/ab_lib.py ab/walt.so --config wal --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c17_walt.out 2> gpurun_out/c17_walt.err || { tail -20 gpurun_out/c17_walt.err; exit 1; }
grep WALT gpurun_out/c17_walt.out || true
