set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_decode_gpu.py tests/test_sst_decode_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_quick.log 2>&1 || { tail -30 gpurun_out/pytest_quick.log; exit 1; }
tail -1 gpurun_out/pytest_quick.log
LINES="decode4k cfg4 decode64k mixed arena" VARIANTS="prod" REPS=2 STEPS=100 bash scripts/ab_pair.sh
