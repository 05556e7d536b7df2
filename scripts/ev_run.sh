TAG=r04w PHASE=1 bash scripts/gpu_evidence.sh || exit 1
TAG=r04w PHASE=3 LINES="decode4k compact sstdec" PROF="compact" bash scripts/gpu_evidence.sh || exit 1
