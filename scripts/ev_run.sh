TAG=r04v PHASE=1 bash scripts/gpu_evidence.sh || exit 1
TAG=r04v PHASE=3 LINES="sst compact decode4k" PROF="sst" bash scripts/gpu_evidence.sh || exit 1
