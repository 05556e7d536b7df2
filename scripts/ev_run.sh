TAG=r04y PHASE=2 PMC1="" PMCM="sstdec" bash scripts/gpu_evidence.sh || exit 1
TAG=r04y PHASE=3 PROF="sstdec compact decode4k" bash scripts/gpu_evidence.sh || exit 1
