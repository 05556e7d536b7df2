"""A/B of lsm_build_sst launch structures: runs `bench.py --config sst` against
a given library build (liblsm_gpu.so or a liblsm_gpu_sstN.so diagnostic build).
Usage: python scripts/ab_sst.py <lib path> [bench args...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "go-lsm_amd")]
import lsmgpu._lib as L  # noqa: E402

L.LIB_PATH = os.path.abspath(sys.argv[1])
import bench  # noqa: E402

bench.main(["--config", "sst", "--no-cpu-baseline"] + sys.argv[2:])
