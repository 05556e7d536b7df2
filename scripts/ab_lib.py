"""A/B of library builds: runs bench.py against a given liblsm_gpu build.
Usage: python scripts/ab_lib.py <lib path> [bench args...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "go-lsm_amd")]
import lsmgpu._lib as L  # noqa: E402

L.LIB_PATH = os.path.abspath(sys.argv[1])
L.CHECK_BUILD_ID = False  # a patched variant: not built from the tree's sources
import bench  # noqa: E402

bench.main(["--no-cpu-baseline"] + sys.argv[2:])
