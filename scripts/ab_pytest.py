"""Runs GPU tests against a diagnostic library variant (parity of a patched
build before it is A/B-timed).  Usage: python scripts/ab_pytest.py <lib> <pytest args...>"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "go-lsm_amd"), os.path.join(ROOT, "oracle")]
import lsmgpu._lib as L  # noqa: E402

L.LIB_PATH = os.path.abspath(sys.argv[1])
L.CHECK_BUILD_ID = False  # a patched variant: not built from the tree's sources
import pytest  # noqa: E402

sys.exit(pytest.main(sys.argv[2:]))
