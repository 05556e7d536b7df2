"""The oracle under ASan + UBSan (host only): oracle/sanitize_main.c fuzzes
every restated decoder, encoder, the bloom / filter-block code, .sst build and
decode (truncated and bit-flipped images), MayContain and the merge, with
every input malloc'd at its exact size.  A sanitizer report fails the run."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not present")
def test_oracle_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", ORACLE, "sanitize"], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(ORACLE, "sanitize_driver")], capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "oracle sanitizer run ok" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
