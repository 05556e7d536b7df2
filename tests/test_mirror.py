"""The C++ mirror (go-lsm_amd/host/golsm.h) run through tests/cpp/mirror_test:
the reference's block / sstable / bloom tests restated in C++ (each case cites
its Go test) plus cross-checks against the oracle.  The GPU run executes every
case; on CPU only the host-only cases run (no codec call without a GPU)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "mirror_test")

HOST_ONLY = ["TestDataBlock_AddAndLen", "TestIndexBlock_Iterator", "TestBloomLowNumbers",
             "TestBuilder"]


def _run(args, timeout):
    p = subprocess.run([BIN] + args, capture_output=True, text=True, timeout=timeout)
    return p.returncode, p.stdout + p.stderr


@pytest.mark.parametrize("case", HOST_ONLY)
def test_mirror_host_logic(case):
    rc, out = _run([case], 60)
    assert rc == 0 and ("PASS " + case) in out, out


def test_mirror_fails_loudly_without_gpu():
    """No CPU fallback: a codec call without a gfx950 device raises."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    rc, out = _run(["TestDataBlock_EncodeDecode"], 60)
    assert rc != 0 and "lsm_ctx_create" in out, out


@pytest.mark.gpu
def test_mirror_all_cases_gpu():
    rc, out = _run([], 600)
    print(out)
    assert rc == 0, out
    assert "FAIL" not in out
