import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "go-lsm_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def _ensure_built():
    """Build the oracle and the product library in-tree if they are missing
    (the GPU box gets the prebuilt .so files with the snapshot)."""
    ora = os.path.join(ROOT, "oracle", "liblsm_oracle.so")
    gpu = os.path.join(ROOT, "go-lsm_amd", "liblsm_gpu.so")
    if not os.path.exists(ora):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True,
                       stdout=subprocess.DEVNULL)
    mirror = os.path.join(ROOT, "go-lsm_amd", "libgolsm.so")
    if not (os.path.exists(gpu) and os.path.exists(mirror)):
        subprocess.run(["make", "-C", os.path.join(ROOT, "go-lsm_amd"), "-j4"], check=True,
                       stdout=subprocess.DEVNULL)
    if not os.path.exists(os.path.join(ROOT, "tests", "cpp", "mirror_test")):
        subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "cpp")], check=True,
                       stdout=subprocess.DEVNULL)


_ensure_built()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def ctx():
    import torch
    import lsmgpu
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    c = lsmgpu.Context(0)
    yield c
    c.close()
