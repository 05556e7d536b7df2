"""CPU tests of the C-ABI library: it loads, exports every symbol declared in
include/lsm_gpu.h, and its host-side logic (builder flush rule, image sizes,
capacities) matches the oracle.  No GPU compute calls here."""
import ctypes
import os
import re

import numpy as np
import pytest

import pyoracle as ora
from lsmgpu import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "lsm_gpu.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(lsm_[a-z0-9_]+)\s*\(", src)))


def test_header_functions_exported():
    lib = _lib.load()
    names = declared_functions()
    assert len(names) >= 15
    for n in names:
        assert hasattr(lib, n), f"{n} declared in lsm_gpu.h but not exported"
    assert set(names) == set(_lib.SIGNATURES), "ctypes table out of sync with the header"


def test_abi_version():
    assert _lib.load().lsm_abi_version() == 7
    assert _lib.load().lsm_input_slack() == 32


def test_ctx_create_without_gpu_fails_cleanly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    h = ctypes.c_void_p()
    rc = _lib.load().lsm_ctx_create(0, ctypes.byref(h))
    assert rc != 0 and not h.value


def test_max_records():
    lib = _lib.load()
    assert lib.lsm_max_records(0, 4092) == 1023
    assert lib.lsm_max_records(1, 4092) == 511
    assert lib.lsm_max_records(2, 4092) == 341


@pytest.mark.parametrize("seed", range(6))
def test_segment_files_matches_oracle(seed):
    lib = _lib.load()
    rng = np.random.default_rng(seed)
    n = int(rng.integers(0, 3000))
    kl = rng.integers(0, 64, n).astype(np.uint64)
    vl = rng.integers(0, 5000, n).astype(np.uint64)
    koff = np.zeros(n + 1, np.uint64)
    voff = np.zeros(n + 1, np.uint64)
    koff[1:] = np.cumsum(kl)
    voff[1:] = np.cumsum(vl)
    for thr in (0, 1, 4096, 65536, 2 * 1024 * 1024):
        want = ora.segment_files(koff, voff, thr)
        got = np.zeros(n + 2, np.uint64)
        nf = lib.lsm_segment_files_host(koff.ctypes.data, voff.ctypes.data, n, thr,
                                        got.ctypes.data)
        assert got[: nf + 1].tolist() == want.tolist()


def test_image_size_matches_oracle():
    lib = _lib.load()
    rng = np.random.default_rng(3)
    n = 500
    koff = np.zeros(n + 1, np.uint64)
    voff = np.zeros(n + 1, np.uint64)
    koff[1:] = np.cumsum(rng.integers(0, 40, n))
    voff[1:] = np.cumsum(rng.integers(0, 300, n))
    for (r0, r1) in [(0, 0), (0, 1), (3, 77), (0, n)]:
        for m in (1, 64, 1000, 1_600_000):
            assert lib.lsm_sst_image_size_host(koff.ctypes.data, voff.ctypes.data, r0, r1, m) == \
                ora.lib().ora_sst_image_size(koff.ctypes.data, voff.ctypes.data, r0, r1, m)
    for g in range(3):
        assert lib.lsm_encoded_size_host(g, koff.ctypes.data, voff.ctypes.data, 5, 300) == \
            ora.lib().ora_encoded_size(g, koff.ctypes.data, voff.ctypes.data, 5, 300)
    assert lib.lsm_filter_block_size(1_600_000) == 200_032


def test_code_object_is_gfx950():
    so = os.path.join(ROOT, "go-lsm_amd", "liblsm_gpu.so")
    blob = open(so, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    for other in (b"--gfx942", b"--gfx90a", b"--gfx1100"):
        assert other not in blob


def test_build_id_ties_library_to_sources(tmp_path):
    """liblsm_gpu.so carries the hash of the sources it was built from
    (go-lsm_amd/build_id.py); load() refuses a library whose id differs from
    the tree's, so a stale prebuilt .so cannot stand in for the sources."""
    import importlib.util
    import shutil
    pkg = os.path.join(ROOT, "go-lsm_amd")
    spec = importlib.util.spec_from_file_location("bid", os.path.join(pkg, "build_id.py"))
    bid = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bid)
    assert _lib.load().lsm_build_id().decode() == bid.source_id(pkg)
    # a copy of the tree with one source byte changed: the same library is refused
    alt = tmp_path / "go-lsm_amd"
    shutil.copytree(os.path.join(pkg, "csrc"), alt / "csrc")
    shutil.copy(os.path.join(pkg, "Makefile"), alt / "Makefile")
    shutil.copy(os.path.join(pkg, "build_id.py"), alt / "build_id.py")
    os.makedirs(tmp_path / "include")
    shutil.copy(HEADER, tmp_path / "include" / "lsm_gpu.h")
    assert bid.source_id(str(alt)) == bid.source_id(pkg)
    with open(alt / "csrc" / "common.h", "a") as f:
        f.write("\n// changed\n")
    assert bid.source_id(str(alt)) != bid.source_id(pkg)
    os.makedirs(alt / "lsmgpu")
    shutil.copy(os.path.join(pkg, "lsmgpu", "_lib.py"), alt / "lsmgpu" / "_lib.py")
    shutil.copy(os.path.join(pkg, "liblsm_gpu.so"), alt / "liblsm_gpu.so")
    spec = importlib.util.spec_from_file_location("alt_lib", str(alt / "lsmgpu" / "_lib.py"))
    alt_lib = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(alt_lib)
    with pytest.raises(RuntimeError, match="built from other sources"):
        alt_lib.load()


def test_build_id_covers_compiler_flags():
    """The id also hashes the compiler, target and flags the Makefile compiles
    with, overrides included (`make ARCH=... HIPFLAGS=...` built a
    library with the default id): the Makefile's defaults give the loader's
    id, any other target or flags another one."""
    import importlib.util
    import subprocess
    pkg = os.path.join(ROOT, "go-lsm_amd")
    spec = importlib.util.spec_from_file_location("bid", os.path.join(pkg, "build_id.py"))
    bid = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bid)
    hipcc, arch, flags = bid.default_flags(pkg)
    assert arch == "gfx950" and "--offload-arch=gfx950" in flags
    assert bid.source_id(pkg, [hipcc, arch, flags]) == bid.source_id(pkg)
    assert bid.source_id(pkg, [hipcc, "gfx942", flags.replace("gfx950", "gfx942")]) != bid.source_id(pkg)
    assert bid.source_id(pkg, [hipcc, arch, flags + " -O0"]) != bid.source_id(pkg)
    # the id make compiles in: defaults, and a command-line override
    def make_id(*args):
        out = subprocess.run(["make", "-n", "-C", pkg, "-B", "build/api.o", *args], capture_output=True,
                             text=True, check=True).stdout
        return out.split("LSM_BUILD_ID='\"")[1].split('"')[0]
    assert make_id() == bid.source_id(pkg)
    assert make_id("HIPFLAGS=-O1 --offload-arch=gfx950") != bid.source_id(pkg)


def test_build_flags_recorded():
    """The library records the compiler, target and flags it was built with
    (lsm_build_flags); the build id is the sources hashed with exactly those,
    so a `make ARCH=... HIPFLAGS=...` build is accepted by load()."""
    import importlib.util
    pkg = os.path.join(ROOT, "go-lsm_amd")
    spec = importlib.util.spec_from_file_location("bid", os.path.join(pkg, "build_id.py"))
    bid = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bid)
    lib = _lib.load()
    flags = lib.lsm_build_flags().decode().split("|")
    assert len(flags) == 3 and flags[1] == "gfx950"
    assert lib.lsm_build_id().decode() == bid.source_id(pkg, flags=flags)
    other = [flags[0], flags[1], flags[2] + " -DX"]
    assert bid.source_id(pkg, flags=other) != bid.source_id(pkg, flags=flags)


@pytest.mark.parametrize("seed", range(4))
def test_stream_max_files_bounds_the_rule(seed):
    """lsm_stream_max_files bounds the file count of every stream: each file
    but the last holds EstimateSize sums >= threshold (builder.go:40-42)."""
    lib = _lib.load()
    rng = np.random.default_rng(seed)
    for _ in range(20):
        n = int(rng.integers(0, 4000))
        kl = rng.integers(0, 64, n).astype(np.uint64)
        vl = rng.integers(0, int(rng.choice([1, 100, 5000])), n).astype(np.uint64)
        koff = np.zeros(n + 1, np.uint64)
        voff = np.zeros(n + 1, np.uint64)
        koff[1:] = np.cumsum(kl)
        voff[1:] = np.cumsum(vl)
        for thr in (0, 1, 16, 17, 4096, 2 * 1024 * 1024):
            nf = len(ora.segment_files(koff, voff, thr)) - 1
            bound = lib.lsm_stream_max_files(n, int(koff[-1]), int(voff[-1]), thr)
            assert nf <= bound <= n
    assert lib.lsm_stream_max_files(3_300_000, 16 * 3_300_000, 100 * 3_300_000, 2 * 1024 * 1024) == 208
    assert lib.lsm_stream_max_files(0, 0, 0, 100) == 0
    assert lib.lsm_stream_max_files(5, 0, 0, 0) == 1
