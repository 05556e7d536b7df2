"""Source invariants the kernels rely on (CPU; reads the HIP sources only).

bloom_or_kernel ORs filter bits into its dynamic LDS slice with no per-location
slice test: a location outside the slice must land outside the workgroup's
LDS allocation, which holds only while the dynamic array `lds_bits` is the
kernel's sole LDS and so starts at LDS address 0 (go-lsm_amd/csrc/encode.hip,
bloom_or_kernel; the kernel falls back to a per-location slice test when it
does not).  A static __shared__ in the kernel or in any device function it
calls would break that silently, except through the .sst image tests, so it
is checked here.
"""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENCODE = os.path.join(ROOT, "go-lsm_amd", "csrc", "encode.hip")


def _bodies(src):
    """name -> body text of every function defined in src (brace matching)."""
    out = {}
    for mt in re.finditer(r"\b([A-Za-z_]\w*)\s*\([^;{)]*(?:\([^)]*\)[^;{)]*)*\)\s*(?:const\s*)?\{", src):
        name, i, depth = mt.group(1), mt.end(), 1
        while depth and i < len(src):
            depth += {"{": 1, "}": -1}.get(src[i], 0)
            i += 1
        out.setdefault(name, src[mt.end():i])
    return out


def _callees(body, names):
    return {n for n in names if re.search(r"\b%s\s*(<[^;()]*>)?\s*\(" % re.escape(n), body)}


def test_bloom_or_kernel_has_no_static_lds():
    src = open(ENCODE).read()
    src = re.sub(r"//[^\n]*", "", src)
    bodies = _bodies(src)
    assert "bloom_or_kernel" in bodies
    seen, todo = set(), ["bloom_or_kernel"]
    while todo:
        f = todo.pop()
        if f in seen:
            continue
        seen.add(f)
        todo += sorted(_callees(bodies[f], set(bodies) - {f}))
    assert {"sst_meta_body", "store_filter_slice", "or_key_locations"} <= seen, seen
    for f in seen:
        decls = re.findall(r"[^;{}]*__shared__[^;]*;", bodies[f])
        if f == "bloom_or_kernel":
            assert len(decls) == 1 and "extern" in decls[0] and "lds_bits" in decls[0], decls
        else:
            assert not decls, (f, decls)


def test_or_pass_keeps_its_fallback():
    src = open(ENCODE).read()
    body = _bodies(re.sub(r"//[^\n]*", "", src))["bloom_or_kernel"]
    assert "lds0 == 0" in body and "true>(" in body
