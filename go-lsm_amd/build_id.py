"""Source identity of liblsm_gpu.so: a hash of every file the library is
compiled from (csrc/, the C ABI header, the Makefile's flags).  The Makefile
compiles it into the library (lsm_build_id()); lsmgpu._lib.load() recomputes
it from the sources next to the library and refuses a library built from
other sources, so a stale prebuilt .so cannot pass for the current tree.
No dependencies beyond the standard library (the Makefile runs it)."""
import hashlib
import os
import sys

PKG = os.path.dirname(os.path.abspath(__file__))


def source_files(pkg=PKG):
    csrc = os.path.join(pkg, "csrc")
    names = sorted(n for n in os.listdir(csrc) if n.endswith((".hip", ".h")))
    files = [("csrc/" + n, os.path.join(csrc, n)) for n in names]
    files.append(("include/lsm_gpu.h", os.path.join(os.path.dirname(pkg), "include", "lsm_gpu.h")))
    files.append(("Makefile", os.path.join(pkg, "Makefile")))
    return files


def source_id(pkg=PKG):
    h = hashlib.sha256()
    for name, path in source_files(pkg):
        with open(path, "rb") as f:
            data = f.read()
        h.update(name.encode() + b"\0" + str(len(data)).encode() + b"\0" + data)
    return h.hexdigest()[:16]


if __name__ == "__main__":
    sys.stdout.write(source_id())
