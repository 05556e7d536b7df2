"""Source identity of liblsm_gpu.so: a hash of every file the library is
compiled from (csrc/, the C ABI header, the Makefile) and of the compiler,
target and flags it was compiled with (the Makefile passes its HIPCC, ARCH
and HIPFLAGS, command-line overrides included; without arguments the
Makefile's own defaults are used).  The Makefile
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


def default_flags(pkg=PKG):
    """HIPCC, ARCH and HIPFLAGS as the Makefile sets them without overrides."""
    v = {}
    with open(os.path.join(pkg, "Makefile")) as f:
        for line in f:
            for name in ("HIPCC", "ARCH", "HIPFLAGS"):
                if line.startswith(name + " ?= "):
                    v[name] = line[len(name) + 4:].strip()
    v["HIPFLAGS"] = v["HIPFLAGS"].replace("$(ARCH)", v["ARCH"])
    return [v["HIPCC"], v["ARCH"], v["HIPFLAGS"]]


def source_id(pkg=PKG, flags=None):
    h = hashlib.sha256()
    flags = [" ".join(x.split()) for x in (flags or default_flags(pkg))]
    h.update(b"flags\0" + "\0".join(flags).encode() + b"\0")
    for name, path in source_files(pkg):
        with open(path, "rb") as f:
            data = f.read()
        h.update(name.encode() + b"\0" + str(len(data)).encode() + b"\0" + data)
    return h.hexdigest()[:16]


if __name__ == "__main__":
    # build_id.py [HIPCC ARCH HIPFLAGS]: the Makefile's effective values
    sys.stdout.write(source_id(flags=sys.argv[1:4] if len(sys.argv) >= 4 else None))
