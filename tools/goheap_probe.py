"""Host-side timing of the LSM_TIE_GOHEAP replay (lsm_goheap_pop_order_host)
on the compaction bench's key ranks (bench_compact.py: 8 level-0 update runs,
newest first, then 3.3M sorted level-1 keys).  No GPU: the replay is host
code.  Usage: python tools/goheap_probe.py [lib.so ...]; prints ms per call
for each library and checks every library's pop order against the first's."""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "go-lsm_amd")]


def compaction_ranks(n1=3_300_000, nfiles=8, per=15_888, seed=0x5EED + 77):
    rng = np.random.default_rng(seed)
    runs = [np.unique(rng.integers(0, n1, per)) for _ in range(nfiles)]
    ids = np.concatenate(runs + [np.arange(n1)])
    return ids.astype(np.uint32)  # ids are dense: the id is the key's rank


def pop_order(lib, rank):
    f = lib.lsm_goheap_pop_order_host
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    order = np.zeros(rank.size, np.uint32)
    t0 = time.perf_counter()
    rc = f(rank.ctypes.data, rank.size, order.ctypes.data)
    dt = time.perf_counter() - t0
    assert rc == 0
    return order, dt


if __name__ == "__main__":
    libs = sys.argv[1:] or [os.path.join(ROOT, "go-lsm_amd", "liblsm_gpu.so")]
    rank = compaction_ranks()
    ref = None
    for path in libs:
        lib = ctypes.CDLL(os.path.abspath(path))
        ts = []
        for _ in range(3):
            order, dt = pop_order(lib, rank)
            ts.append(dt)
        same = ref is None or np.array_equal(order, ref)
        ref = order if ref is None else ref
        print(f"{path}: n={rank.size} best {min(ts) * 1e3:.1f} ms, mean {np.mean(ts) * 1e3:.1f} ms, "
              f"order {'==' if same else '!='} first")
