"""Per-iteration phases of the pipelined sst_regions_kernel from a stamps
build (scripts/p_dstamps.py).  Usage: python scripts/diag_regions2.py ab/<lib>.so"""
import ctypes, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "go-lsm_amd")]
import lsmgpu._lib as L
L.LIB_PATH = os.path.abspath(sys.argv[1])
import lsmgpu
from lsmgpu import synth
ctx = lsmgpu.Context(0)
n = 100_000 * 33
keys, koff, vals, voff = synth.kv_stream(n)
batch = lsmgpu.batch_to_device(ctx, keys, koff, vals, voff)
starts = lsmgpu.segment_files(ctx, koff, voff, lsmgpu.MAX_SSTABLE_SIZE)
sb = lsmgpu.prepare_sst(ctx, batch, starts)
nf = len(starts) - 1
spans = (sb.max_recs + 511) // 512
nw = nf * spans * 2
st = torch.zeros(nw * 16, dtype=torch.int64, device=ctx.torch_device)
lib = ctypes.CDLL(L.LIB_PATH)
for it in range(3):
    st.zero_()
    assert lib.lsm_debug_set_rstamps(ctypes.c_void_p(st.data_ptr())) == 0
    lsmgpu.build_sst_into(ctx, batch, sb)
    torch.cuda.synchronize()
a = st.cpu().numpy().reshape(nw, 4, 4).astype(np.float64)
ok = (a > 0).all(axis=(1, 2))
a = a[ok]
t0 = np.median(a[:, 0, 0]) - 1e6
print(f"waves with 4 full iterations: {ok.sum()} of {nw}")
for it in range(4):
    for name, (i, j) in {"plan+issue": (0, 1), "wait": (1, 2), "finish": (2, 3)}.items():
        d = (a[:, it, j] - a[:, it, i]) / 100.0
        print(f"iter {it} {name:11s} mean {d.mean():6.2f} p50 {np.median(d):6.2f} p90 {np.percentile(d, 90):6.2f} us")
    if it < 3:
        d = (a[:, it + 1, 0] - a[:, it, 3]) / 100.0
        print(f"iter {it} {'loop tail':11s} mean {d.mean():6.2f}")
life = (a[:, 3, 3] - a[:, 0, 0]) / 100.0
print(f"4-chunk life mean {life.mean():.2f} p50 {np.median(life):.2f} us")
