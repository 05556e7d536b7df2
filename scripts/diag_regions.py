"""Timeline of sst_regions_kernel waves from a stamps build (scripts/p_rstamps.py):
per-phase durations and average resident waves per CU.
Usage: python scripts/diag_regions.py ab/<lib>.so [--bloom]"""
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
rch = (sb.max_recs + 255) // 256
nw = nf * rch * 4
st = torch.zeros(nw * 8, dtype=torch.int64, device=ctx.torch_device)
lib = ctypes.CDLL(L.LIB_PATH)
for it in range(3):
    st.zero_()
    assert lib.lsm_debug_set_rstamps(ctypes.c_void_p(st.data_ptr())) == 0
    lsmgpu.build_sst_into(ctx, batch, sb)
    torch.cuda.synchronize()
a = st.cpu().numpy().reshape(nw, 8)[:, :5].astype(np.float64)
a = a[a[:, 0] > 0]
t0 = a[:, 0].min()
a = (a - t0) / 100.0  # 100 MHz -> us
span = a[:, 4].max()
life = a[:, 4] - a[:, 0]
print(f"waves {len(a)} span {span:.1f} us, mean resident waves/CU {life.sum() / span / 256:.2f}")
for name, (i, j) in {"setup->V landed": (0, 1), "V landed->V stored": (1, 2),
                     "V stored->IDX landed": (2, 3), "IDX landed->end(stores done)": (3, 4),
                     "lifetime": (0, 4)}.items():
    d = a[:, j] - a[:, i]
    print(f"{name:30s} mean {d.mean():7.2f} p50 {np.median(d):7.2f} p90 {np.percentile(d, 90):7.2f} us")
# start-time profile: waves started per 10 us
h = np.histogram(a[:, 0], bins=np.arange(0, span + 10, 10))[0]
print("starts per 10us:", h.tolist())
