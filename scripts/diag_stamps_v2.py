"""Diagnostic: per-block phase timing of decode_v2_kernel from the stamped
build (liblsm_gpu_stamps.so), s_memrealtime at 100 MHz: start, first record,
after the global verification, end.  Never used by the product."""
import ctypes, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "go-lsm_amd"))
import lsmgpu  # noqa: E402
from lsmgpu import _lib, synth  # noqa: E402
_lib.LIB_PATH = os.path.join(ROOT, "go-lsm_amd", "liblsm_gpu_stamps.so")
lib = _lib.load()
lib.lsm_debug_set_stamps.argtypes = [ctypes.c_void_p]
lib.lsm_debug_set_stamps.restype = ctypes.c_int
cfg = os.environ.get("CFG", "decode64k")
ctx = lsmgpu.Context(0)
dev = ctx.torch_device
if cfg == "decode64k":
    nblk = 6400
    buf, blk_off, blk_len = synth.uniform_kv_blocks(np.arange(nblk), recs=528, slot=65536)
else:
    nblk = 100_000
    buf, blk_off, blk_len = synth.uniform_kv_blocks(np.arange(nblk))
d_in = lsmgpu.to_device_bytes(buf, dev)
d_off = torch.tensor(blk_off.view(np.int64), device=dev)
d_len = torch.tensor(blk_len.view(np.int32), device=dev)
r = lsmgpu.alloc_decode_offset(ctx, 1, nblk, int(d_in.numel()))
st = torch.zeros(nblk * 4, dtype=torch.int64, device=dev)
assert lib.lsm_debug_set_stamps(ctypes.c_void_p(st.data_ptr())) == 0
for _ in range(5):
    lsmgpu.decode_into(ctx, 1, d_in, d_off, d_len, r)
torch.cuda.synchronize()
s = st.cpu().numpy().reshape(nblk, 4).astype(np.float64) / 100.0
t0 = s[:, 0].min()
s -= t0
def q(x):
    return "p10 %.2f  p50 %.2f  p90 %.2f  max %.2f" % tuple(np.percentile(x, [10, 50, 90, 100]).tolist())
print(cfg, "kernel span %.1f us" % s[:, 3].max())
print("start        :", q(s[:, 0]))
print("first record :", q(s[:, 1] - s[:, 0]))
has2 = s[:, 2] > 0
if has2.any():
    print("to verified  :", q(s[has2, 2] - s[has2, 1]), "n=%d" % has2.sum())
    print("after verify :", q(s[has2, 3] - s[has2, 2]))
print("lifetime     :", q(s[:, 3] - s[:, 0]))
ts = np.linspace(0, s[:, 3].max(), 30)
print("resident per CU:", [round(int(((s[:, 0] <= t) & (s[:, 3] > t)).sum()) / 256, 1) for t in ts])
