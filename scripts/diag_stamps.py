"""Diagnostic: per-workgroup phase timing of decode_lanes_kernel from the
stamped build (liblsm_gpu_stamps.so).  Reports, in microseconds of
s_memrealtime (100 MHz), the staging+DMA wait (t1-t0), the chase (t2-t1) and
the number of workgroups resident over time.  Never used by the product."""
import ctypes
import os
import sys

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

B = int(os.environ.get("DIAG_BLOCKS_PER_WG", "4"))  # spec kernel: 4 waves x 1 block
ctx = lsmgpu.Context(0)
dev = ctx.torch_device
nblk = 100_000
buf, blk_off, blk_len = synth.uniform_kv_blocks(np.arange(nblk))
d_in = lsmgpu.to_device_bytes(buf, dev)
d_off = torch.tensor(blk_off.view(np.int64), device=dev)
d_len = torch.tensor(blk_len.view(np.int32), device=dev)
r = lsmgpu.alloc_decode_offset(ctx, 1, nblk, int(d_in.numel()))
grid = (nblk + B - 1) // B
st = torch.zeros(grid * 4, dtype=torch.int64, device=dev)
assert lib.lsm_debug_set_stamps(ctypes.c_void_p(st.data_ptr())) == 0
for _ in range(5):
    lsmgpu.decode_into(ctx, 1, d_in, d_off, d_len, r)
torch.cuda.synchronize()
s = st.cpu().numpy().reshape(grid, 4).astype(np.float64) / 100.0  # us
t0 = s[:, 0].min()
s -= t0
dma = s[:, 1] - s[:, 0]
chase = s[:, 2] - s[:, 1]
life = s[:, 3] - s[:, 0]


def q(x):
    return "p10 %.2f  p50 %.2f  p90 %.2f  mean %.2f" % tuple(np.percentile(x, [10, 50, 90]).tolist() + [x.mean()])


print("B=%d grid=%d kernel span %.1f us" % (B, grid, s[:, 3].max()))
print("stage+DMA wait :", q(dma))
print("chase          :", q(chase))
print("lifetime       :", q(life))
ts = np.linspace(0, s[:, 3].max(), 40)
res = [int(((s[:, 0] <= t) & (s[:, 3] > t)).sum()) for t in ts]
print("resident WGs over time:", res)
print("per CU (256):", [round(x / 256, 1) for x in res])
