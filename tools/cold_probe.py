"""Cold vs resident ceilings (tools only): the Infinity Cache (MALL, 256 MB)
keeps part of a 409.6 MB buffer read back to back, so rates measured by
re-reading one buffer are not HBM rates.  Each probe here runs K launches
rotating over R distinct buffers (R = 1: resident steady state; R = 8:
3.3 GB, cold) and prints GB/s of the bytes each launch moves:
  read_x4   -- plain streaming read, global_load_dwordx4, 2,048 workgroups
  read_lds  -- streaming read by LDS-DMA (the decode's load instruction)
  blocks    -- the decode's memory pattern without the parse: 100,000 x 4 KiB
               blocks by LDS-DMA (nt), 33 x 16 B descriptors written per block
  decode    -- lsm_decode_blocks on config 2 (the headline kernel)"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "go-lsm_amd"))
L = ctypes.CDLL(os.path.join(ROOT, "tools", "libhbm_probe.so"))
L.probe_blocks.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                           ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
for f in ("probe_read", "probe_read_lds"):
    getattr(L, f).argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int,
                              ctypes.c_void_p]
import lsmgpu._lib as _L  # noqa: E402
if os.environ.get("LIB"):  # a diagnostic library variant (scripts/build_variant.sh)
    _L.LIB_PATH = os.path.abspath(os.environ["LIB"])
import lsmgpu  # noqa: E402
from lsmgpu import synth  # noqa: E402

K = int(os.environ.get("K", "40"))
RS = (1, 8)
nblk = 100_000
ctx = lsmgpu.Context(0)
dev = ctx.torch_device
s = torch.cuda.current_stream()
buf, off, ln = synth.uniform_kv_blocks(np.arange(nblk, dtype=np.int64), recs=33, slot=4096)
d_off = torch.tensor(off.view(np.int64), device=dev)
d_len = torch.tensor(ln.view(np.int32), device=dev)
ins = [lsmgpu.to_device_bytes(buf, dev) for _ in range(max(RS))]
outs = [lsmgpu.alloc_decode_offset(ctx, lsmgpu.GRAMMAR_KV, nblk, int(ins[0].numel()))
        for _ in range(max(RS))]
outs_c = [lsmgpu.codec._decode_out(r) for r in outs]
pdesc = [torch.empty(nblk * 33 * 16, dtype=torch.uint8, device=dev) for _ in range(max(RS))]
sink = torch.zeros(4, dtype=torch.int32, device=dev)
n = nblk * 4096


def rate(fn, nbytes, R):
    for i in range(2 * R):
        fn(i % R)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for i in range(K):
        fn(i % R)
    e1.record(s)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / K
    return {"GBps": round(nbytes / (us * 1e-6) / 1e9, 1), "us": round(us, 2)}


probes = {
    "read_x4": (lambda i: L.probe_read(ins[i].data_ptr(), n, sink.data_ptr(), 2048, s.cuda_stream), n),
    "read_lds": (lambda i: L.probe_read_lds(ins[i].data_ptr(), n, sink.data_ptr(), 2048, s.cuda_stream), n),
    "blocks": (lambda i: L.probe_blocks(7, ins[i].data_ptr(), d_off.data_ptr(), d_len.data_ptr(), nblk,
                                        pdesc[i].data_ptr(), 0, s.cuda_stream),
               n + nblk * (12 + 33 * 16)),
    "decode": (lambda i: lib_decode(i), 464_000_000),
}


def lib_decode(i):
    rc = ctx.lib.lsm_decode_blocks(ctx.handle, lsmgpu.GRAMMAR_KV, ctypes.c_void_p(ins[i].data_ptr()),
                                   ctypes.c_void_p(d_off.data_ptr()), ctypes.c_void_p(d_len.data_ptr()),
                                   nblk, ctypes.byref(outs_c[i]), ctypes.c_void_p(s.cuda_stream))
    assert rc == 0


res = {}
only = os.environ.get("ONLY")
for name, (fn, nbytes) in probes.items():
    if only and name not in only.split(","):
        continue
    for R in RS:
        res[f"{name}_R{R}"] = rate(fn, nbytes, R)
print(json.dumps(res), flush=True)
