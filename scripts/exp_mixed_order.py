"""Experiment: config-5 decode time vs block order (as generated / largest
first) for a given library build.  Usage: python scripts/exp_mixed_order.py ab/<lib>.so"""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "go-lsm_amd")]
import lsmgpu._lib as L
L.LIB_PATH = os.path.abspath(sys.argv[1])
import lsmgpu
from lsmgpu import synth
ctx = lsmgpu.Context(0)
dev = ctx.torch_device
buf, off, ln, _ = synth.mixed_kv_blocks(1 << 30, seed=synth.SEED)
d_in = lsmgpu.to_device_bytes(buf, dev)
s = torch.cuda.current_stream()
def qclass(n):
    n = n.astype(np.int64)
    l = np.floor(np.log2(np.maximum(n, 1))).astype(np.int64)
    c = 4 * (l - 1) + ((n >> np.maximum(l - 2, 0)) & 3)
    return np.where(n < 4, n, c)
rng = np.random.default_rng(1)
cls = qclass(ln)
by_class = np.lexsort((rng.random(ln.size), -cls))  # class desc, random inside a class
for name, order in (("generated", np.arange(off.size)), ("largest-first", np.argsort(-ln.astype(np.int64), kind="stable")),
                    ("class-desc", by_class)):
    o, l = off[order], ln[order]
    d_off = torch.tensor(o.view(np.int64), device=dev)
    d_len = torch.tensor(l.view(np.int32), device=dev)
    r = lsmgpu.alloc_decode_offset(ctx, lsmgpu.GRAMMAR_KV, o.size, int(d_in.numel()))
    for _ in range(5):
        lsmgpu.decode_into(ctx, lsmgpu.GRAMMAR_KV, d_in, d_off, d_len, r, stream=s)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(50):
        lsmgpu.decode_into(ctx, lsmgpu.GRAMMAR_KV, d_in, d_off, d_len, r, stream=s)
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 50
    print(f"{os.path.basename(sys.argv[1])} {name}: {ms * 1e3:.1f} us, nblk {o.size}", flush=True)
    if name == "generated" and hasattr(lsmgpu, "schedule_workspace"):
        ws = lsmgpu.schedule_workspace(ctx, o.size)
        for _ in range(5):
            lsmgpu.decode_into(ctx, lsmgpu.GRAMMAR_KV, d_in, d_off, d_len, r, stream=s, schedule=ws)
        torch.cuda.synchronize()
        e0.record(s)
        for _ in range(50):
            lsmgpu.decode_into(ctx, lsmgpu.GRAMMAR_KV, d_in, d_off, d_len, r, stream=s, schedule=ws)
        e1.record(s)
        torch.cuda.synchronize()
        print(f"  scheduled entry: {e0.elapsed_time(e1) / 50 * 1e3:.1f} us", flush=True)
