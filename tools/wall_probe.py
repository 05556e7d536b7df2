"""Where the wall clock of the headline step goes (tools only).

Config 2 (100,000 x 4 KiB KV blocks, DESC, offset placement), K launches of
lsm_decode_blocks timed five ways:
  events   -- an event pair recorded around every launch (bench.py r02 loop)
  plain    -- no events inside the wall-timed loop
  direct   -- no events, the ctypes argument tuple built once (launch cost
              of the Python driver taken out)
  twostream-- launches alternate between two streams with two output sets
              (independent batches in flight: one kernel's tail overlaps
              the next one's ramp)
  graph    -- the K launches captured once into a HIP graph, replayed
Prints a JSON line of ms per step (wall) for each, best of R repeats, and
the host-side cost of one launch call."""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "go-lsm_amd"))
import lsmgpu  # noqa: E402
from lsmgpu import codec, synth, _lib  # noqa: E402

K = int(os.environ.get("K", "20"))
R = int(os.environ.get("R", "5"))
ctx = lsmgpu.Context(0)
dev = ctx.torch_device
buf, off, ln = synth.uniform_kv_blocks(np.arange(100_000, dtype=np.int64), recs=33, slot=4096)
nblk = off.size
d_in = lsmgpu.to_device_bytes(buf, dev)
d_off = torch.tensor(off.view(np.int64), device=dev)
d_len = torch.tensor(ln.view(np.int32), device=dev)
outs = [lsmgpu.alloc_decode_offset(ctx, lsmgpu.GRAMMAR_KV, nblk, int(d_in.numel())) for _ in range(2)]
parsed = float(ln.astype(np.float64).sum())
s0 = torch.cuda.current_stream()
s1 = torch.cuda.Stream()
lib = ctx.lib


def launch(r, s):
    codec.decode_into(ctx, lsmgpu.GRAMMAR_KV, d_in, d_off, d_len, r, stream=s)


outs_c = [codec._decode_out(r) for r in outs]
argv = [(ctx.handle, lsmgpu.GRAMMAR_KV, ctypes.c_void_p(d_in.data_ptr()),
         ctypes.c_void_p(d_off.data_ptr()), ctypes.c_void_p(d_len.data_ptr()), nblk,
         ctypes.byref(o), ctypes.c_void_p(s.cuda_stream)) for o, s in zip(outs_c, (s0, s1))]


def direct(i):
    rc = lib.lsm_decode_blocks(*argv[i])
    if rc:
        raise RuntimeError(rc)


def wall(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / K


def v_events():
    st = [torch.cuda.Event(enable_timing=True) for _ in range(K)]
    en = [torch.cuda.Event(enable_timing=True) for _ in range(K)]
    for i in range(K):
        st[i].record(s0)
        launch(outs[0], s0)
        en[i].record(s0)


def v_plain():
    for _ in range(K):
        launch(outs[0], s0)


def v_direct():
    for _ in range(K):
        direct(0)


def v_twostream():
    ev = torch.cuda.Event()
    ev.record(s0)
    s1.wait_event(ev)
    for i in range(K):
        direct(i & 1)
    ev2 = torch.cuda.Event()
    ev2.record(s1)
    s0.wait_event(ev2)


g = torch.cuda.CUDAGraph()
for _ in range(3):
    v_plain()
torch.cuda.synchronize()
with torch.cuda.graph(g):
    cs = torch.cuda.current_stream()
    for _ in range(K):
        codec.decode_into(ctx, lsmgpu.GRAMMAR_KV, d_in, d_off, d_len, outs[0], stream=cs)


def v_graph():
    g.replay()


res = {"K": K}
for name, fn in (("events", v_events), ("plain", v_plain), ("direct", v_direct),
                 ("twostream", v_twostream), ("graph", v_graph)):
    fn()
    ms = sorted(wall(fn) for _ in range(R))
    res[name] = {"ms_best": round(ms[0], 5), "ms_median": round(ms[len(ms) // 2], 5),
                 "GiBps_best": round(parsed / (ms[0] * 1e-3) / 2 ** 30, 1)}
# host cost of one launch call (the GPU runs behind; queue depth bounded by K)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(K):
    launch(outs[0], s0)
res["host_us_per_decode_into"] = round((time.perf_counter() - t0) * 1e6 / K, 2)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(K):
    direct(0)
res["host_us_per_direct_call"] = round((time.perf_counter() - t0) * 1e6 / K, 2)
torch.cuda.synchronize()
# outputs still right after all of it
for r in outs:
    assert int((r.status[:nblk] != 0).sum()) == 0 and int(r.nrec[:nblk].sum()) == 33 * nblk
print(json.dumps(res), flush=True)
