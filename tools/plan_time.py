"""Diagnostic: section times of the stream build's plan kernel from a
variant library that stamps s_memtime into d_counts[4..9] (start, after the
stream's ends, after round 1's loads, after the rule, after the layout, end).
Usage: python tools/plan_time.py ab/<variant>.so"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "go-lsm_amd"))
import lsmgpu._lib as L  # noqa: E402
L.LIB_PATH = os.path.abspath(sys.argv[1])
L.CHECK_BUILD_ID = False
import lsmgpu  # noqa: E402
from lsmgpu import synth  # noqa: E402
from lsmgpu.codec import _ptr  # noqa: E402

ctx = lsmgpu.Context(0)
n = 3_300_000
keys, koff, vals, voff = synth.kv_stream(n)
batch = lsmgpu.batch_to_device(ctx, keys, koff, vals, voff)
ss = lsmgpu.prepare_sst_stream(ctx, batch)
ss.counts = torch.zeros(16, dtype=torch.int64, device=ctx.torch_device)
junk = torch.empty(1 << 30, dtype=torch.uint8, device=ctx.torch_device)
for mode in ("rule", "build", "build-cold"):
    d = []
    for it in range(12):
        if mode == "build-cold":
            junk.add_(1)
        if mode == "rule":
            L.check(ctx.lib.lsm_segment_files(ctx.handle, _ptr(batch.koff), _ptr(batch.voff), n,
                                              lsmgpu.MAX_SSTABLE_SIZE, ss.nfile_max, _ptr(ss.d_file_start),
                                              _ptr(ss.counts), None), "seg")
        else:
            lsmgpu.build_sst_stream_into(ctx, batch, ss)
        torch.cuda.synchronize()
        t = ss.counts.cpu().numpy()[4:10].astype(np.int64)
        d.append(np.diff(t))
    d = np.array(d[2:])
    print(mode, "ticks per section:",
          np.median(d, axis=0).tolist(), "total", int(np.median(d.sum(axis=1))))
