"""Diagnostic: the stream build's plan kernel (sst_stream_plan_kernel) alone.
Runs the builder rule (lsm_segment_files) on config 3's stream back to back
(warm translations), then each after a 2 GB sweep (cold), and the full stream
build; run under rocprofv3 --kernel-trace to read each launch's duration."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "go-lsm_amd"))
import lsmgpu  # noqa: E402
from lsmgpu import synth  # noqa: E402

ctx = lsmgpu.Context(0)
n = 3_300_000
keys, koff, vals, voff = synth.kv_stream(n)
batch = lsmgpu.batch_to_device(ctx, keys, koff, vals, voff)
junk = torch.empty(1 << 31, dtype=torch.uint8, device=ctx.torch_device)
for _ in range(20):
    lsmgpu.segment_files_device(ctx, batch)
for _ in range(20):
    junk.add_(1)
    lsmgpu.segment_files_device(ctx, batch)
ss = lsmgpu.prepare_sst_stream(ctx, batch)
for _ in range(20):
    lsmgpu.build_sst_stream_into(ctx, batch, ss)
torch.cuda.synchronize()
print("ok", ss.result().nfile)
