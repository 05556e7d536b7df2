"""Diagnostic: how many WAL segments' guessed entry points match the true
chain (the stitch re-chases every miss).  Reads lsm_wal_replay's workspace
segment table {entry, exit, nrec, status} after a replay."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "go-lsm_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import lsmgpu  # noqa: E402
import pyoracle as ora  # noqa: E402
from lsmgpu import synth  # noqa: E402
ctx = lsmgpu.Context(0)
dev = ctx.torch_device
buf, off, ln, nrec = synth.wal_logs(2)
d = lsmgpu.to_device_bytes(buf, dev)
o = torch.tensor(off.view(np.int64), device=dev)
l = torch.tensor(ln.view(np.int32), device=dev)
mx = int(ln.max())
r = lsmgpu.alloc_decode_offset(ctx, 1, 2, int(d.numel()))
ws = lsmgpu.wal_workspace(ctx, 2, mx)
lsmgpu.wal_replay_into(ctx, d, o, l, mx, r, ws)
torch.cuda.synchronize()
segs = (mx + 16383) // 16384
slots = 16384 // 8 + 1
n = 2 * segs
tab = ws[2 * n * slots * 16: 2 * n * slots * 16 + 2 * n * 16].cpu().numpy().view(np.uint32).reshape(2, segs, 2, 4)
for w in range(2):
    st, od, _ = ora.decode_block(1, buf, int(off[w]), int(ln[w]))
    starts = set((od["rec_off"] - off[w]).tolist())
    nseg = (int(ln[w]) + 16383) // 16384
    first_true = [min(x for x in starts if x >= s * 16384) if any(x >= s * 16384 for x in starts) else -1 for s in range(nseg)]
    miss = [(s, int(tab[w, s, 0, 0]), int(tab[w, s, 1, 0]), first_true[s]) for s in range(nseg)
            if first_true[s] not in (int(tab[w, s, 0, 0]), int(tab[w, s, 1, 0]))]
    print("log", w, "segments", nseg, "guess == true entry:", nseg - len(miss), "misses:", miss[:8])
