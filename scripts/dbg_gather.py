"""Diagnose lsm_gather_kvs byte mismatches (prints the records around each)."""
import os
import random
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "go-lsm_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import lsmgpu  # noqa: E402
from test_merge_gpu import lay_out, random_pairs  # noqa: E402

ctx = lsmgpu.Context(0)
rng = random.Random(11)
pairs = random_pairs(rng, 6000, b"abcdefgh", 14, tomb=0.1, maxval=300)
buf, kd, vd, kpos, vpos = lay_out(pairs, False, random.Random(0))
dev = ctx.torch_device
d_buf = lsmgpu.to_device_bytes(buf, dev)
d_kd = torch.from_numpy(kd.view(np.int32).reshape(-1, 4).copy()).to(dev)
d_vd = torch.from_numpy(vd.view(np.int32).reshape(-1, 4).copy()).to(dev)
idx = np.arange(len(pairs), dtype=np.uint32)
for mode in ("identity", "reverse"):
    sel = idx if mode == "identity" else idx[::-1].copy()
    d_idx = torch.from_numpy(sel.view(np.int32)).to(dev)
    kb = sum(len(k) for k, _ in pairs)
    vb = sum(len(v) for _, v in pairs)
    b = lsmgpu.gather_kvs(ctx, d_buf, d_kd, d_vd, d_idx, len(sel), kb, vb)
    torch.cuda.synchronize()
    keys = b"".join(pairs[i][0] for i in sel)
    got = b.keys[:len(keys)].cpu().numpy().tobytes()
    koff = b.koff.cpu().numpy()
    bad = [i for i in range(len(keys)) if got[i] != keys[i]]
    print(mode, "key mismatches", len(bad), "of", len(keys))
    for x in bad[:8]:
        r = int(np.searchsorted(koff, x, side="right")) - 1
        i = sel[r]
        print(f"  byte {x} rec {r} (pair {i}) dst {koff[r]} (dst%4={koff[r] % 4}) len {len(pairs[i][0])} "
              f"src {int(kpos[i])} (src%4={int(kpos[i]) % 4}) wave {r // 64} lane {r % 64} "
              f"got {got[x]} want {keys[x]}")
    vals = b"".join(pairs[i][1] for i in sel)
    gv = b.vals[:len(vals)].cpu().numpy().tobytes()
    print(mode, "value mismatches", sum(1 for i in range(len(vals)) if gv[i] != vals[i]))
