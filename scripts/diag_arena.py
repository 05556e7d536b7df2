"""Diagnostics: ARENA mismatches vs the oracle on tiny-record KV blocks, for
several alignments and block lengths (LIN vs streamed ring)."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "go-lsm_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import lsmgpu, pyoracle as ora
from test_decode_gpu import rand_records
ctx = lsmgpu.Context(0)
grammar = 1
rng = np.random.default_rng(8)
full = rand_records(rng, grammar, 1500, kmax=8, vmax=8)
for h in range(0, 16, 3):
    for cut in (6000, 8100, 9000, 12000, len(full)):
        st, d, _ = ora.decode_block(grammar, np.frombuffer(full, np.uint8), 0, cut)
        blk = full[:int(d["rec_off"][-1] + 8 + d["key_len"][-1] + d["val_len"][-1])]
        buf = np.zeros(16 + len(blk) + 64, np.uint8); buf[h:h + len(blk)] = np.frombuffer(blk, np.uint8)
        d_in = lsmgpu.to_device_bytes(buf, ctx.torch_device)
        d_off = torch.tensor([h], dtype=torch.int64, device=ctx.torch_device)
        d_len = torch.tensor([len(blk)], dtype=torch.int32, device=ctx.torch_device)
        r = lsmgpu.decode_blocks(ctx, grammar, d_in, d_off, d_len, arena=True, placement="offset")
        torch.cuda.synchronize()
        st, d, _ = ora.decode_block(grammar, buf, h, len(blk))
        ok, ov = ora.materialize(grammar, buf, d)
        ka = r.key_arena.cpu().numpy()[h:h + ok.size]; va = r.val_arena.cpu().numpy()[h:h + ov.size]
        dk = np.nonzero(ka != ok)[0]; dv = np.nonzero(va != ov)[0]
        line = f"h={h} len={len(blk)} nrec={len(d)} kdiff={dk.size} vdiff={dv.size}"
        if dk.size:
            kcum = np.concatenate([[0], np.cumsum(d["key_len"].astype(np.int64))])
            i = int(np.searchsorted(kcum, dk[0], side="right") - 1)
            line += f" first_k_rec={i} rec_off={int(d['rec_off'][i]) - h} stream={int(d['rec_off'][i]) - h + h} kl={int(d['key_len'][i])} bytes={dk[:6].tolist()}"
        if dv.size:
            vcum = np.concatenate([[0], np.cumsum(d["val_len"].astype(np.int64))])
            i = int(np.searchsorted(vcum, dv[0], side="right") - 1)
            line += f" first_v_rec={i} rec_off={int(d['rec_off'][i]) - h} vl={int(d['val_len'][i])}"
        print(line, flush=True)
