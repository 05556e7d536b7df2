"""Diagnostic: per-segment WAL replay tables against the true chain, for a
library built with -DLSM_WAL_SEG_KIB=K (env SEG_KIB).  For every segment and
phase whose entry is a true record start, the chain's record count and exit
must match the serial chase's; mismatches are printed."""
import bisect, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "go-lsm_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import lsmgpu  # noqa: E402
import pyoracle as ora  # noqa: E402
from lsmgpu import synth  # noqa: E402
SEG = int(os.environ.get("SEG_KIB", "16")) * 1024
ctx = lsmgpu.Context(0)
dev = ctx.torch_device
buf0, off0, ln0, _ = synth.wal_logs(3, memtable_bytes=96 * 1024)
logs = [buf0[o:o + l].tobytes() for o, l in zip(off0, ln0)]
offs, pos, parts = [], 0, []
for lg in logs:  # as tests/test_wal_gpu.py packs them
    offs.append(pos)
    pad = (16 - len(lg) % 16) % 16 + 16
    parts += [np.frombuffer(lg, np.uint8), np.zeros(pad, np.uint8)]
    pos += len(lg) + pad
buf = np.concatenate(parts)
d = lsmgpu.to_device_bytes(buf, dev)
o = torch.tensor(np.array(offs, np.uint64).view(np.int64), device=dev)
lens = [len(x) for x in logs]
l = torch.tensor(np.array(lens, np.uint32).view(np.int32), device=dev)
mx = max(lens)
r = lsmgpu.alloc_decode_offset(ctx, lsmgpu.GRAMMAR_KV, len(logs), int(d.numel()))
ws = lsmgpu.wal_workspace(ctx, len(logs), mx)
lsmgpu.wal_replay_into(ctx, d, o, l, mx, r, ws)
torch.cuda.synchronize()
segs = (mx + SEG - 1) // SEG
slots = SEG // 8 + 1
n = len(logs) * segs
w8 = ws.cpu().numpy()
tab = w8[n * 2 * slots * 16: n * 2 * slots * 16 + n * 2 * 16].view(np.uint32).reshape(len(logs), segs, 2, 4)
fin = w8[n * 2 * (slots * 16 + 16): n * 2 * (slots * 16 + 16) + n * 8].view(np.uint32).reshape(len(logs), segs, 2)
print("SEG", SEG, "segs", segs, "nrec", r.nrec.cpu().numpy(), "status", r.status.cpu().numpy())
for w in range(len(logs)):
    st, od, _ = ora.decode_block(lsmgpu.GRAMMAR_KV, buf, offs[w], lens[w])
    starts = sorted((od["rec_off"] - offs[w]).tolist())
    L = lens[w]
    print("log", w, "len", L, "true records", len(starts))
    bad = 0
    for s in range(segs):
        E = min((s + 1) * SEG, L)
        for ph in range(2):
            entry, ex, nr, stt = (int(x) for x in tab[w, s, ph])
            if entry >= L or entry not in starts:
                continue
            i0 = bisect.bisect_left(starts, entry)
            i1 = bisect.bisect_left(starts, E)
            tex = starts[i1] if i1 < len(starts) else L
            if nr != i1 - i0 or ex != tex or stt != 0:
                bad += 1
                if bad <= 6:
                    print(f"  seg {s} ph {ph}: entry {entry} got (exit {ex}, nrec {nr}, st {stt})"
                          f" want (exit {tex}, nrec {i1 - i0})  fin {fin[w, s].tolist()}")
    print("  bad chains:", bad, " fin pre/cnt first segs:", fin[w, :4].tolist())
