"""Diagnostic: at the get0 bench's level 0 (3 overlapping tables, 1M probes),
the time of lsm_level0_get against lsm_may_contain over the same tables (the
grouped MayContain with LDS-staged filters).  Usage: python tools/l0_mc_time.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "go-lsm_amd")]
import lsmgpu  # noqa: E402
from lsmgpu import synth  # noqa: E402
import bench_sstdec as B  # noqa: E402


def timed(fn, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


ctx = lsmgpu.Context(0)
dev = ctx.torch_device
tabs = B.level0_tables(0)
imgs, offs, lens, pos = [], [], [], 0
for ids, vals in tabs:
    n = ids.size
    batch = lsmgpu.batch_to_device(ctx, synth.keys_for(ids).reshape(-1), np.arange(n + 1, dtype=np.uint64) * np.uint64(16),
                                   vals.reshape(-1).copy(), np.arange(n + 1, dtype=np.uint64) * np.uint64(synth.VAL_LEN))
    sb = lsmgpu.build_sst(ctx, batch, np.array([0, n], np.uint64))
    torch.cuda.synchronize()
    size = int(sb.file_size[0])
    imgs.append(sb.out[:size]); offs.append(pos); lens.append(size)
    pos += (size + 15) // 16 * 16
d_img = torch.zeros(pos + 64, dtype=torch.uint8, device=dev)
for im, o in zip(imgs, offs):
    d_img[o:o + im.numel()] = im
r = lsmgpu.decode_sst(ctx, d_img, np.array(offs, np.uint64), np.array(lens, np.uint64))
tree = lsmgpu.level_get_tree(ctx, d_img, r)
nprobe = 1 << 20
rng = np.random.default_rng(5)
union = np.unique(np.concatenate([t[0] for t in tabs]))
missing = np.setdiff1d(np.arange(40_000), union)
ids = rng.permutation(np.concatenate([rng.choice(union, nprobe // 2), rng.choice(missing, nprobe // 4),
                                      rng.integers(10 ** 12, 10 ** 13, nprobe - nprobe // 2 - nprobe // 4)]))
probes = lsmgpu.batch_to_device(ctx, synth.keys_for(ids).reshape(-1), np.arange(nprobe + 1, dtype=np.uint64) * np.uint64(16),
                                np.zeros(1, np.uint8), np.zeros(nprobe + 1, np.uint64))
table = torch.empty(nprobe, dtype=torch.int32, device=dev)
result = torch.empty(nprobe, dtype=torch.int32, device=dev)
value = torch.empty((nprobe, 4), dtype=torch.int32, device=dev)
hit = torch.zeros((nprobe, 3), dtype=torch.uint8, device=dev)
print("level0_get ms", round(timed(lambda: lsmgpu.level0_get_into(ctx, d_img, r, probes, table, result, value, tree=tree)), 4))
print("may_contain ms", round(timed(lambda: lsmgpu.may_contain_into(ctx, d_img, r, probes, hit)), 4))
print("hits per table", hit.sum(0).tolist())
