"""GPU parity of lsm_level0_get: the batched Get of level 0 --
Manager.searchFromLevel0 (sstable/manager.go:160-176) running searchFromTable
(:209-223) over every table in order, newest first -- against the oracle
(ora_level0_get, checked against a Python restatement of the Go text in
tests/test_oracle_level_get.py).  Bit-exact: the answering table, the result
code and the value view of every probe.
"""
import numpy as np
import pytest
import torch

import lsmgpu
import pyoracle as ora

pytestmark = pytest.mark.gpu


def csr(items):
    data = b"".join(items)
    off = np.zeros(len(items) + 1, np.uint64)
    off[1:] = np.cumsum([len(x) for x in items])
    return np.frombuffer(data, np.uint8) if data else np.zeros(0, np.uint8), off


def build(keys, vals, m=4096, k=4):
    kb, ko = csr(keys)
    vb, vo = csr(vals)
    img, _ = ora.build_sst(kb if kb.size else np.zeros(1, np.uint8), ko,
                           vb if vb.size else np.zeros(1, np.uint8), vo, 0, len(keys), m=m, k=k)
    return img.copy()


def place(rng, images):
    offs, pos, parts = [], 0, []
    for im in images:
        gap = int(rng.integers(0, 23))
        parts += [np.zeros(gap, np.uint8), im]
        pos += gap
        offs.append(pos)
        pos += im.size
    buf = np.concatenate(parts + [np.zeros(16, np.uint8)])
    return buf, np.array(offs, np.uint64)


def run(ctx, rng, images, probes):
    """Level-0 Get on the GPU (with and without the Seek tree) against the
    oracle; -> (table, res, val)."""
    kb, ko = csr(probes)
    batch = lsmgpu.batch_to_device(ctx, kb if kb.size else np.zeros(1, np.uint8), ko,
                                   np.zeros(1, np.uint8), np.zeros(len(probes) + 1, np.uint64))
    buf, offs = place(rng, images)
    lens = np.array([im.size for im in images], np.uint64)
    d_img = lsmgpu.to_device_bytes(buf, ctx.torch_device)
    r = lsmgpu.decode_sst(ctx, d_img, offs, lens)
    t0, res0, val0 = lsmgpu.level0_get(ctx, d_img, r, batch)  # bisecting the index
    tree = lsmgpu.level_get_tree(ctx, d_img, r)
    t1, res, val = lsmgpu.level0_get(ctx, d_img, r, batch, tree=tree)
    if tree.max_nidx > 1:
        part = lsmgpu.level_get_tree(ctx, d_img, r, max_nidx=tree.max_nidx // 2)
        t2, res2, val2 = lsmgpu.level0_get(ctx, d_img, r, batch, tree=part)
        assert torch.equal(t1, t2) and torch.equal(res, res2) and torch.equal(val, val2)
    torch.cuda.synchronize()
    assert torch.equal(t0, t1) and torch.equal(res, res0) and torch.equal(val, val0)
    table = t1.cpu().numpy()
    res = res.cpu().numpy()
    val = val.cpu().numpy().view(lsmgpu.DESC_DTYPE).reshape(-1)
    dec = [ora.sst_decode(im) for im in images]
    wt, wr, wo, wl = ora.level0_get(buf, offs, lens, [d[1] for d in dec], [d[2] for d in dec],
                                    [d[3] for d in dec], kb if kb.size else np.zeros(1, np.uint8), ko,
                                    0, len(probes))
    bad = np.argwhere((table != wt) | (res != wr) | (val["rec_off"] != wo) | (val["val_len"] != wl))
    assert bad.size == 0, [(probes[i], table[i], wt[i], res[i], wr[i], val[i], wo[i], wl[i])
                           for i in bad[:6, 0]]
    assert (val["key_len"] == 0).all()
    return table, res, val


def test_level0_newest_wins_and_false_positives(ctx):
    """Three overlapping tables, newest first: a key held by two tables is
    answered by the newer one with its own value; tiny filters in the newer
    tables pass keys they do not hold (false positives), and the Seek miss
    moves on to the older table that holds them."""
    rng = np.random.default_rng(301)
    all_keys = [b"key%05d" % i for i in range(3000)]
    sets = [sorted(set(rng.choice(3000, 900, replace=False).tolist())) for _ in range(3)]
    images, held = [], set()
    for t, s in enumerate(sets):
        keys = [all_keys[i] for i in s]
        vals = [b"t%d-%d" % (t, i) for i in s]
        m, k = (256, 2) if t < 2 else (1 << 16, 6)  # the newer tables' filters pass most keys
        images.append(build(keys, vals, m=m, k=k))
        held |= set(keys)
    probes = all_keys + [b"", b"zzz", b"key", b"key00000\x00"]
    table, res, val = run(ctx, rng, images, probes)
    both = set(all_keys[i] for i in sets[0]) & set(all_keys[i] for i in sets[1])
    i = probes.index(sorted(both)[0])
    assert table[i] == 0 and res[i] == ora.GET_FOUND
    only_old = [p for p in all_keys if p in set(all_keys[i] for i in sets[2])
                and p not in set(all_keys[i] for i in sets[0]) | set(all_keys[i] for i in sets[1])]
    j = probes.index(only_old[0])
    assert table[j] == 2 and res[j] == ora.GET_FOUND
    assert (res == ora.GET_FOUND).sum() == len(held)


def test_level0_error_in_newer_table_ends_the_search(ctx):
    """A corrupted value offset in the newest table: its error is the answer
    even when an older table holds the key (searchFromLevel0 returns the
    error), and the other error codes surface the same way."""
    rng = np.random.default_rng(302)
    keys = [b"e%04d" % i for i in range(0, 400, 2)]
    im0 = build(keys, [b"new%d" % i for i in range(len(keys))], m=1 << 14, k=5)
    im1 = build(keys, [b"old%d" % i for i in range(len(keys))], m=1 << 14, k=5)
    rc, meta, idesc, ival, _ = ora.sst_decode(im0)
    n = im0.size
    for j, off in {0: -5, 1: n, 2: n - 2, 3: int(meta.idx_off)}.items():
        at = int(idesc["rec_off"][j]) + 4 + int(idesc["key_len"][j])
        im0[at:at + 8] = np.frombuffer(int(off).to_bytes(8, "little", signed=True), np.uint8)
    probes = keys + [b"e%04d" % i for i in range(1, 400, 2)]
    table, res, _ = run(ctx, rng, [im0, im1], probes)
    assert res[0] == ora.GET_SEEK_FAILED and table[0] == 0
    assert set(res[:4].tolist()) >= {ora.GET_SEEK_FAILED, ora.GET_VALUE_LENGTH}
    assert (res[4:len(keys)] == ora.GET_FOUND).all() and (table[4:len(keys)] == 0).all()
    assert (table[len(keys):] == -1).all()


def test_level0_empty_tables_and_empty_level(ctx):
    """A table with no records between two others, and a level with no
    tables at all (every probe absent, table -1)."""
    rng = np.random.default_rng(303)
    a = build([b"a1", b"a3", b"a5"], [b"x", b"", b"z"])
    e = build([], [])
    b = build([b"a2", b"a3", b"a9"], [b"q", b"w", b"e"])
    probes = [b"a1", b"a2", b"a3", b"a4", b"a9", b"", b"b"]
    table, res, _ = run(ctx, rng, [a, e, b], probes)
    assert table.tolist() == [0, 2, 0, -1, 2, -1, -1]
    kb, ko = csr(probes)
    batch = lsmgpu.batch_to_device(ctx, kb, ko, np.zeros(1, np.uint8), np.zeros(len(probes) + 1, np.uint64))
    d_img = torch.zeros(16, dtype=torch.uint8, device=ctx.torch_device)
    r = lsmgpu.decode_sst(ctx, d_img, np.zeros(0, np.uint64), np.zeros(0, np.uint64))
    t, res, _ = lsmgpu.level0_get(ctx, d_img, r, batch)
    torch.cuda.synchronize()
    assert (t.cpu().numpy() == -1).all() and (res.cpu().numpy() == ora.GET_ABSENT).all()


def test_level0_bench_shape_sample(ctx):
    """The bench's level 0 at reduced size: three tables of 16-byte keys and
    100-byte values (go-lsm's filter), overlapping strides of one key space,
    held and absent probes interleaved."""
    from lsmgpu import synth
    rng = np.random.default_rng(304)
    n = 6000
    images = []
    for t in range(3):
        ids = np.arange(t, 3 * n, 2)[:n]  # table t holds ids t, t+2, ... (overlapping)
        keys = [synth.keys_for(np.array([i]))[0].tobytes() for i in ids]
        vals = [bytes([t]) * 100 for _ in ids]
        images.append(build(keys, vals, m=1_600_000, k=16))
    probes = [synth.keys_for(np.array([i]))[0].tobytes() for i in rng.integers(0, 4 * n, 20_000)]
    table, res, _ = run(ctx, rng, images, probes)
    assert (res == ora.GET_FOUND).sum() > 5000


def test_level_get_tree_size_checked(ctx):
    """lsm_level_get / lsm_level0_get refuse a Seek tree smaller than the
    level's shape (one built for fewer tables): LSM_ESPACE, nothing read."""
    rng = np.random.default_rng(305)
    images = [build([b"k%03d" % i for i in range(50)], [b"v"] * 50) for _ in range(3)]
    buf, offs = place(rng, images)
    lens = np.array([im.size for im in images], np.uint64)
    d_img = lsmgpu.to_device_bytes(buf, ctx.torch_device)
    r = lsmgpu.decode_sst(ctx, d_img, offs, lens)
    tree = lsmgpu.level_get_tree(ctx, d_img, r)
    short = lsmgpu.SeekTree(tree.data[:tree.data.numel() // 2], tree.max_nidx)
    kb, ko = csr([b"k001", b"k777"])
    batch = lsmgpu.batch_to_device(ctx, kb, ko, np.zeros(1, np.uint8), np.zeros(3, np.uint64))
    with pytest.raises(RuntimeError, match="code -4"):
        lsmgpu.level0_get(ctx, d_img, r, batch, tree=short)
    table, may = lsmgpu.level_may_contain(ctx, d_img, r, batch)
    with pytest.raises(RuntimeError, match="code -4"):
        lsmgpu.level_get(ctx, d_img, r, batch, table, may, tree=short)
