"""GPU parity of lsm_level_may_contain: Manager.searchFromLevelWithSparseIndex
(sstable/manager.go:178-207) up to searchFromTable's MayContain (:209-212) --
Go's sort.Search over the level's MinKeys, index-- when > 0, then
SSTable.MayContain (sstable.go:300-305) of that one table -- against the
oracle (ora_level_may_contain, itself checked against a Python restatement
of the Go text in tests/test_oracle_may_contain.py).  Bit-exact: the
candidate table and the may bit of every probe.
"""
import struct

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


def build(keys, m, k):
    kb, ko = csr(keys)
    vb, vo = csr([b"v" * (len(x) % 7) for x in keys])
    img, _ = ora.build_sst(kb, ko, vb, vo, 0, len(keys), m=m, k=k)
    return img


def bounds(img):
    rc, meta, *_ = ora.sst_decode(img)
    return (img[meta.min_key_off:meta.min_key_off + meta.min_key_len].tobytes(),
            img[meta.max_key_off:meta.max_key_off + meta.max_key_len].tobytes())


def check(ctx, rng, images, probes):
    """Images at odd offsets in one buffer, decoded on the GPU; the level
    search of every probe against the oracle.  -> (table, may)."""
    kb, ko = csr(probes)
    batch = lsmgpu.batch_to_device(ctx, kb, ko, np.zeros(1, np.uint8),
                                   np.zeros(len(probes) + 1, np.uint64))
    if images:
        offs, pos, parts = [], 0, []
        for im in images:
            gap = int(rng.integers(0, 23))
            parts += [np.zeros(gap, np.uint8), im]
            pos += gap
            offs.append(pos)
            pos += im.size
        buf = np.concatenate(parts)
        offs = np.array(offs, np.uint64)
    else:
        buf, offs = np.zeros(16, np.uint8), np.zeros(0, np.uint64)
    d_img = lsmgpu.to_device_bytes(buf, ctx.torch_device)
    r = lsmgpu.decode_sst(ctx, d_img, offs, np.array([im.size for im in images], np.uint64))
    table, may = lsmgpu.level_may_contain(ctx, d_img, r, batch)
    # the same search over the level's sparse index built beforehand
    # (lsm_level_index_build + lsm_level_may_contain_indexed)
    index = lsmgpu.level_index(ctx, d_img, r)
    t2 = torch.full_like(table, -7)
    m2 = torch.full_like(may, 7)
    if batch.n:
        lsmgpu.level_may_contain_into(ctx, d_img, r, batch, t2, m2, index=index)
    torch.cuda.synchronize()
    assert torch.equal(t2, table) and torch.equal(m2, may), "indexed search differs"
    table, may = table.cpu().numpy(), may.cpu().numpy()
    metas = [ora.sst_decode(im)[1] for im in images]
    wt, wm = ora.level_may_contain(buf, offs, metas, kb, ko, 0, len(probes))
    bad = np.argwhere((table != wt) | (may != wm))
    assert bad.size == 0, [(probes[i], table[i], wt[i], may[i], wm[i]) for i in bad[:6, 0]]
    return table, may


def sorted_level(rng, nfile, m=2048, k=3, per=40, pre=b"lv"):
    images = []
    for f in range(nfile):
        keys = sorted({pre + b"%06d" % (f * 1000 + int(x)) for x in rng.integers(100, 900, per)})
        images.append(build(keys, m=m, k=k))
    return images


def test_level_search_edges(ctx):
    """The verdict's cases: a key below the first MinKey (candidate 0, no
    hit), a key equal to a MinKey and to a MaxKey, a key above the last
    MaxKey (the last table, no hit), keys in the gaps, held keys, and the
    empty level (candidate -1)."""
    rng = np.random.default_rng(101)
    images = sorted_level(rng, 24)
    bnd = [bounds(im) for im in images]
    probes = [b"", b"a", b"lv", b"lv000000", b"lv000099"]             # below the first MinKey
    probes += [b for pair in bnd for b in pair]                          # every MinKey / MaxKey
    probes += [mx + b"\x00" for _, mx in bnd] + [b"zzz", b"lv999999"]   # gaps, above the last MaxKey
    probes += [b"lv%06d" % int(x) for x in rng.integers(0, 25000, 3000)]
    table, may = check(ctx, rng, images, probes)
    assert table[0] == 0 and may[0] == 0                                 # below: index 0, MinKey > key
    assert table[probes.index(bnd[5][0])] == 5 and may[probes.index(bnd[5][0])] == 1
    assert table[probes.index(b"zzz")] == 23 and may[probes.index(b"zzz")] == 0
    assert may.sum() > 100
    table, may = check(ctx, rng, [], probes)                             # the empty level
    assert (table == -1).all() and (may == 0).all()


def test_level_search_equal_minkeys_and_unsorted(ctx):
    """Tables with equal MinKeys (sort.Search lands after the last of them),
    and a level whose MinKeys are out of order (Go's exact bisection order
    decides the candidate; the kernel must run the same steps)."""
    rng = np.random.default_rng(102)
    images = sorted_level(rng, 12)
    mn = bounds(images[6])[0]
    twin = build([mn, mn + b"\x01", mn + b"\x02"], m=512, k=2)
    dup = images[:6] + [twin] + images[6:]
    probes = [b"lv%06d" % int(x) for x in rng.integers(0, 13000, 1500)]
    probes += [mn, mn + b"\x01", mn + b"\x03", b""]
    check(ctx, rng, dup, probes)
    perm = [5, 0, 9, 2, 11, 7, 1, 10, 3, 8, 4, 6]
    check(ctx, rng, [images[i] for i in perm], probes)


def test_level_search_failed_tables(ctx):
    """A table whose header fails (searched as MinKey "", answers 0) and one
    whose filter fails (searched by its MinKey, answers 0), among intact
    tables; k = 0 (Test true) and m = 0 < k (answered 0)."""
    rng = np.random.default_rng(103)
    images = sorted_level(rng, 10)
    hdr_bad = build([b"lv004500"], m=64, k=2).copy()
    hdr_bad[:4] = np.frombuffer(struct.pack("<I", 10 ** 6), np.uint8)
    flt_bad = images[7].copy()
    mnl = int(np.frombuffer(flt_bad[:4].tobytes(), "<u4")[0])
    mxl = int(np.frombuffer(flt_bad[4 + mnl:8 + mnl].tobytes(), "<u4")[0])
    at = 8 + mnl + mxl + 8 + 16
    flt_bad[at:at + 8] = np.frombuffer(struct.pack(">Q", (1 << 64) - 1), np.uint8)
    k0 = build([b"lv003200", b"lv003800"], m=64, k=1).copy()
    at0 = 8 + 2 * 8 + 8
    k0[at0 + 8:at0 + 16] = np.frombuffer(struct.pack(">Q", 0), np.uint8)   # k = 0
    m0 = build([b"lv002200", b"lv002800"], m=64, k=2).copy()
    m0[at0:at0 + 8] = np.frombuffer(struct.pack(">Q", 0), np.uint8)        # m = 0 < k
    level = images[:2] + [m0] + images[2:3] + [k0] + images[3:5] + [hdr_bad] + images[5:7] + \
        [flt_bad] + images[8:]
    probes = [b"lv%06d" % int(x) for x in rng.integers(0, 11000, 2500)] + [b"", b"lv004500"]
    check(ctx, rng, level, probes)


def test_level_search_production_filters(ctx):
    """go-lsm's filter (m = 1.6M bits, k = 16: the LDS copy and its L2 tail),
    40 tables, 120k probes: many classify workgroups feed every table."""
    rng = np.random.default_rng(104)
    images = []
    for f in range(40):
        keys = sorted({b"P%08d" % (f * 100000 + int(x)) for x in rng.integers(0, 90000, 2500)})
        images.append(build(keys, m=1_600_000, k=16))
    held = [b"P%08d" % (f * 100000 + int(x)) for f in range(40) for x in rng.integers(0, 90000, 8)]
    probes = held + [b"P%08d" % int(x) for x in rng.integers(0, 4_100_000, 120_000)]
    table, may = check(ctx, rng, images, probes)
    assert may.sum() > 0.01 * len(probes)


def test_level_search_many_tables_fallback(ctx):
    """More tables than the LDS search holds (2,048): the per-probe kernel."""
    rng = np.random.default_rng(105)
    images = [build([b"T%06d" % (3 * f), b"T%06d" % (3 * f + 1)], m=64, k=1) for f in range(2100)]
    probes = [b"T%06d" % int(x) for x in rng.integers(0, 6400, 4000)] + [b"", b"U"]
    check(ctx, rng, images, probes)


def test_level_search_two_passes(ctx):
    """More probes than one pass (1,024 workgroups x 2,048 probes): the
    second pass's outputs land at its own offsets."""
    rng = np.random.default_rng(106)
    images = sorted_level(rng, 16, m=4096, k=3, per=200, pre=b"Q")
    n = 2 * 1024 * 2048 + 12345
    x = rng.integers(0, 17000, n)
    probes = [b"Q%06d" % int(v) for v in x]
    check(ctx, rng, images, probes)


def test_level_search_mixed_filter_shapes(ctx):
    """Tables whose filters take the 16-byte hash record (m <= 2^21, k <= 16)
    beside tables that take the full sum256 (m just above 2^21, k = 20) in one
    level: both record kinds and both test paths in one call."""
    rng = np.random.default_rng(105)
    shapes = [(2048, 4), (3_000_000, 7), (4096, 20), (1_600_000, 16), (1 << 21, 16), ((1 << 21) + 1, 3),
              (64, 17), (700_000, 9)]
    images, held = [], []
    for f, (m, k) in enumerate(shapes):
        keys = sorted({b"X%07d" % (f * 100000 + int(x)) for x in rng.integers(0, 90000, 600)})
        images.append(build(keys, m=m, k=k))
        held += keys[::40]
    probes = held + [b"X%07d" % int(x) for x in rng.integers(0, 850_000, 20_000)] + [b"", b"Y"]
    table, may = check(ctx, rng, images, probes)
    assert may[:len(held)].all()
