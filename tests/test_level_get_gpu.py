"""GPU parity of lsm_level_get: the batched Get past MayContain --
searchFromTable (sstable/manager.go:209-223): Iterator.Seek over the candidate
table's IndexBlock (sstable/block/index.go:157-181) and GetValueByOffset
(sstable.go:271-296, Value.DecodeFrom kv.go:181-200) -- against the oracle
(ora_level_get, checked against a Python restatement of the Go text in
tests/test_oracle_level_get.py).  Bit-exact: the result code of every probe
and the value view (offset and length) of every hit.
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
    img, _ = ora.build_sst(kb, ko, vb, vo, 0, len(keys), m=m, k=k)
    return img.copy()


def place(rng, images):
    offs, pos, parts = [], 0, []
    for im in images:
        gap = int(rng.integers(0, 23))
        parts += [np.zeros(gap, np.uint8), im]
        pos += gap
        offs.append(pos)
        pos += im.size
    buf = np.concatenate(parts) if parts else np.zeros(16, np.uint8)
    return buf, np.array(offs, np.uint64)


def run(ctx, rng, images, probes):
    """Level search + Get on the GPU against the oracle; -> (res, voff, vlen)."""
    kb, ko = csr(probes)
    batch = lsmgpu.batch_to_device(ctx, kb, ko, np.zeros(1, np.uint8),
                                   np.zeros(len(probes) + 1, np.uint64))
    buf, offs = place(rng, images)
    lens = np.array([im.size for im in images], np.uint64)
    d_img = lsmgpu.to_device_bytes(buf, ctx.torch_device)
    r = lsmgpu.decode_sst(ctx, d_img, offs, lens)
    table, may = lsmgpu.level_may_contain(ctx, d_img, r, batch)
    res0, val0 = lsmgpu.level_get(ctx, d_img, r, batch, table, may)  # bisecting the index
    # through the Seek tree: built for every table, and for a max_nidx below
    # some tables' (they walk the index); the same answers
    tree = lsmgpu.level_get_tree(ctx, d_img, r)
    res, val = lsmgpu.level_get(ctx, d_img, r, batch, table, may, tree=tree)
    if tree.max_nidx > 1:
        part = lsmgpu.level_get_tree(ctx, d_img, r, max_nidx=tree.max_nidx // 2)
        res1, val1 = lsmgpu.level_get(ctx, d_img, r, batch, table, may, tree=part)
        assert torch.equal(res, res1) and torch.equal(val, val1)
    # the level's whole Get in one call (the Seek inside the filter test, the
    # tree's top groups in LDS), with the tree, a partial tree and none
    for tr in (tree, part if tree.max_nidx > 1 else tree, None):
        ft, fm, fr, fv = lsmgpu.level_search_get(ctx, d_img, r, batch, tree=tr)
        assert torch.equal(ft, table) and torch.equal(fm, may)
        assert torch.equal(fr, res) and torch.equal(fv, val)
    torch.cuda.synchronize()
    assert torch.equal(res, res0) and torch.equal(val, val0)
    table, may = table.cpu().numpy(), may.cpu().numpy()
    res = res.cpu().numpy()
    val = val.cpu().numpy().view(lsmgpu.DESC_DTYPE).reshape(-1)
    dec = [ora.sst_decode(im) for im in images]
    wt, wm = ora.level_may_contain(buf, offs, [d[1] for d in dec], kb, ko, 0, len(probes))
    assert np.array_equal(table, wt) and np.array_equal(may, wm)
    wr, wo, wl = ora.level_get(buf, offs, lens, [d[1] for d in dec], [d[2] for d in dec],
                               [d[3] for d in dec], kb, ko, 0, len(probes), wt, wm)
    bad = np.argwhere((res != wr) | (val["rec_off"] != wo) | (val["val_len"] != wl))
    assert bad.size == 0, [(probes[i], res[i], wr[i], val[i], wo[i], wl[i]) for i in bad[:6, 0]]
    assert (val["key_len"] == 0).all()
    found = res == ora.GET_FOUND
    for i in np.flatnonzero(found)[:200]:  # the view holds the value's own bytes
        o, n = int(val["rec_off"][i]), int(val["val_len"][i])
        assert int.from_bytes(buf[o:o + 4].tobytes(), "little") == n
    return res, val


def level(rng, nfile, per=60, pre=b"gk"):
    images, held = [], []
    for f in range(nfile):
        keys = sorted({pre + b"%06d" % (f * 1000 + int(x)) for x in rng.integers(100, 900, per)})
        vals = [b"v%d:" % f + bytes(rng.integers(0, 256, int(rng.integers(0, 40))).astype(np.uint8))
                for _ in keys]
        images.append(build(keys, vals))
        held += keys
    return images, held


def test_get_hits_misses_and_bounds(ctx):
    """Held keys (found, with their own value), absent keys between them,
    below the first MinKey and above the last MaxKey, every MinKey / MaxKey,
    keys one byte longer or shorter than held ones (the equal-key boundary of
    Seek), and the empty key."""
    rng = np.random.default_rng(201)
    images, held = level(rng, 20)
    probes = list(held[::3]) + [b"", b"a", b"gk", b"zzz", b"gk999999"]
    probes += [h + b"\x00" for h in held[::17]] + [h[:-1] for h in held[::13]]
    probes += [b"gk%06d" % int(x) for x in rng.integers(0, 21000, 3000)]
    res, _ = run(ctx, rng, images, probes)
    assert (res == ora.GET_FOUND).sum() > len(held) // 3
    assert (res == ora.GET_ABSENT).sum() > 1000


def test_get_duplicate_keys_and_shared_prefixes(ctx):
    """An index holding equal keys (Seek takes the first), keys that share
    more than 16 bytes (the prefix tie goes to the bytes), zero bytes inside
    keys, empty values."""
    rng = np.random.default_rng(202)
    long = b"p" * 20
    keys = sorted([long + b"%03d" % i for i in range(0, 300, 3)] + [long + b"030"] * 3 +
                  [b"q\x00\x00", b"q\x00\x00\x00", b"q\x00\x01"])
    vals = [b"" if i % 5 == 0 else b"val%d" % i for i in range(len(keys))]
    im = build(keys, vals, m=1 << 14, k=7)
    probes = keys + [long + b"%03d" % i for i in range(300)] + [long, long[:16], b"q", b"q\x00"]
    res, val = run(ctx, rng, [im], probes)
    i = probes.index(long + b"030")
    assert res[i] == ora.GET_FOUND


def test_get_corrupted_offsets(ctx):
    """Index offsets that lead GetValueByOffset astray: negative (the Seek
    fails), at and past the end of the file (the length read fails), onto a
    length above 1<<30 and onto a length longer than the rest of the file."""
    rng = np.random.default_rng(203)
    images, held = level(rng, 4, per=30)
    im = images[1]
    rc, meta, idesc, ival, _ = ora.sst_decode(im)
    assert rc == 0 and meta.nidx >= 8
    n = im.size
    bad_off = {0: -5, 1: n, 2: n - 2, 3: n - 3, 4: int(meta.idx_off), 5: int(meta.data_off)}
    # 4: the index region's first entry read as a value (klen as a length:
    # short reads), 5: patched below to a huge length
    for j, off in bad_off.items():
        at = int(idesc["rec_off"][j]) + 4 + int(idesc["key_len"][j])
        im[at:at + 8] = np.frombuffer(int(off).to_bytes(8, "little", signed=True), np.uint8)
    v0 = int(ival[0])
    dat = int(meta.data_off)
    im[dat:dat + 4] = np.frombuffer(((1 << 30) + 1).to_bytes(4, "little"), np.uint8)
    # entry 6: a value length running past the end of the file
    at6 = int(ival[6])
    im[at6:at6 + 4] = np.frombuffer((n - at6).to_bytes(4, "little"), np.uint8)
    images[1] = im
    keys1 = [im[int(d["rec_off"]) + 4:int(d["rec_off"]) + 4 + int(d["key_len"])].tobytes()
             for d in idesc]
    probes = keys1 + held[::2]
    res, _ = run(ctx, rng, images, probes)
    codes = set(res[:len(keys1)].tolist())
    assert {ora.GET_SEEK_FAILED, ora.GET_VALUE_LENGTH, ora.GET_VALUE_TOO_LONG,
            ora.GET_VALUE_SHORT, ora.GET_FOUND} <= codes, codes
    assert v0 != 0


def test_get_full_level_sample(ctx):
    """A level shaped like the bench's (.sst images of 16-byte "k%015d" keys
    and 100-byte values, go-lsm's filter), held and absent keys interleaved."""
    rng = np.random.default_rng(204)
    from lsmgpu import synth
    n = 40_000
    keys, koff, vals, voff = synth.kv_stream(n)
    starts = lsmgpu.segment_files(ctx, koff, voff, lsmgpu.MAX_SSTABLE_SIZE)
    images = []
    for f in range(len(starts) - 1):
        img, _ = ora.build_sst(keys, koff, vals, voff, int(starts[f]), int(starts[f + 1]))
        images.append(img)
    ids = rng.integers(0, 2 * n, 20_000)
    probes = [synth.keys_for(np.array([i]))[0].tobytes() for i in ids]
    res, _ = run(ctx, rng, images, probes)
    assert (res == ora.GET_FOUND).sum() == int((ids < n).sum())


def test_get_deep_unsorted_index(ctx):
    """Deep tables (n > 2,048: several tree groups) whose index entries are
    NOT sorted: Seek's answer is then whatever Go's bisection path reaches,
    and the tree must take exactly those steps.  One sorted table beside it,
    and keys sharing 18 bytes (prefix ties: the bytes past 16 decide)."""
    rng = np.random.default_rng(205)
    lp = b"shared-prefix-xyz-"
    sk = sorted({lp + b"%07d" % int(x) for x in rng.integers(0, 10 ** 7, 3000)})
    im_sorted = build(sk, [b"s%d" % i for i in range(len(sk))], m=1 << 16, k=5)
    uk = [b"u%06d" % int(x) for x in rng.permutation(5000)[:2600]]  # shuffled
    im_unsorted = build(uk, [b"u%d" % i for i in range(len(uk))], m=1 << 16, k=5)
    probes = sk[::2] + [lp + b"%07d" % int(x) for x in rng.integers(0, 10 ** 7, 2000)]
    probes += uk + [b"u%06d" % int(x) for x in rng.integers(0, 5000, 2000)] + [lp, lp[:16]]
    res, _ = run(ctx, rng, [im_sorted, im_unsorted], probes)
    assert (res[:len(sk[::2])] == ora.GET_FOUND).all()


def test_seek_tree_shapes(ctx):
    """Tables of every size from 0 to 70 entries (every top-block depth
    1-3 and group count up to three), each probed with all its keys and the
    keys between them, against the oracle with and without the tree."""
    rng = np.random.default_rng(206)
    images, probes = [], []
    for n in list(range(1, 18)) + [31, 32, 33, 63, 64, 65, 70]:
        keys = [b"t%03d-%05d" % (n, 10 * x) for x in range(n)]
        images.append(build(keys, [b"%d" % x for x in range(n)], m=2048, k=3))
        probes += keys + [b"t%03d-%05d" % (n, 10 * x + 5) for x in range(-1, n)]
    res, _ = run(ctx, rng, images, probes)
    assert (res == ora.GET_FOUND).sum() == sum(list(range(1, 18)) + [31, 32, 33, 63, 64, 65, 70])


def test_get_other_filter_shapes(ctx):
    """Tables whose filters are not go-lsm's shape (m above 2^21, k above 16:
    the level search passes the full sum256, and the fused Get reads the
    probe's key instead of a stashed prefix) beside go-lsm-shaped ones."""
    rng = np.random.default_rng(207)
    images, held = [], []
    for f in range(6):
        keys = sorted({b"fs%06d" % (f * 1000 + int(x)) for x in rng.integers(100, 900, 80)})
        m, k = ((3_000_000, 20) if f % 2 else (1 << 15, 5))
        images.append(build(keys, [b"v%d" % f] * len(keys), m=m, k=k))
        held += keys
    probes = held[::2] + [b"fs%06d" % int(x) for x in rng.integers(0, 7000, 1500)]
    res, _ = run(ctx, rng, images, probes)
    assert (res[:len(held[::2])] == ora.GET_FOUND).all()
