"""GPU parity of lsm_may_contain (batched SSTable.MayContain, sstable.go:300-305;
SURVEY.md §8(f) row f3) against the oracle: the range check in Go string
order (Python bytes order is the same) and Filter.Test (bloom.go:371-379) of
the filter block decoded by the oracle (ora_filter_decode + ora_bloom_test).
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


_DECODED = {}


def _file(img):
    """(meta, min key, max key, filter, stored bits) of an image, decoded once."""
    kid = (id(img), img.size)
    if kid not in _DECODED:
        rc, meta, *_ = ora.sst_decode(img)
        mn = img[meta.min_key_off:meta.min_key_off + meta.min_key_len].tobytes()
        mx = img[meta.max_key_off:meta.max_key_off + meta.max_key_len].tobytes()
        f = nbits = None
        if meta.stage not in (1, 2):
            hdr = 8 + meta.min_key_len + meta.max_key_len
            f, nbits, _ = ora.Bloom.decode(img[hdr:])
        _DECODED[kid] = (img, meta, mn, mx, f, nbits)  # img kept alive: id() stays unique
    return _DECODED[kid][1:]


def expected(img, key):
    """SSTable.MayContain (sstable.go:300-305) of a decoded image: the range
    check, then Filter.Test of the decoded filter (bits past the stored bit
    count read 0).  Where Go panics (m == 0 < k: location() divides by zero)
    the ABI answers 0."""
    meta, mn, mx, f, nbits = _file(img)
    if meta.stage in (1, 2):
        return 0
    if mn > key or mx < key:
        return 0
    r = f.test_decoded(key)
    return 0 if r < 0 else r


def test_may_contain_vs_oracle(ctx):
    rng = np.random.default_rng(21)
    images, present = [], []
    for f in range(6):  # disjoint, sorted key ranges (level >= 1 files)
        keys = sorted({b"user%06d" % int(x) for x in rng.integers(f * 1000, f * 1000 + 1000, 300)})
        images.append(build(keys, m=2048, k=3))  # small filter: false positives occur
        present += keys
    # overlapping range, variable-length keys with shared prefixes (L0-like)
    keys = sorted({b"user%06d" % int(x) + b"x" * int(rng.integers(0, 30)) for x in rng.integers(0, 6000, 200)})
    images.append(build(keys, m=1_600_000, k=16))
    present += keys
    images.append(build([], m=1024, k=2))                              # empty table
    images.append(build([b"a"], m=64, k=0))                            # k = 0: Test is true
    bad = build([b"q"], m=64, k=2).copy()
    bad[:4] = np.frombuffer(struct.pack("<I", 10 ** 6), np.uint8)
    images.append(bad)                                                 # header fails: 0
    probes = list(present[::3])
    probes += [b"user%06d" % int(x) for x in rng.integers(0, 7000, 600)]
    probes += [b"", b"user", b"user000000", b"user000000\x00", b"user005999", b"zzzz", b"a", b"q",
               b"user%06d" % 999 + b"x" * 40]
    # nfile = 10 (byte write-out) and 8 (dword write-out)
    for subset in (images, images[:8]):
        check(ctx, rng, subset, probes)


def check(ctx, rng, images, probes, held_check=True):
    # images at odd offsets in one buffer
    offs, pos, parts = [], 0, []
    for im in images:
        gap = int(rng.integers(0, 23))
        parts += [np.zeros(gap, np.uint8), im]
        pos += gap
        offs.append(pos)
        pos += im.size
    buf = np.concatenate(parts)
    d_img = lsmgpu.to_device_bytes(buf, ctx.torch_device)
    r = lsmgpu.decode_sst(ctx, d_img, np.array(offs, np.uint64),
                          np.array([im.size for im in images], np.uint64))
    kb, ko = csr(probes)
    batch = lsmgpu.batch_to_device(ctx, kb, ko, np.zeros(1, np.uint8), np.zeros(len(probes) + 1, np.uint64))
    hit = lsmgpu.may_contain(ctx, d_img, r, batch).cpu().numpy()
    torch.cuda.synchronize()
    checked = 0
    for f, im in enumerate(images):
        for i, key in enumerate(probes):
            want = expected(im, key)
            if want is None:
                continue
            assert hit[i, f] == want, (f, key, hit[i, f], want)
            checked += 1
    assert checked > 0.9 * len(images) * len(probes)
    # no false negatives for the keys each file holds (intact files only)
    for f, im in enumerate(images[:7] if held_check else []):
        rc, meta, idesc, _, _ = ora.sst_decode(im)
        held = {im[d["rec_off"] + 4:d["rec_off"] + 4 + d["key_len"]].tobytes() for d in idesc}
        for i, key in enumerate(probes):
            if key in held:
                assert hit[i, f] == 1


def test_may_contain_many_files(ctx):
    """More than one 128-file tile, nfile % 4 != 0 and == 0, keys shared by
    several overlapping files."""
    rng = np.random.default_rng(33)
    images = []
    for f in range(136):
        lo = int(rng.integers(0, 5000))
        keys = sorted({b"k%05d" % int(x) for x in rng.integers(lo, lo + 400, 40)})
        images.append(build(keys, m=512, k=2))
    probes = [b"k%05d" % int(x) for x in rng.integers(0, 5500, 300)] + [b"", b"z"]
    for subset in (images, images[:135]):
        check(ctx, rng, subset, probes)


def test_may_contain_sorted_disjoint_files(ctx):
    """Level >= 1 shape: files in key order with disjoint ranges (the tile
    binary search), over two tiles; probes at the exact bounds, in the gaps
    between files, before the first and after the last file."""
    rng = np.random.default_rng(44)
    images, bounds = [], []
    for f in range(70):
        keys = sorted({b"s%06d" % (f * 1000 + int(x)) + b"x" * int(x % 3) for x in rng.integers(0, 900, 30)})
        images.append(build(keys, m=2048, k=4))
        bounds += [keys[0], keys[-1]]
    probes = bounds + [b"s%06d" % int(x) for x in rng.integers(0, 72000, 400)]
    probes += [b"", b"r", b"s", b"t", b"s%06d" % 69950 + b"\x00"]
    check(ctx, rng, images, probes)
    check(ctx, rng, images[:64], probes)


def test_may_contain_sorted_large_filters(ctx):
    """Grouped path with the production filter (m = 1.6M bits, k = 16: all
    four LDS parts hold stored words), files at odd offsets, probes held,
    in the gaps and outside the level."""
    rng = np.random.default_rng(55)
    images = []
    for f in range(5):
        keys = sorted({b"L%07d" % (f * 10000 + int(x)) for x in rng.integers(0, 9000, 400)})
        images.append(build(keys, m=1_600_000, k=16))
    probes = [b"L%07d" % int(x) for x in rng.integers(0, 52000, 3000)] + [b"", b"L", b"M"]
    check(ctx, rng, images, probes)


def test_may_contain_sorted_mixed_filter_shapes(ctx):
    """Grouped path with files whose filters take the 16-byte hash record
    (m <= 2^21, k <= 16) beside files that take the full sum256 (m just above
    2^21, k = 20): both record kinds and both test paths in one call."""
    rng = np.random.default_rng(56)
    shapes = [(2048, 4), (3_000_000, 7), (4096, 20), (1_600_000, 16), (1 << 21, 16), ((1 << 21) + 1, 3),
              (64, 17), (700_000, 9)]
    images = []
    for f, (m, k) in enumerate(shapes):
        keys = sorted({b"X%07d" % (f * 10000 + int(x)) for x in rng.integers(0, 9000, 300)})
        images.append(build(keys, m=m, k=k))
    probes = [b"X%07d" % int(x) for x in rng.integers(0, 85000, 3000)] + [b"", b"X", b"Y"]
    check(ctx, rng, images, probes)


def test_may_contain_sorted_shared_long_prefixes(ctx):
    """Grouped path where every bound shares its first 16+ bytes (the LDS
    bound prefixes tie and the byte comparison decides): keys "tenant-...-/"
    + a counter, files disjoint and in order; probes at the bounds, between
    files, equal to the shared prefix, one byte longer or shorter."""
    rng = np.random.default_rng(66)
    pre = b"tenant-00000000000/"  # 19 bytes
    images, bounds = [], []
    for f in range(40):
        keys = sorted({pre + b"%06d" % (f * 1000 + int(x)) for x in rng.integers(0, 900, 25)})
        images.append(build(keys, m=4096, k=3))
        bounds += [keys[0], keys[-1]]
    probes = bounds + [pre + b"%06d" % int(x) for x in rng.integers(0, 41000, 500)]
    probes += [pre, pre[:16], pre[:15], pre + b"\x00", pre[:16] + b"\xff", pre + b"999999", b""]
    probes += [pre[:16] + b"%09d" % int(x) for x in rng.integers(0, 10**9, 50)]  # ties, then bytes
    assert all(bounds[i] < bounds[i + 1] for i in range(len(bounds) - 1))  # sorted, disjoint
    check(ctx, rng, images, probes)


def _patch_nbits(img, nbits):
    """The image with its stored bitset length (the u64be after m and k,
    bloom.go:239-250 / bitset.ReadFrom) lowered: the filter block keeps its
    length prefix, so the .sst framing is unchanged and only the bits at and
    past nbits read as 0 (bitset.Test past its length)."""
    img = img.copy()
    mnl = int(np.frombuffer(img[:4].tobytes(), "<u4")[0])
    mxl = int(np.frombuffer(img[4 + mnl:8 + mnl].tobytes(), "<u4")[0])
    at = 8 + mnl + mxl + 8 + 16
    img[at:at + 8] = np.frombuffer(struct.pack(">Q", nbits), np.uint8)
    return img


def _patch_min_key(img, new_min):
    """Overwrite the header's MinKey bytes (same length): a file that decodes
    cleanly with MinKey > MaxKey."""
    img = img.copy()
    assert int(np.frombuffer(img[:4].tobytes(), "<u4")[0]) == len(new_min)
    img[4:4 + len(new_min)] = np.frombuffer(new_min, np.uint8)
    return img


def test_may_contain_min_greater_than_max_header(ctx):
    """F0=[a,b], F1=[z,c] (corrupted MinKey > MaxKey), F2=[d,e].
    The bound sequence is not sorted, so the grouped path must not be taken;
    "dd" is in F2's range and Go tests F2's filter."""
    rng = np.random.default_rng(5)
    f0 = build([b"a", b"ab", b"b"], m=4096, k=3)
    f1 = _patch_min_key(build([b"c"], m=4096, k=3), b"z")
    f2 = build([b"d", b"dd", b"e"], m=4096, k=3)
    probes = [b"a", b"b", b"c", b"d", b"dd", b"de", b"e", b"z", b"zz", b"", b"aa"]
    check(ctx, rng, [f0, f1, f2], probes, held_check=False)
    # the same shape inside a larger, otherwise sorted and disjoint level
    imgs = [build([b"k%03d_%d" % (i, j) for j in range(4)], m=2048, k=2) for i in range(9)]
    imgs[4] = _patch_min_key(imgs[4], b"k999_0")
    probes = [b"k%03d_%d" % (i, j) for i in range(10) for j in range(5)]
    check(ctx, rng, imgs, probes, held_check=False)


def test_may_contain_truncated_bitset_and_k_zero(ctx):
    """Stored bit count below m (bitset.Test is false past its length) on the
    grouped path (sorted disjoint files) and the per-probe path (overlapping
    files); k = 0 (Test is true) and m = 0 < k (Go panics; answered 0)."""
    rng = np.random.default_rng(6)
    sorted_imgs = []
    for i in range(6):
        keys = [b"r%02d_%05d" % (i, j) for j in range(400)]
        img = build(keys, m=8192, k=4)
        if i % 2 == 0:
            img = _patch_nbits(img, [0, 64, 4000][i // 2])
        sorted_imgs.append(img)
    probes = [b"r%02d_%05d" % (i, j) for i in range(7) for j in range(0, 420, 7)]
    check(ctx, rng, sorted_imgs, probes, held_check=False)     # grouped path
    overl = sorted_imgs[:3] + [build([b"r00_00000", b"r05_99999"], m=4096, k=3)]
    check(ctx, rng, overl, probes, held_check=False)           # per-probe path
    for m in (0, 64):
        k0 = build([b"r00_00001", b"r00_00300"], m=64, k=1)
        # patch k to 0, and m (the u64be before k) to `m`
        mnl = int(np.frombuffer(k0[:4].tobytes(), "<u4")[0])
        at = 8 + 2 * mnl + 8
        k0 = k0.copy()
        k0[at:at + 8] = np.frombuffer(struct.pack(">Q", m), np.uint8)
        k0[at + 8:at + 16] = np.frombuffer(struct.pack(">Q", 0), np.uint8)
        check(ctx, rng, [k0] + sorted_imgs[1:], probes, held_check=False)
    m0 = build([b"r00_00001", b"r00_00300"], m=64, k=2).copy()
    mnl = int(np.frombuffer(m0[:4].tobytes(), "<u4")[0])
    at = 8 + 2 * mnl + 8
    m0[at:at + 8] = np.frombuffer(struct.pack(">Q", 0), np.uint8)  # m = 0, k = 2
    check(ctx, rng, [m0] + sorted_imgs[1:], probes, held_check=False)


def test_may_contain_nbits_overflow_rejected(ctx):
    """a stored bit count near 2^64 with no stored words must fail
    the filter decode (bitset.ReadFrom cannot read that many words) instead
    of passing a wrapped (nbits + 63) / 64 check and letting MayContain read
    bit positions far past the image.  GPU and oracle: stage LSM_SST_FILTER,
    no hit, on both the grouped and the per-probe path."""
    rng = np.random.default_rng(8)
    sorted_imgs = [build([b"w%02d_%04d" % (i, j) for j in range(50)], m=4096, k=3) for i in range(4)]
    probes = [b"w%02d_%04d" % (i, j) for i in range(5) for j in range(0, 60, 3)]
    for nb in ((1 << 64) - 1, (1 << 64) - 63, (1 << 64) - 64, 1 << 63):
        bad = _patch_nbits(sorted_imgs[1], nb)
        rc, meta, *_ = ora.sst_decode(bad)
        assert meta.stage == 2, (nb, meta.stage)   # LSM_SST_FILTER
        imgs = [sorted_imgs[0], bad] + sorted_imgs[2:]
        d_img = lsmgpu.to_device_bytes(np.concatenate(imgs), ctx.torch_device)
        offs = np.cumsum([0] + [im.size for im in imgs[:-1]]).astype(np.uint64)
        r = lsmgpu.decode_sst(ctx, d_img, offs, np.array([im.size for im in imgs], np.uint64))
        assert int(r.meta_numpy()[1]["stage"]) == 2
        check(ctx, rng, imgs, probes, held_check=False)                 # grouped path
        check(ctx, rng, imgs + [build([b"w00_0000", b"w04_9999"], m=64, k=1)], probes,
              held_check=False)                                         # per-probe path


def test_may_contain_per_probe_path_many_probes(ctx):
    """Overlapping files (the per-probe path) with more probes than one pass
    of its capped grid covers (1,024 workgroups x 256 probes): every row of
    the hit matrix against the oracle's batched MayContain, nfile % 4 == 0
    (dword write-out) and != 0 (byte write-out)."""
    rng = np.random.default_rng(77)
    images = []
    for f in range(5):
        lo = int(rng.integers(0, 40_000))
        keys = sorted({b"p%07d" % int(x) for x in rng.integers(lo, lo + 60_000, 3000)})
        images.append(build(keys, m=20_000, k=4))
    n = 300_000
    probes = [b"p%07d" % int(x) for x in rng.integers(0, 110_000, n)]
    kb, ko = csr(probes)
    for imgs in (images[:4], images):
        offs = np.cumsum([0] + [im.size for im in imgs[:-1]]).astype(np.uint64)
        buf = np.concatenate(imgs)
        d_img = lsmgpu.to_device_bytes(buf, ctx.torch_device)
        r = lsmgpu.decode_sst(ctx, d_img, offs, np.array([im.size for im in imgs], np.uint64))
        batch = lsmgpu.batch_to_device(ctx, kb, ko, np.zeros(1, np.uint8), np.zeros(n + 1, np.uint64))
        hit = lsmgpu.may_contain(ctx, d_img, r, batch).cpu().numpy()
        torch.cuda.synchronize()
        metas = [ora.sst_decode(im)[1] for im in imgs]
        want = ora.may_contain_batch(buf, offs, metas, kb, ko, 0, n)
        assert np.array_equal(hit, want), np.argwhere(hit != want)[:8]
        # not vacuous: a probe lies in a file's 60k-key range with p ~ 0.55 and
        # then hits with p ~ 0.05 (held) + 0.04 (false positive, m = 20,000,
        # k = 4, 3,000 keys), so ~ 0.2 of the probes hit some file; the exact
        # matrix is checked against the oracle above
        assert hit.any(axis=1).sum() > n // 10
