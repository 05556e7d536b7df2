"""CPU: the oracle's batched SSTable.MayContain (ora_may_contain_batch, the
probe line's CPU baseline) agrees with the per-file restatement: the range
check in Go string order, then Filter.Test of the decoded filter
(sstable.go:300-305, bloom.go:371-379)."""
import struct

import numpy as np

import pyoracle as ora


def _img(keys, m, k):
    data = b"".join(keys)
    ko = np.zeros(len(keys) + 1, np.uint64)
    ko[1:] = np.cumsum([len(x) for x in keys])
    vo = np.arange(len(keys) + 1, dtype=np.uint64)
    img, _ = ora.build_sst(np.frombuffer(data, np.uint8) if data else np.zeros(0, np.uint8), ko,
                           np.full(max(len(keys), 1), 7, np.uint8), vo, 0, len(keys), m=m, k=k)
    return img


def _expected(img, key):
    rc, meta, *_ = ora.sst_decode(img)
    if meta.stage in (1, 2):
        return 0
    mn = img[meta.min_key_off:meta.min_key_off + meta.min_key_len].tobytes()
    mx = img[meta.max_key_off:meta.max_key_off + meta.max_key_len].tobytes()
    if mn > key or mx < key:
        return 0
    hdr = 8 + meta.min_key_len + meta.max_key_len
    f, _, _ = ora.Bloom.decode(img[hdr:])
    r = f.test_decoded(key)
    return 0 if r < 0 else r


def test_batch_matches_per_file_restatement():
    rng = np.random.default_rng(4)
    imgs = []
    for i in range(5):
        ks = sorted({b"key%05d" % int(x) for x in rng.integers(i * 500, i * 500 + 500, 120)})
        imgs.append(_img(ks, m=1024, k=3))
    imgs.append(_img([b"a", b"zz"], m=64, k=0))            # k = 0: Test is true
    bad = _img([b"q"], m=64, k=2).copy()
    bad[:4] = np.frombuffer(struct.pack("<I", 10 ** 6), np.uint8)
    imgs.append(bad)                                       # header fails
    off = np.cumsum([0] + [x.size for x in imgs[:-1]]).astype(np.uint64)
    buf = np.concatenate(imgs)
    metas = [ora.sst_decode(x)[1] for x in imgs]
    probes = [b"key%05d" % int(x) for x in rng.integers(0, 2600, 300)] + [b"", b"a", b"q", b"zz"]
    kb = np.frombuffer(b"".join(probes), np.uint8)
    ko = np.zeros(len(probes) + 1, np.uint64)
    ko[1:] = np.cumsum([len(p) for p in probes])
    hit = ora.may_contain_batch(buf, off, metas, kb, ko, 0, len(probes))
    for i, p in enumerate(probes):
        for f, im in enumerate(imgs):
            assert hit[i, f] == _expected(im, p), (p, f)


def test_filter_nbits_near_2_64_fails_decode():
    """nbits near 2^64 with no stored words is a failed filter
    decode (stage LSM_SST_FILTER = 2; bitset.ReadFrom cannot read that many
    words), not a wrapped (nbits + 63) / 64 that passes the length check.
    Also through ora_filter_decode directly and the batched MayContain."""
    img = _img([b"n%03d" % i for i in range(20)], m=1024, k=3)
    mnl = int(np.frombuffer(img[:4].tobytes(), "<u4")[0])
    at = 8 + 2 * mnl + 8 + 16
    for nb in ((1 << 64) - 1, (1 << 64) - 63, 1 << 63):
        bad = img.copy()
        bad[at:at + 8] = np.frombuffer(struct.pack(">Q", nb), np.uint8)
        rc, meta, *_ = ora.sst_decode(bad)
        assert meta.stage == 2, (nb, meta.stage)
        kb = np.frombuffer(b"n005", np.uint8)
        hit = ora.may_contain_batch(bad, np.zeros(1, np.uint64), [meta], kb,
                                    np.array([0, 4], np.uint64), 0, 1)
        assert hit[0, 0] == 0
    good = ora.sst_decode(img)[1]
    assert good.stage == 0
