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


def _go_sort_search(n, f):
    """Go's sort.Search (sort/search.go), step for step."""
    i, j = 0, n
    while i < j:
        h = (i + j) >> 1
        if not f(h):
            i = h + 1
        else:
            j = h
    return i


def _level_expected(imgs, key):
    """searchFromLevelWithSparseIndex (manager.go:178-207) up to MayContain
    (:209-212), written from the Go text: sort.Search on MinKey > key,
    index-- when > 0, then the candidate's MayContain; a table whose header did
    not decode searches as the zero Header (MinKey "")."""
    def min_key(h):
        rc, meta, *_ = ora.sst_decode(imgs[h])
        if meta.stage == 1:
            return b""
        return imgs[h][meta.min_key_off:meta.min_key_off + meta.min_key_len].tobytes()
    index = _go_sort_search(len(imgs), lambda h: min_key(h) > key)
    if index > 0:
        index -= 1
    if index < len(imgs):
        return index, _expected(imgs[index], key)
    return -1, 0


def test_level_search_matches_go_restatement():
    """ora_level_may_contain against the Python restatement of the Go code:
    a sorted disjoint level (keys below the first MinKey -> table 0 and no
    hit, equal to a MinKey, above the last MaxKey, in the gaps), equal
    MinKeys, an unsorted level (the exact bisection order decides), a table
    whose header fails, and the empty level."""
    rng = np.random.default_rng(12)
    sorted_lv = []
    for i in range(9):
        ks = sorted({b"lv%05d" % (i * 1000 + int(x)) for x in rng.integers(100, 900, 60)})
        sorted_lv.append(_img(ks, m=2048, k=3))
    dup = sorted_lv[:4] + [_img([b"lv03950", b"lv03990"], m=512, k=2)] + sorted_lv[4:]
    unsorted = [sorted_lv[i] for i in (3, 0, 7, 1, 8, 2, 5, 4, 6)]
    bad = _img([b"lv05500"], m=64, k=2).copy()
    bad[:4] = np.frombuffer(struct.pack("<I", 10 ** 6), np.uint8)
    with_bad = sorted_lv[:5] + [bad] + sorted_lv[5:]
    probes = [b"lv%05d" % int(x) for x in rng.integers(0, 9500, 400)]
    probes += [b"", b"a", b"lv", b"lv00000", b"lv99999", b"zz"]
    for im in sorted_lv:  # each table's exact MinKey and MaxKey
        rc, meta, *_ = ora.sst_decode(im)
        probes += [im[meta.min_key_off:meta.min_key_off + meta.min_key_len].tobytes(),
                   im[meta.max_key_off:meta.max_key_off + meta.max_key_len].tobytes()]
    kb = np.frombuffer(b"".join(probes), np.uint8)
    ko = np.zeros(len(probes) + 1, np.uint64)
    ko[1:] = np.cumsum([len(p) for p in probes])
    seen_index0_miss = seen_hit = False
    for lv in (sorted_lv, dup, unsorted, with_bad, []):
        off = np.cumsum([0] + [x.size for x in lv[:-1]]).astype(np.uint64) if lv else np.zeros(0, np.uint64)
        buf = np.concatenate(lv) if lv else np.zeros(16, np.uint8)
        metas = [ora.sst_decode(x)[1] for x in lv]
        table, may = ora.level_may_contain(buf, off, metas, kb, ko, 0, len(probes))
        for i, p in enumerate(probes):
            want = _level_expected(lv, p)
            assert (int(table[i]), int(may[i])) == want, (p, table[i], may[i], want)
            seen_index0_miss |= lv is sorted_lv and p < b"lv00100" and want == (0, 0)
            seen_hit |= want[1] == 1
    assert seen_index0_miss and seen_hit
