"""ora_level_get (the batched Get past MayContain) against a pure-Python
restatement of the Go text: Iterator.Seek (sstable/block/index.go:157-181),
Iterator.Valid / Key (index.go:128-140), sstable.Iterator.Value
(sstable/iterator.go:34-46) -> GetValueByOffset (sstable.go:271-296) ->
Value.DecodeFrom (kv.go:181-200).  CPU only."""
import numpy as np

import pyoracle as ora


def go_get(file, entries, key):
    """entries: [(key bytes, offset)] of the table's IndexBlock; file: bytes."""
    left, right = 0, len(entries)
    while left < right:                      # index.go:160-167
        mid = left + (right - left) // 2
        if entries[mid][0] < key:            # Go string <: bytewise, then length
            left = mid + 1
        else:
            right = mid
    if left >= len(entries) or entries[left][0] != key:   # index.go:170-180
        return ora.GET_ABSENT, None
    off = entries[left][1]
    if off < 0:                              # file.Seek(offset, io.SeekStart)
        return ora.GET_SEEK_FAILED, None
    rest = file[off:] if off < len(file) else b""
    if len(rest) < 4:                        # binary.Read: EOF / ErrUnexpectedEOF
        return ora.GET_VALUE_LENGTH, None
    n = int.from_bytes(rest[:4], "little")
    if n > 1 << 30:                          # kv.go:188-190
        return ora.GET_VALUE_TOO_LONG, None
    if len(rest) - 4 < n:                    # io.ReadFull
        return ora.GET_VALUE_SHORT, None
    return ora.GET_FOUND, (off, n)


def test_oracle_level_get_matches_go_restatement():
    rng = np.random.default_rng(7)
    for trial in range(40):
        keys = sorted({bytes(rng.integers(97, 100, int(rng.integers(0, 6))).astype(np.uint8))
                       for _ in range(int(rng.integers(1, 60)))})
        if trial % 3 == 0 and keys:                        # equal keys in the index
            keys = sorted(keys + [keys[len(keys) // 2]] * 2)
        vals = [bytes(rng.integers(0, 256, int(rng.integers(0, 9))).astype(np.uint8)) for _ in keys]
        kb = np.frombuffer(b"".join(keys) or b"\0", np.uint8)
        ko = np.concatenate([[0], np.cumsum([len(k) for k in keys])]).astype(np.uint64)
        vb = np.frombuffer(b"".join(vals) or b"\0", np.uint8)
        vo = np.concatenate([[0], np.cumsum([len(v) for v in vals])]).astype(np.uint64)
        img, _ = ora.build_sst(kb, ko, vb, vo, 0, len(keys), m=512, k=3)
        img = img.copy()
        rc, meta, idesc, ival, _ = ora.sst_decode(img)
        # corrupt a few offsets: negative, past the end, onto the footer
        for j in range(len(idesc)):
            if rng.random() < 0.2:
                at = int(idesc["rec_off"][j]) + 4 + int(idesc["key_len"][j])
                o = int(rng.choice([-1, img.size, img.size - 3, img.size - 32, int(meta.idx_off)]))
                img[at:at + 8] = np.frombuffer(o.to_bytes(8, "little", signed=True), np.uint8)
        rc, meta, idesc, ival, _ = ora.sst_decode(img)
        file = img.tobytes()
        entries = [(file[int(d["rec_off"]) + 4:int(d["rec_off"]) + 4 + int(d["key_len"])], int(v))
                   for d, v in zip(idesc, ival)]
        probes = list({k for k in keys}) + [b"", b"a", b"zz", b"ab\x00"] + \
            [bytes(rng.integers(97, 100, 3).astype(np.uint8)) for _ in range(30)]
        pb = np.frombuffer(b"".join(probes) or b"\0", np.uint8)
        po = np.concatenate([[0], np.cumsum([len(p) for p in probes])]).astype(np.uint64)
        base = 5
        buf = np.concatenate([np.zeros(base, np.uint8), img])
        table = np.zeros(len(probes), np.int32)
        may = np.ones(len(probes), np.uint8)
        may[::7] = 0
        res, voff, vlen = ora.level_get(buf, [base], [img.size], [meta], [idesc], [ival], pb, po, 0,
                                        len(probes), table, may)
        for i, p in enumerate(probes):
            want, view = go_get(file, entries, p) if may[i] else (ora.GET_ABSENT, None)
            assert res[i] == want, (trial, p, res[i], want)
            if view:
                assert voff[i] == base + view[0] and vlen[i] == view[1]
            else:
                assert voff[i] == 0 and vlen[i] == 0


def test_oracle_level0_get_matches_go_restatement():
    """ora_level0_get against searchFromLevel0 (manager.go:160-176) restated
    over go_get: every table in order, MayContain first (the oracle's
    may_contain_batch, itself pinned against the per-file restatement), the
    first non-nil value or error wins.  Overlapping tables, keys held by two
    tables (the newer wins), tiny filters (false positives in newer tables
    with the key in an older one), corrupted offsets in a newer table (its
    error, not the older value), an empty table and an empty level."""
    rng = np.random.default_rng(11)
    for trial in range(25):
        nfile = int(rng.integers(0, 5))
        images, tables = [], []
        for t in range(nfile):
            nk = 0 if (trial % 7 == 3 and t == 1) else int(rng.integers(1, 40))
            keys = sorted({bytes(rng.integers(97, 101, int(rng.integers(1, 5))).astype(np.uint8))
                           for _ in range(nk)})
            vals = [b"t%d-" % t + bytes(rng.integers(0, 256, int(rng.integers(0, 6))).astype(np.uint8))
                    for _ in keys]
            kb = np.frombuffer(b"".join(keys) or b"\0", np.uint8)
            ko = np.concatenate([[0], np.cumsum([len(k) for k in keys])]).astype(np.uint64)
            vb = np.frombuffer(b"".join(vals) or b"\0", np.uint8)
            vo = np.concatenate([[0], np.cumsum([len(v) for v in vals])]).astype(np.uint64)
            m, k = (64, 1) if trial % 2 else (1024, 4)
            img, _ = ora.build_sst(kb, ko, vb, vo, 0, len(keys), m=m, k=k)
            img = img.copy()
            rc, meta, idesc, ival, _ = ora.sst_decode(img)
            if t == 0 and trial % 3 == 0:
                for j in range(len(idesc)):
                    if rng.random() < 0.3:
                        at = int(idesc["rec_off"][j]) + 4 + int(idesc["key_len"][j])
                        o = int(rng.choice([-1, img.size, img.size - 3]))
                        img[at:at + 8] = np.frombuffer(o.to_bytes(8, "little", signed=True), np.uint8)
                rc, meta, idesc, ival, _ = ora.sst_decode(img)
            images.append(img)
            tables.append((meta, idesc, ival))
        offs, pos = [], 3
        for im in images:
            offs.append(pos)
            pos += im.size + 5
        buf = np.zeros(pos + 16, np.uint8)
        for o, im in zip(offs, images):
            buf[o:o + im.size] = im
        probes = [b"", b"a", b"zz"] + [bytes(rng.integers(97, 101, int(rng.integers(1, 5))).astype(np.uint8))
                                       for _ in range(80)]
        pb = np.frombuffer(b"".join(probes) or b"\0", np.uint8)
        po = np.concatenate([[0], np.cumsum([len(p) for p in probes])]).astype(np.uint64)
        lens = [im.size for im in images]
        table, res, voff, vlen = ora.level0_get(buf, offs, lens, [t[0] for t in tables],
                                                [t[1] for t in tables], [t[2] for t in tables],
                                                pb, po, 0, len(probes))
        may = ora.may_contain_batch(buf, offs, [t[0] for t in tables], pb, po, 0, len(probes)) \
            if nfile else np.zeros((len(probes), 1), np.uint8)
        for i, p in enumerate(probes):
            want, wt, view = ora.GET_ABSENT, -1, None
            for t in range(nfile):
                if not may[i, t]:
                    continue
                file = images[t].tobytes()
                meta, idesc, ival = tables[t]
                entries = [(file[int(d["rec_off"]) + 4:int(d["rec_off"]) + 4 + int(d["key_len"])], int(v))
                           for d, v in zip(idesc, ival)]
                r, v = go_get(file, entries, p)
                if r == ora.GET_ABSENT:
                    continue
                want, wt, view = r, t, v
                break
            assert res[i] == want and table[i] == wt, (trial, p, res[i], want, table[i], wt)
            if view:
                assert voff[i] == offs[wt] + view[0] and vlen[i] == view[1]
            else:
                assert voff[i] == 0 and vlen[i] == 0
