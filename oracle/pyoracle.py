"""ctypes binding of oracle/liblsm_oracle.so — TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() (as the checker) and
bench.py's cpu_baseline leg.  The product path never touches it.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liblsm_oracle.so")

GRAMMAR_V, GRAMMAR_KV, GRAMMAR_IDX = 0, 1, 2
DESC_DTYPE = np.dtype([("rec_off", "<u8"), ("key_len", "<u4"), ("val_len", "<u4")])


class SstMeta(ctypes.Structure):
    _fields_ = [
        ("min_key_off", ctypes.c_uint64), ("min_key_len", ctypes.c_uint64),
        ("max_key_off", ctypes.c_uint64), ("max_key_len", ctypes.c_uint64),
        ("filter_m", ctypes.c_uint64), ("filter_k", ctypes.c_uint64),
        ("filter_nbits", ctypes.c_uint64), ("filter_words_off", ctypes.c_uint64),
        ("data_off", ctypes.c_int64), ("data_size", ctypes.c_int64),
        ("idx_off", ctypes.c_int64), ("idx_size", ctypes.c_int64),
        ("stage", ctypes.c_int32), ("status", ctypes.c_int32),
        ("nidx", ctypes.c_uint32), ("ndata", ctypes.c_uint32),
    ]


_lib = None
vp = ctypes.c_void_p
u64 = ctypes.c_uint64


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} missing: run `make -C oracle`")
    L = ctypes.CDLL(LIB_PATH)
    sig = {
        "ora_decode_block": (ctypes.c_int, [ctypes.c_int, vp, u64, u64, vp, vp, u64, vp]),
        "ora_materialize": (u64, [ctypes.c_int, vp, vp, u64, vp, vp, vp]),
        "ora_encoded_size": (u64, [ctypes.c_int, vp, vp, u64, u64]),
        "ora_encode_records": (u64, [ctypes.c_int, vp, vp, vp, vp, u64, u64, vp, vp]),
        "ora_sum256": (None, [vp, u64, vp]),
        "ora_mmh3_x64_128": (None, [vp, u64, ctypes.c_uint32, vp]),
        "ora_mmh3_verification": (ctypes.c_uint32, []),
        "ora_location": (u64, [vp, u64]),
        "ora_bloom_add": (None, [vp, u64, u64, vp, u64]),
        "ora_bloom_test": (ctypes.c_int, [vp, u64, u64, vp, u64]),
        "ora_filter_test": (ctypes.c_int, [vp, u64, u64, u64, vp, u64]),
        "ora_may_contain_batch": (None, [vp, vp, vp, ctypes.c_uint32, vp, vp, u64, u64, vp]),
        "ora_level_may_contain": (None, [vp, vp, vp, ctypes.c_uint32, vp, vp, u64, u64, vp, vp]),
        "ora_level_get": (None, [vp, vp, vp, vp, vp, vp, vp, vp, vp, u64, u64, vp, vp, vp, vp, vp]),
        "ora_level0_get": (None, [vp, vp, vp, vp, ctypes.c_uint32, vp, vp, vp, vp, vp, u64, u64, vp, vp,
                                  vp, vp]),
        "ora_estimate_parameters": (None, [u64, ctypes.c_double, vp, vp]),
        "ora_filter_block_size": (u64, [u64]),
        "ora_filter_encode": (u64, [vp, u64, u64, vp]),
        "ora_filter_decode": (ctypes.c_int, [vp, u64, vp, vp, vp, vp, u64, vp]),
        "ora_segment_files": (u64, [vp, vp, u64, u64, vp]),
        "ora_sst_image_size": (u64, [vp, vp, u64, u64, u64]),
        "ora_build_sst": (u64, [vp, vp, vp, vp, u64, u64, u64, u64, vp, vp]),
        "ora_sst_decode": (ctypes.c_int, [vp, u64, ctypes.POINTER(SstMeta), vp, vp, u64, vp,
                                          u64]),
        "ora_bench_decode_golike": (u64, [ctypes.c_int, vp, vp, vp, u64, ctypes.c_int]),
        "ora_sst_decode_file": (ctypes.c_int64, [ctypes.c_char_p]),
        "ora_merge_kvs": (u64, [vp, vp, vp, vp, vp, u64, ctypes.c_int, u64, ctypes.c_int, vp, vp,
                                vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def _p(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def _bytes(b) -> np.ndarray:
    if isinstance(b, np.ndarray):
        return np.ascontiguousarray(b, dtype=np.uint8).reshape(-1)
    return np.frombuffer(bytes(b), dtype=np.uint8)


def decode_block(grammar, buf, off=0, length=None, cap=None):
    """-> (status, desc[nrec], idx_val[nrec] or None)."""
    buf = _bytes(buf)
    if length is None:
        length = buf.size - off
    if cap is None:
        cap = {0: length // 4, 1: length // 8, 2: length // 12}[grammar]
    desc = np.zeros(max(cap, 1), dtype=DESC_DTYPE)
    iv = np.zeros(max(cap, 1), dtype=np.int64) if grammar == GRAMMAR_IDX else None
    n = ctypes.c_uint32()
    st = lib().ora_decode_block(grammar, _p(buf), off, length, _p(desc), _p(iv), cap,
                                ctypes.byref(n))
    k = n.value
    return st, desc[:k].copy(), (iv[:k].copy() if iv is not None else None)


def decode_blocks(grammar, buf, blk_off, blk_len):
    """Decode every block; -> (status[nblk], nrec[nblk], list of desc arrays, list of idx)."""
    buf = _bytes(buf)
    sts, nrs, ds, ivs = [], [], [], []
    for o, l in zip(blk_off, blk_len):
        st, d, iv = decode_block(grammar, buf, int(o), int(l))
        sts.append(st)
        nrs.append(len(d))
        ds.append(d)
        ivs.append(iv)
    return np.array(sts, dtype=np.int32), np.array(nrs, dtype=np.int64), ds, ivs


def materialize(grammar, buf, desc):
    buf = _bytes(buf)
    desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
    kb = int(desc["key_len"].sum()) if grammar != GRAMMAR_V else 0
    vb = int(desc["val_len"].sum()) if grammar != GRAMMAR_IDX else 0
    ka = np.zeros(max(kb, 1), dtype=np.uint8)
    va = np.zeros(max(vb, 1), dtype=np.uint8)
    vbo = ctypes.c_uint64()
    lib().ora_materialize(grammar, _p(buf), _p(desc), desc.size, _p(ka), _p(va),
                          ctypes.byref(vbo))
    return ka[:kb], va[:vb]


def encode_records(grammar, keys, koff, vals, voff, r0, r1, idx_off=None):
    koff = np.ascontiguousarray(koff, dtype=np.uint64)
    voff = np.ascontiguousarray(voff, dtype=np.uint64)
    keys = _bytes(keys) if keys is not None else np.zeros(1, np.uint8)
    vals = _bytes(vals) if vals is not None else np.zeros(1, np.uint8)
    n = lib().ora_encoded_size(grammar, _p(koff), _p(voff), r0, r1)
    out = np.zeros(max(n, 1), dtype=np.uint8)
    io = np.ascontiguousarray(idx_off, dtype=np.int64) if idx_off is not None else None
    w = lib().ora_encode_records(grammar, _p(keys), _p(koff), _p(vals), _p(voff), r0, r1,
                                 _p(io), _p(out))
    assert w == n
    return out[:n]


def sum256(data):
    d = _bytes(data)
    h = np.zeros(4, dtype=np.uint64)
    lib().ora_sum256(_p(d) if d.size else None, d.size, _p(h))
    return tuple(int(x) for x in h)


def mmh3_x64_128(data, seed=0):
    d = _bytes(data)
    o = np.zeros(2, dtype=np.uint64)
    lib().ora_mmh3_x64_128(_p(d) if d.size else None, d.size, seed, _p(o))
    return int(o[0]), int(o[1])


def mmh3_verification():
    return lib().ora_mmh3_verification()


class Bloom:
    """Filter (bloom.go) over native u64 words."""

    def __init__(self, m, k):
        self.m, self.k = m, k
        self.words = np.zeros(max((m + 63) // 64, 1), dtype=np.uint64)

    def add(self, key):
        d = _bytes(key)
        lib().ora_bloom_add(_p(self.words), self.m, self.k, _p(d) if d.size else None, d.size)
        return self

    def test(self, key):
        d = _bytes(key)
        return bool(lib().ora_bloom_test(_p(self.words), self.m, self.k,
                                         _p(d) if d.size else None, d.size))

    def test_and_add(self, key):
        present = self.test(key)
        self.add(key)
        return present

    def encode(self):
        n = lib().ora_filter_block_size(self.m)
        out = np.zeros(n, dtype=np.uint8)
        lib().ora_filter_encode(_p(self.words), self.m, self.k, _p(out))
        return out

    @staticmethod
    def decode(buf):
        b = _bytes(buf)
        m, k, nb, used = (ctypes.c_uint64() for _ in range(4))
        # probe size first
        rc = lib().ora_filter_decode(_p(b), b.size, ctypes.byref(m), ctypes.byref(k),
                                     ctypes.byref(nb), None, 0, ctypes.byref(used))
        if rc != 0:
            raise ValueError(f"filter decode failed ({rc})")
        f = Bloom(int(m.value), int(k.value))
        words = np.zeros(max((nb.value + 63) // 64, 1), dtype=np.uint64)
        rc = lib().ora_filter_decode(_p(b), b.size, ctypes.byref(m), ctypes.byref(k),
                                     ctypes.byref(nb), _p(words), words.size,
                                     ctypes.byref(used))
        if rc != 0:
            raise ValueError(f"filter decode failed ({rc})")
        f.words = words
        f.nbits = int(nb.value)
        return f, int(nb.value), int(used.value)

    def test_decoded(self, key):
        """Filter.Test of a decoded filter: 1, 0, or -1 where Go panics."""
        d = _bytes(key)
        return int(lib().ora_filter_test(_p(self.words), self.nbits, self.m, self.k,
                                         _p(d) if d.size else None, d.size))


def estimate_parameters(n, p):
    m, k = ctypes.c_uint64(), ctypes.c_uint64()
    lib().ora_estimate_parameters(n, p, ctypes.byref(m), ctypes.byref(k))
    return int(m.value), int(k.value)


def segment_files(koff, voff, threshold):
    koff = np.ascontiguousarray(koff, dtype=np.uint64)
    voff = np.ascontiguousarray(voff, dtype=np.uint64)
    n = koff.size - 1
    starts = np.zeros(n + 2, dtype=np.uint64)
    nf = lib().ora_segment_files(_p(koff), _p(voff), n, threshold, _p(starts))
    return starts[: nf + 1].copy()


def build_sst(keys, koff, vals, voff, r0, r1, m=1_600_000, k=16):
    koff = np.ascontiguousarray(koff, dtype=np.uint64)
    voff = np.ascontiguousarray(voff, dtype=np.uint64)
    keys = _bytes(keys) if len(keys) else np.zeros(1, np.uint8)
    vals = _bytes(vals) if len(vals) else np.zeros(1, np.uint8)
    n = lib().ora_sst_image_size(_p(koff), _p(voff), r0, r1, m)
    out = np.zeros(n, dtype=np.uint8)
    footer = np.zeros(4, dtype=np.int64)
    w = lib().ora_build_sst(_p(keys), _p(koff), _p(vals), _p(voff), r0, r1, m, k, _p(out),
                            _p(footer))
    assert w == n
    return out, footer


def sst_decode(image):
    """-> (rc, meta, idx_desc, idx_val, data_desc)."""
    b = _bytes(image)
    cap_i = b.size // 12 + 1
    cap_d = b.size // 4 + 1
    idesc = np.zeros(cap_i, dtype=DESC_DTYPE)
    ival = np.zeros(cap_i, dtype=np.int64)
    ddesc = np.zeros(cap_d, dtype=DESC_DTYPE)
    meta = SstMeta()
    rc = lib().ora_sst_decode(_p(b), b.size, ctypes.byref(meta), _p(idesc), _p(ival), cap_i,
                              _p(ddesc), cap_d)
    return rc, meta, idesc[: meta.nidx].copy(), ival[: meta.nidx].copy(), \
        ddesc[: meta.ndata].copy()


TIE_INPUT, TIE_GOHEAP = 0, 1


def merge_kvs(buf, koff, klen, voff, vlen, level, threshold, tie=TIE_INPUT):
    """CompactAndMergeKVs (merge.go:42-94) over views into buf ->
    (out: written pairs' input indices, starts: file starts in out)."""
    buf = _bytes(buf)
    koff = np.ascontiguousarray(koff, dtype=np.uint64)
    voff = np.ascontiguousarray(voff, dtype=np.uint64)
    klen = np.ascontiguousarray(klen, dtype=np.uint32)
    vlen = np.ascontiguousarray(vlen, dtype=np.uint32)
    n = klen.size
    out = np.zeros(max(n, 1), np.uint32)
    starts = np.zeros(n + 2, np.uint64)
    nf = u64(0)
    cnt = lib().ora_merge_kvs(_p(buf) if buf.size else None, _p(koff), _p(klen), _p(voff), _p(vlen),
                              n, level, threshold, tie, _p(out), _p(starts), ctypes.byref(nf))
    return out[:cnt].copy(), starts[:nf.value + 1].copy()


def merge_pairs(pairs, level, threshold, tie=TIE_INPUT):
    """merge_kvs over a list of (key bytes, value bytes) -> (out, starts)."""
    blob, koff, klen, voff, vlen, pos = [], [], [], [], [], 0
    for k, v in pairs:
        koff.append(pos); klen.append(len(k)); blob.append(k); pos += len(k)
        voff.append(pos); vlen.append(len(v)); blob.append(v); pos += len(v)
    return merge_kvs(b"".join(blob) or b"\0", koff, klen, voff, vlen, level, threshold, tie)


def bench_decode_golike(grammar, buf, blk_off, blk_len, threads=1):
    buf = _bytes(buf)
    blk_off = np.ascontiguousarray(blk_off, dtype=np.uint64)
    blk_len = np.ascontiguousarray(blk_len, dtype=np.uint32)
    return lib().ora_bench_decode_golike(grammar, _p(buf), _p(blk_off), _p(blk_len),
                                         blk_off.size, threads)


def sst_decode_file(path):
    """SSTable.DecodeFrom + GetDataBlockFromFile from a file with one read(2)
    per field (the reference's *os.File pattern) -> pairs, or < 0."""
    return int(lib().ora_sst_decode_file(os.fsencode(path)))


def may_contain_batch(img, file_off, metas, keys, koff, k0, k1):
    """Batched SSTable.MayContain of keys [k0, k1) -> uint8 (k1-k0, nfile).
    metas: the files' SstMeta (a ctypes array or list)."""
    img = _bytes(img)
    file_off = np.ascontiguousarray(file_off, dtype=np.uint64)
    keys = _bytes(keys) if len(keys) else np.zeros(1, np.uint8)
    koff = np.ascontiguousarray(koff, dtype=np.uint64)
    nfile = len(metas)
    arr = metas if isinstance(metas, ctypes.Array) else (SstMeta * nfile)(*metas)
    hit = np.zeros((k1 - k0, max(nfile, 1)), np.uint8)
    lib().ora_may_contain_batch(_p(img), _p(file_off), ctypes.cast(arr, vp), nfile, _p(keys),
                                _p(koff), k0, k1, _p(hit))
    return hit


def level_may_contain(img, file_off, metas, keys, koff, k0, k1):
    """searchFromLevelWithSparseIndex's candidate table + MayContain for keys
    [k0, k1) over one level's tables in sparse-index order
    -> (int32 table (k1-k0,), uint8 may (k1-k0,))."""
    img = _bytes(img)
    file_off = np.ascontiguousarray(file_off, dtype=np.uint64) if len(file_off) else np.zeros(1, np.uint64)
    keys = _bytes(keys) if len(keys) else np.zeros(1, np.uint8)
    koff = np.ascontiguousarray(koff, dtype=np.uint64)
    nfile = len(metas)
    arr = metas if isinstance(metas, ctypes.Array) else (SstMeta * max(nfile, 1))(*metas)
    table = np.zeros(max(k1 - k0, 1), np.int32)
    may = np.zeros(max(k1 - k0, 1), np.uint8)
    lib().ora_level_may_contain(_p(img), _p(file_off), ctypes.cast(arr, vp), nfile, _p(keys),
                                _p(koff), k0, k1, _p(table), _p(may))
    return table[:k1 - k0], may[:k1 - k0]


GET_ABSENT, GET_FOUND, GET_SEEK_FAILED, GET_VALUE_LENGTH, GET_VALUE_TOO_LONG, GET_VALUE_SHORT = range(6)


def level_get_index(idx_descs, idx_vals):
    """The tables' decoded index rows concatenated -> (desc, vals, base)."""
    nfile = len(idx_descs)
    base = np.zeros(max(nfile, 1), np.uint64)
    if nfile:
        base[:] = np.concatenate([[0], np.cumsum([len(d) for d in idx_descs])[:-1]]).astype(np.uint64)
    desc = np.concatenate(list(idx_descs) + [np.zeros(1, DESC_DTYPE)]).astype(DESC_DTYPE)
    vals = np.concatenate(list(idx_vals) + [np.zeros(1, np.int64)]).astype(np.int64)
    return desc, vals, base


def level_get(img, file_off, file_len, metas, idx_descs, idx_vals, keys, koff, k0, k1, table, may,
              index=None):
    """searchFromTable past MayContain (manager.go:209-223) for keys [k0, k1):
    Iterator.Seek over the candidate table's decoded index, then
    GetValueByOffset.  idx_descs / idx_vals: per table, sst_decode's index
    rows (rec_off relative to the file); index: level_get_index of them,
    prepared once.  table / may: rows k0 .. k1 of the level search.
    -> (int32 res, uint64 val_off into img, uint32 val_len), each (k1-k0,)."""
    img = _bytes(img)
    nfile = len(metas)
    file_off = np.ascontiguousarray(file_off, dtype=np.uint64) if nfile else np.zeros(1, np.uint64)
    file_len = np.ascontiguousarray(file_len, dtype=np.uint64) if nfile else np.zeros(1, np.uint64)
    arr = metas if isinstance(metas, ctypes.Array) else (SstMeta * max(nfile, 1))(*metas)
    desc, vals, base = index if index is not None else level_get_index(idx_descs, idx_vals)
    keys = _bytes(keys) if len(keys) else np.zeros(1, np.uint8)
    koff = np.ascontiguousarray(koff, dtype=np.uint64)
    n = k1 - k0
    table = np.ascontiguousarray(table, dtype=np.int32)
    may = np.ascontiguousarray(may, dtype=np.uint8)
    res = np.zeros(max(n, 1), np.int32)
    voff = np.zeros(max(n, 1), np.uint64)
    vlen = np.zeros(max(n, 1), np.uint32)
    lib().ora_level_get(_p(img), _p(file_off), _p(file_len), ctypes.cast(arr, vp), _p(desc), _p(vals),
                        _p(base), _p(keys), _p(koff), k0, k1, _p(table), _p(may), _p(res), _p(voff),
                        _p(vlen))
    return res[:n], voff[:n], vlen[:n]


def level0_get(img, file_off, file_len, metas, idx_descs, idx_vals, keys, koff, k0, k1, index=None):
    """Manager.searchFromLevel0 (manager.go:160-176) for keys [k0, k1): every
    table in order (newest first), searchFromTable on each; the first value or
    error wins.  -> (int32 table, int32 res, uint64 val_off, uint32 val_len)."""
    img = _bytes(img)
    nfile = len(metas)
    file_off = np.ascontiguousarray(file_off, dtype=np.uint64) if nfile else np.zeros(1, np.uint64)
    file_len = np.ascontiguousarray(file_len, dtype=np.uint64) if nfile else np.zeros(1, np.uint64)
    arr = metas if isinstance(metas, ctypes.Array) else (SstMeta * max(nfile, 1))(*metas)
    desc, vals, base = index if index is not None else level_get_index(idx_descs, idx_vals)
    keys = _bytes(keys) if len(keys) else np.zeros(1, np.uint8)
    koff = np.ascontiguousarray(koff, dtype=np.uint64)
    n = k1 - k0
    table = np.zeros(max(n, 1), np.int32)
    res = np.zeros(max(n, 1), np.int32)
    voff = np.zeros(max(n, 1), np.uint64)
    vlen = np.zeros(max(n, 1), np.uint32)
    lib().ora_level0_get(_p(img), _p(file_off), _p(file_len), ctypes.cast(arr, vp), nfile, _p(desc),
                         _p(vals), _p(base), _p(keys), _p(koff), k0, k1, _p(table), _p(res), _p(voff),
                         _p(vlen))
    return table[:n], res[:n], voff[:n], vlen[:n]
