"""Pins the CPU restatement (oracle/) against go-lsm's own test vectors.

Each test names the reference test it translates.  These run on CPU only.
"""
import json
import math
import os
import struct

import numpy as np
import pytest

import pyoracle as ora

HERE = os.path.dirname(os.path.abspath(__file__))
REF = json.load(open(os.path.join(HERE, "golden", "reference_vectors.json")))
ORV = np.load(os.path.join(HERE, "golden", "oracle_vectors.npz"))


def csr(items):
    items = [bytes(x) for x in items]
    off = np.zeros(len(items) + 1, np.uint64)
    off[1:] = np.cumsum([len(x) for x in items]) if items else []
    data = np.frombuffer(b"".join(items) + b"\0", np.uint8)[:-1] if items else np.zeros(0, np.uint8)
    return data, off


def enc_values(values):
    vals, voff = csr(values)
    koff = np.zeros(len(values) + 1, np.uint64)
    return ora.encode_records(ora.GRAMMAR_V, None, koff, vals, voff, 0, len(values))


# ---- sstable/block/index_test.go -------------------------------------------

@pytest.mark.parametrize("case", REF["index_entry_encode"])
def test_index_entry_encode_kat(case):
    keys, koff = csr([case["key"].encode()])
    out = ora.encode_records(ora.GRAMMAR_IDX, keys, koff, None, np.zeros(2, np.uint64), 0, 1,
                             idx_off=[case["offset"]])
    assert out.tobytes().hex() == case["bytes"]


def _index_block(entries):
    keys, koff = csr([k.encode() for k, _ in entries])
    return ora.encode_records(ora.GRAMMAR_IDX, keys, koff, None, np.zeros(len(entries) + 1,
                              np.uint64), 0, len(entries), idx_off=[o for _, o in entries])


def test_index_block_roundtrip_and_limits():
    ib = REF["index_block"]
    data = _index_block(ib["entries"])
    st, desc, iv = ora.decode_block(ora.GRAMMAR_IDX, data, 0, data.size)
    assert st == 0 and len(desc) == 3
    for (k, o), d, v in zip(ib["entries"], desc, iv):
        assert data[d["rec_off"] + 4:d["rec_off"] + 4 + d["key_len"]].tobytes() == k.encode()
        assert v == o
    # partial size: exactly the first entry (index_test.go:141-147)
    two = _index_block(ib["entries"][:2])
    st, desc, iv = ora.decode_block(ora.GRAMMAR_IDX, two, 0, ib["partial_size_first_entry"])
    assert st == 0 and len(desc) == 1 and iv[0] == 100
    # truncated data with size = first entry (index_test.go:149-153): error
    trunc = two[: ib["partial_size_first_entry"] - ib["truncate_by"]]
    st, desc, _ = ora.decode_block(ora.GRAMMAR_IDX, trunc, 0, trunc.size)
    assert st != 0 and len(desc) == 0


# ---- sstable/block/data_test.go ---------------------------------------------

@pytest.mark.parametrize("case", REF["data_block_roundtrip"])
def test_data_block_roundtrip(case):
    entries = [e.encode() for e in case["entries"]]
    buf = enc_values(entries)
    size = case["size"]
    n = buf.size if size <= 0 else min(size, buf.size)  # LimitReader(r, size)
    st, desc, _ = ora.decode_block(ora.GRAMMAR_V, buf, 0, n)
    assert st == 0
    assert len(desc) == len(entries)
    for e, d in zip(entries, desc):
        assert buf[d["rec_off"] + 4:d["rec_off"] + 4 + d["val_len"]].tobytes() == e


def test_data_block_size_limit():
    c = REF["data_block_size_limit"]
    buf = enc_values([e.encode() for e in c["entries"]])
    st, desc, _ = ora.decode_block(ora.GRAMMAR_V, buf, 0, c["insufficient"]["size"])
    assert st == ora_status("TRUNC_VAL")
    st, desc, _ = ora.decode_block(ora.GRAMMAR_V, buf, 0, c["partial"]["size"])
    assert st == 0 and len(desc) == c["partial"]["count"]


@pytest.mark.parametrize("case", REF["data_block_corrupt"])
def test_data_block_corrupt(case):
    buf = np.frombuffer(bytes.fromhex(case["bytes"]), np.uint8)
    st, desc, _ = ora.decode_block(ora.GRAMMAR_V, buf, 0, buf.size)
    assert st != 0 and len(desc) == 0


def ora_status(name):
    return {"OK": 0, "TRUNC_LEN_PREFIX": 1, "TRUNC_KEY": 2, "KEY_TOO_LONG": 3,
            "TRUNC_VLEN": 4, "VAL_TOO_LONG": 5, "TRUNC_VAL": 6, "IDX_OVERRUN": 7}[name]


def test_data_block_trailing_length_bytes():
    # 1-3 bytes where a u32 length is due: ErrUnexpectedEOF (data.go:65-66)
    buf = enc_values([b"value1"])
    for extra in (1, 2, 3):
        b = np.concatenate([buf, np.zeros(extra, np.uint8)])
        st, desc, _ = ora.decode_block(ora.GRAMMAR_V, b, 0, b.size)
        assert st == ora_status("TRUNC_LEN_PREFIX") and len(desc) == 1


# ---- kv/kv_test.go -------------------------------------------------------------

@pytest.mark.parametrize("case", REF["kv_pairs"])
def test_kv_pair_roundtrip(case):
    k = bytes.fromhex(case["key"])
    v = bytes.fromhex(case["value"])
    keys, koff = csr([k])
    vals, voff = csr([v])
    buf = ora.encode_records(ora.GRAMMAR_KV, keys, koff, vals, voff, 0, 1)
    assert buf.tobytes() == struct.pack("<I", len(k)) + k + struct.pack("<I", len(v)) + v
    st, desc, _ = ora.decode_block(ora.GRAMMAR_KV, buf, 0, buf.size)
    assert st == 0 and len(desc) == 1
    ka, va = ora.materialize(ora.GRAMMAR_KV, buf, desc)
    assert ka.tobytes() == k and va.tobytes() == v
    is_deleted = va.tobytes() == bytes.fromhex(REF["tombstone"]["bytes"])
    assert is_deleted == ("deleted" in case["src"] or k == b"deleted_key")


def test_kv_caps_and_truncations():
    # kv.go:84 klen > 1<<20 ; kv.go:102 vlen > 1<<30
    assert ora.decode_block(ora.GRAMMAR_KV, struct.pack("<I", (1 << 20) + 1) + bytes(8))[0] == 3
    assert ora.decode_block(ora.GRAMMAR_KV, struct.pack("<I", 1 << 20))[0] == 2
    b = struct.pack("<I", 1) + b"k" + struct.pack("<I", (1 << 30) + 1)
    assert ora.decode_block(ora.GRAMMAR_KV, b)[0] == 5
    b = struct.pack("<I", 1) + b"k" + struct.pack("<I", 1 << 30)
    assert ora.decode_block(ora.GRAMMAR_KV, b)[0] == 6
    assert ora.decode_block(ora.GRAMMAR_KV, struct.pack("<I", 1) + b"k" + b"\1\0")[0] == 4
    assert ora.decode_block(ora.GRAMMAR_KV, b"\1\0")[0] == 1


@pytest.mark.parametrize("val", REF["key_values"] + REF["value_values"])
def test_key_value_roundtrip(val):
    # Key.EncodeTo / Value.EncodeTo share the [u32 len][bytes] form (kv.go:124-200)
    v = bytes.fromhex(val)
    buf = enc_values([v])
    st, desc, _ = ora.decode_block(ora.GRAMMAR_V, buf, 0, buf.size)
    assert st == 0 and desc[0]["val_len"] == len(v)


def test_tombstone_bytes():
    t = REF["tombstone"]
    assert len(bytes.fromhex(t["bytes"])) == t["len"] == 13


# ---- sstable/bloom ---------------------------------------------------------------

def test_mmh3_smhasher_verification():
    assert ora.mmh3_verification() == int(REF["murmur"]["smhasher_verification_mmh3_x64_128"], 16)


def test_sum256_equals_mmh3_pair_basic():
    # murmur_test.go:12-35 over data = [0,1,...,len-1], len 0..1000
    big = (np.arange(1001) % 256).astype(np.uint8)
    h = ORV["sum256_0_1000"]
    for n in range(0, 1001):
        d = big[:n]
        s = ora.sum256(d)
        assert s == tuple(int(x) for x in h[n])
        assert s == ora.mmh3_x64_128(d) + ora.mmh3_x64_128(np.append(d, np.uint8(1)))


def test_sum256_equals_mmh3_pair_random():
    # murmur_test.go:46-70 (random data)
    rng = np.random.default_rng(7)
    for n in list(range(0, 64)) + [127, 128, 255, 256, 999, 1000]:
        for _ in range(3):
            d = rng.integers(0, 256, n, dtype=np.uint8)
            assert ora.sum256(d) == ora.mmh3_x64_128(d) + ora.mmh3_x64_128(np.append(d, np.uint8(1)))


def test_bloom_basic():
    c = REF["bloom_basic"]
    f = ora.Bloom(c["m"], c["k"])
    f.add(c["add"].encode())
    n3a = f.test_and_add(c["test_and_add"].encode())
    assert f.test(c["add"].encode())
    assert not f.test(c["absent"].encode())
    assert not n3a
    assert f.test(c["test_and_add"].encode())


def test_bloom_string_estimates():
    c = REF["bloom_string"]
    m, k = ora.estimate_parameters(c["n"], c["p"])
    assert (m, k) == (c["expect_m"], c["expect_k"])
    f = ora.Bloom(m, k)
    f.add(b"Love")
    n3a = f.test_and_add(b"in")
    assert f.test(b"Love") and not f.test(b"is") and f.test(b"in") and not n3a
    assert not f.test(b"blooms")
    f.add(b"blooms")
    assert f.test(b"blooms")


def test_bloom_fpp():
    c = REF["bloom_fpp"]
    m, k = ora.estimate_parameters(c["n"], c["p"])
    f = ora.Bloom(m, k)
    for i in range(1000):
        f.add(struct.pack(">I", i))
    fp = sum(f.test(struct.pack(">I", i + 1000)) for i in range(1000))
    assert fp / 1000.0 <= c["max_fpp"]


def test_bloom_approximated_size():
    c = REF["bloom_approx_size"]
    m, k = ora.estimate_parameters(1000, 0.001)
    f = ora.Bloom(m, k)
    for key in c["keys"]:
        f.add(key.encode())
    x = float(sum(bin(int(w)).count("1") for w in f.words))
    size = -1 * m / k * math.log(1 - x / m)
    assert int(math.floor(size + 0.5)) == c["expect"]


def test_bloom_location_chi_square():
    c = REF["bloom_location_chi2"]
    m, k, rounds = c["m"], c["k"], c["rounds"]
    counts = np.zeros(m)
    hs = np.zeros(4, np.uint64)
    for x in range(rounds):
        h = ora.sum256(struct.pack("<I", x))
        hs[:] = h
        for i in range(k):
            counts[ora.lib().ora_location(hs.ctypes.data, i) % m] += 1
    e = k * rounds / m
    chi = float(((counts - e) ** 2 / e).sum())
    assert chi < c["crit_df7"]


def test_filter_encode_decode():
    c = REF["bloom_filter_encode"]
    f = ora.Bloom(c["m"], c["k"])
    for key in c["keys"]:
        f.add(key.encode())
    blob = f.encode()
    nw = (c["m"] + 63) // 64
    assert blob.size == 8 + 24 + 8 * nw
    assert struct.unpack("<Q", blob[:8].tobytes())[0] == 24 + 8 * nw
    assert struct.unpack(">QQQ", blob[8:32].tobytes()) == (c["m"], c["k"], c["m"])
    g, nbits, used = ora.Bloom.decode(blob)
    assert (g.m, g.k, nbits, used) == (c["m"], c["k"], c["m"], blob.size)
    assert np.array_equal(g.words, f.words)
    for key in c["keys"]:
        assert g.test(key.encode())
    assert not g.test(c["absent"].encode())


# ---- builder / .sst ------------------------------------------------------------------

def test_builder_flush_boundary():
    thr = REF["builder"]["max_sstable_size"]
    half = thr // 2
    # two records of EstimateSize exactly thr/2 -> flush exactly at 2 MiB (>=)
    koff = np.zeros(3, np.uint64)
    voff = np.array([0, half - 16, 2 * (half - 16)], np.uint64)
    assert ora.segment_files(koff, voff, thr).tolist() == [0, 2]
    voff = np.array([0, half - 16, 2 * (half - 16) - 1], np.uint64)  # thr - 1: no flush
    assert ora.segment_files(koff, voff, thr).tolist() == [0, 2]
    # three records where the flush happens after the second
    voff = np.array([0, half - 16, 2 * (half - 16), 2 * (half - 16) + 5], np.uint64)
    koff = np.zeros(4, np.uint64)
    assert ora.segment_files(koff, voff, thr).tolist() == [0, 2, 3]
    assert ora.segment_files(koff, voff, 0).tolist() == [0, 3]


def test_sst_worked_example():
    w = REF["sst_worked_example"]
    n = 40000
    koff = np.arange(n + 1, dtype=np.uint64) * 16
    voff = np.arange(n + 1, dtype=np.uint64) * 100
    starts = ora.segment_files(koff, voff, REF["builder"]["max_sstable_size"])
    assert int(starts[1] - starts[0]) == w["records_per_file"]
    size = ora.lib().ora_sst_image_size(koff.ctypes.data, voff.ctypes.data, 0,
                                        w["records_per_file"], 1_600_000)
    assert size == w["file_bytes"]
    assert w["header"] + w["filter"] + w["data"] + w["index"] + w["footer"] == w["file_bytes"]


def _sst_from(keys, values, m=1_600_000, k=16):
    kd, koff = csr([x.encode() for x in keys])
    vd, voff = csr([x.encode() for x in values])
    return ora.build_sst(kd, koff, vd, voff, 0, len(keys), m=m, k=k)


def test_sst_sample_roundtrip():
    c = REF["sst_sample"]
    img, footer = _sst_from(c["keys"], c["values"])
    assert np.array_equal(img, ORV["sst_sample"])
    rc, meta, idesc, ival, ddesc = ora.sst_decode(img)
    assert rc == 0 and meta.nidx == 2 and meta.ndata == 2
    hdr_min = img[meta.min_key_off:meta.min_key_off + meta.min_key_len].tobytes()
    hdr_max = img[meta.max_key_off:meta.max_key_off + meta.max_key_len].tobytes()
    assert (hdr_min, hdr_max) == (b"key1", b"key2")
    assert (meta.filter_m, meta.filter_k) == (1_600_000, 16)
    assert meta.data_off == 8 + 8 + 200032 and footer[0] == meta.data_off
    for i in range(2):
        key = img[idesc[i]["rec_off"] + 4:idesc[i]["rec_off"] + 4 + idesc[i]["key_len"]]
        val = img[ddesc[i]["rec_off"] + 4:ddesc[i]["rec_off"] + 4 + ddesc[i]["val_len"]]
        assert key.tobytes() == c["keys"][i].encode()
        assert val.tobytes() == c["values"][i].encode()
        # GetValueByOffset(Indexes[i].Offset) (sstable.go:271-296)
        assert ival[i] == ddesc[i]["rec_off"]
    # MayContain via the decoded filter (sstable.go:300-305)
    f, _, _ = ora.Bloom.decode(img[meta.max_key_off + meta.max_key_len:])  # after the header
    assert f.test(b"key1") and f.test(b"key2") and not f.test(b"nonexistent")


def test_sst_iterator_fixture():
    c = REF["sst_iterator"]
    img, _ = _sst_from(c["keys"], c["values"], m=c["m"], k=c["k"])
    assert np.array_equal(img, ORV["sst_iter"])
    rc, meta, idesc, ival, ddesc = ora.sst_decode(img)
    assert rc == 0 and meta.ndata == 5
    vals = [img[d["rec_off"] + 4:d["rec_off"] + 4 + d["val_len"]].tobytes() for d in ddesc]
    assert vals == [v.encode() for v in c["values"]]


def test_sst_header_cases():
    for mn, mx in REF["header"]["cases"]:
        keys = [mn, mx] if mn != mx else [mn]
        img, _ = _sst_from(keys, ["v"] * len(keys))
        rc, meta, *_ = ora.sst_decode(img)
        assert rc == 0
        assert img[meta.min_key_off:meta.min_key_off + meta.min_key_len].tobytes() == mn.encode()
        assert img[meta.max_key_off:meta.max_key_off + meta.max_key_len].tobytes() == mx.encode()


def test_sst_empty_table_quirk():
    # TestEmptyDataBlock (sstable_test.go:402-415): EncodeTo/DecodeFrom of an empty
    # table succeed.  DecodeDataBlock with DataHandle.Size == 0 reads unlimited to EOF
    # (data.go:51-54) and trips on the footer bytes -- stage 5 in the oracle.
    img, footer = _sst_from([], [])
    assert footer[1] == 0 and footer[3] == 0
    rc, meta, idesc, ival, ddesc = ora.sst_decode(img)
    assert meta.nidx == 0
    assert rc == 5 and meta.status == ora_status("TRUNC_VAL")


def test_sst_corrupted_header():
    # TestDecodeFrom_CorruptedHeader (sstable_test.go:310-323)
    rc, meta, *_ = ora.sst_decode(np.frombuffer(b"invalid data", np.uint8))
    assert rc == 1


def test_footer_cases():
    # footer_test.go: footer = 4 x i64le; ^int64(0) == -1
    for case in REF["footer"]["cases"]:
        b = struct.pack("<qqqq", *case)
        assert len(b) == REF["footer"]["footer_size"]
        assert struct.unpack("<qqqq", b) == tuple(case)


def test_merge_basic_vector():
    """merge_test.go:12-60 through the merge oracle (both tie orders), and the
    one table it builds: its keys, values and filter."""
    v = REF["merge_basic"]
    pairs = [(k.encode(), x.encode()) for k, x in v["pairs"]]
    for tie in (ora.TIE_INPUT, ora.TIE_GOHEAP):
        out, starts = ora.merge_pairs(pairs, v["level"], 2 * 1024 * 1024, tie)
        assert [pairs[i][0].decode() for i in out] == v["expect_keys"]
        assert [pairs[i][1].decode() for i in out] == v["expect_values"]
        assert len(starts) - 1 == v["expect_tables"]
    keys = b"".join(pairs[i][0] for i in out)
    vals = b"".join(pairs[i][1] for i in out)
    koff = np.concatenate([[0], np.cumsum([len(pairs[i][0]) for i in out])]).astype(np.uint64)
    voff = np.concatenate([[0], np.cumsum([len(pairs[i][1]) for i in out])]).astype(np.uint64)
    img, _ = ora.build_sst(np.frombuffer(keys, np.uint8), koff, np.frombuffer(vals, np.uint8),
                           voff, 0, len(out))
    rc, meta, *_ = ora.sst_decode(img)
    assert rc == 0 and meta.nidx == 4
    hdr = 8 + meta.min_key_len + meta.max_key_len
    f, _, _ = ora.Bloom.decode(img[hdr:])
    assert all(f.test(k.encode()) for k in v["may_contain"])
    assert not any(f.test(k.encode()) for k in v["absent"])
