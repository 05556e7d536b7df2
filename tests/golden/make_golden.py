"""Writes tests/golden/reference_vectors.json and tests/golden/oracle_vectors.npz.

reference_vectors.json: the inputs and expected outcomes that go-lsm's own
tests hold for the hot path, transcribed as data (file:line cited per case).
Expected bytes that those tests construct with encoding/binary are spelled
out here byte by byte from the Go semantics (e.g. index_test.go:13-58).

oracle_vectors.npz: seeded small inputs with the CPU restatement's outputs
(sum256 over [0..len) for len 0..1000 as murmur_test.go:12-35 does, and
small .sst images).  Those values are produced by oracle/ in this
container; sum256 is cross-checked against the independent SMHasher MMH3
whose published verification value (0x6384BA69) is asserted before writing.

Run:  python tests/golden/make_golden.py
"""
import json
import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import pyoracle as ora  # noqa: E402


def u32(v):
    return struct.pack("<I", v)


def i64(v):
    return struct.pack("<q", v)


def hexs(b):
    return bytes(b).hex()


def reference_vectors():
    v = {}
    # index_test.go:13-58 TestIndexEntry_Encode — the only exact-byte KAT.
    v["index_entry_encode"] = [
        {"src": "sstable/block/index_test.go:20-33", "key": "key1", "offset": 123,
         "bytes": hexs(u32(4) + b"key1" + i64(123))},
        {"src": "sstable/block/index_test.go:34-46", "key": "", "offset": 0,
         "bytes": hexs(u32(0) + i64(0))},
    ]
    # index_test.go:60-89 TestIndexBlock_EncodeDecode; :126-154 size limits.
    v["index_block"] = {
        "src": "sstable/block/index_test.go:60-154",
        "entries": [["key1", 100], ["key2", 200], ["key3", 300]],
        "partial_size_first_entry": 4 + 4 + 8,
        "truncate_by": 2,
    }
    # data_test.go:13-87 TestDataBlock_EncodeDecode
    v["data_block_roundtrip"] = [
        {"src": "sstable/block/data_test.go:20-25", "entries": [], "size": 0},
        {"src": "sstable/block/data_test.go:26-31", "entries": ["value1"], "size": 0},
        {"src": "sstable/block/data_test.go:32-37", "entries": ["value1", "value2", "value3"], "size": 0},
        {"src": "sstable/block/data_test.go:38-43", "entries": ["value1", "value2"], "size": 100},
        {"src": "sstable/block/data_test.go:44-56", "entries": ["value1", "value2"], "size": 20},
    ]
    # data_test.go:89-131 TestDataBlock_DecodeWithSizeLimit
    v["data_block_size_limit"] = {
        "src": "sstable/block/data_test.go:89-131",
        "entries": ["value1", "value2", "value3"],
        "insufficient": {"size": 9, "error": True},
        "partial": {"size": 20, "error": False, "count": 2},
    }
    # data_test.go:133-162 TestDataBlock_DecodeCorruptedData
    v["data_block_corrupt"] = [
        {"src": "sstable/block/data_test.go:135-147", "bytes": hexs(u32(999999)), "error": True},
        {"src": "sstable/block/data_test.go:149-161", "bytes": hexs(u32(10) + b"incom"),
         "error": True},
    ]
    # kv_test.go:10-104 TestKeyValuePair_EncodeDecode
    v["kv_pairs"] = [
        {"src": "kv/kv_test.go:17-25", "key": hexs(b"test_key"), "value": hexs(b"test_value")},
        {"src": "kv/kv_test.go:26-34", "key": "", "value": hexs(b"value_only")},
        {"src": "kv/kv_test.go:35-43", "key": hexs(b"key_only"), "value": ""},
        {"src": "kv/kv_test.go:44-52", "key": hexs(b"deleted_key"),
         "value": hexs("～DELETED～".encode())},
        {"src": "kv/kv_test.go:53-61", "key": hexs(b"large_key_" + bytes(1000)),
         "value": hexs(bytes(2000))},
    ]
    v["tombstone"] = {"src": "kv/kv.go:30", "bytes": hexs("～DELETED～".encode()), "len": 13}
    # kv_test.go:126-211 Key / Value round trips
    v["key_values"] = [hexs(b"test_key"), "", hexs(bytes(1000))]
    v["value_values"] = [hexs(b"test_value"), "", hexs("～DELETED～".encode()), hexs(bytes(2000))]
    # footer_test.go:10-127: handle 16 B, footer 32 B; ^int64(0) == -1.
    v["footer"] = {
        "src": "sstable/block/footer_test.go:10-127",
        "handle_size": 16, "footer_size": 32,
        "cases": [[0, 0, 0, 0], [100, 200, 300, 400], [-1, -1, -1, -1]],
        "handle_cases": [[0, 0], [1234, 5678], [-1, -1]],
    }
    # header_test.go:14-123
    v["header"] = {"src": "sstable/block/header_test.go:14-45",
                   "cases": [["key1", "key2"], ["", "key2"], ["same", "same"]]}
    # bloom_test.go behavioural KATs
    v["bloom_basic"] = {"src": "sstable/bloom/bloom_test.go:13-29", "m": 1000, "k": 4,
                        "add": "Bess", "test_and_add": "Emma", "absent": "Jane"}
    v["bloom_string"] = {"src": "sstable/bloom/bloom_test.go:98-119", "n": 1000, "p": 0.001,
                         "expect_m": 14378, "expect_k": 10}
    v["bloom_fpp"] = {"src": "sstable/bloom/bloom_test.go:386-409", "n": 1000, "p": 0.001,
                      "max_fpp": 0.001}
    v["bloom_approx_size"] = {"src": "sstable/bloom/bloom_test.go:376-384",
                              "keys": ["Love", "is", "in", "bloom"], "expect": 4}
    v["bloom_location_chi2"] = {"src": "sstable/bloom/bloom_test.go:158-213", "m": 8, "k": 3,
                                "rounds": 100000, "crit_df7": 20.278}
    v["bloom_filter_encode"] = {"src": "sstable/bloom/bloom_test.go:433-458", "m": 1024, "k": 5,
                                "keys": ["apple", "banana", "cherry"], "absent": "durian"}
    # builder_test.go:48-78 ShouldFlush boundary; sstable.go:21
    v["builder"] = {"src": "sstable/builder_test.go:48-78", "max_sstable_size": 2 * 1024 * 1024,
                    "estimate_size": "4+k+4+v+8 (kv.go:118-121)"}
    # SURVEY.md §8 worked example (README.md:83 "2.2M")
    v["sst_worked_example"] = {"records_per_file": 15888, "file_bytes": 2297320,
                               "header": 40, "filter": 200032, "data": 1652352,
                               "index": 444864, "footer": 32}
    # sstable_test.go:29-55 createSampleSSTable; iterator_test.go:15-49
    v["sst_sample"] = {"src": "sstable/sstable_test.go:29-55",
                       "keys": ["key1", "key2"], "values": ["value1", "value2"]}
    v["sst_iterator"] = {"src": "sstable/iterator_test.go:15-49", "m": 1024, "k": 5,
                         "keys": ["a", "b", "c", "d", "e"], "values": ["A", "B", "C", "D", "E"]}
    # merge_test.go:12-60 TestCompactAndMergeBlocks_Basic: sorted, deduplicated,
    # the first "beta" (B) kept, one level-1 table of 4 entries
    v["merge_basic"] = {"src": "sstable/merge_test.go:12-60", "level": 1,
                        "pairs": [["alpha", "A"], ["beta", "B"], ["beta", "B2"], ["carrot", "C"],
                                  ["delta", "D"]],
                        "expect_keys": ["alpha", "beta", "carrot", "delta"],
                        "expect_values": ["A", "B", "C", "D"], "expect_tables": 1,
                        "may_contain": ["alpha", "delta"], "absent": ["nonexistent", "deletedKey"]}
    v["murmur"] = {"src": "sstable/bloom/murmur_test.go:12-35", "max_len": 1000,
                   "smhasher_verification_mmh3_x64_128": "0x6384ba69"}
    return v


def oracle_vectors():
    assert ora.mmh3_verification() == 0x6384BA69, "independent MMH3 is not SMHasher-exact"
    big = np.arange(1000, dtype=np.int64).astype(np.uint8)
    h = np.zeros((1001, 4), dtype=np.uint64)
    for n in range(1001):
        d = big[:n]
        s = ora.sum256(d)
        a = ora.mmh3_x64_128(d)
        b = ora.mmh3_x64_128(np.concatenate([d, np.array([1], np.uint8)]))
        assert s == a + b, n
        h[n] = s
    # sample .sst (sstable_test.go:29-55 data, default bloom)
    keys = np.frombuffer(b"key1key2", np.uint8)
    vals = np.frombuffer(b"value1value2", np.uint8)
    koff = np.array([0, 4, 8], np.uint64)
    voff = np.array([0, 6, 12], np.uint64)
    sst, footer = ora.build_sst(keys, koff, vals, voff, 0, 2)
    # iterator_test.go data with m=1024,k=5
    keys2 = np.frombuffer(b"abcde", np.uint8)
    vals2 = np.frombuffer(b"ABCDE", np.uint8)
    ko2 = np.arange(6, dtype=np.uint64)
    sst2, footer2 = ora.build_sst(keys2, ko2, vals2, ko2, 0, 5, m=1024, k=5)
    return {"sum256_0_1000": h, "sst_sample": sst, "sst_sample_footer": footer,
            "sst_iter": sst2, "sst_iter_footer": footer2}


def main():
    with open(os.path.join(HERE, "reference_vectors.json"), "w") as f:
        json.dump(reference_vectors(), f, indent=1, sort_keys=True)
    np.savez_compressed(os.path.join(HERE, "oracle_vectors.npz"), **oracle_vectors())
    print("wrote", HERE)


if __name__ == "__main__":
    main()
