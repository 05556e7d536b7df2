"""GPU parity of lsm_merge_kvs / lsm_gather_kvs (the compaction merge,
CompactAndMergeKVs merge.go:42-94) against the oracle
(ora_merge_kvs, ORA_TIE_INPUT: equal keys in input order, merge.go:41's
contract -- see test_merge_oracle.py for the heap's own order).

Bit-exact: the written pairs' input indices, the file starts, the gathered
CSR batch and, end to end, the .sst images built from the merge.
"""
import random

import numpy as np
import pytest
import torch

import lsmgpu
import pyoracle as ora

pytestmark = pytest.mark.gpu

TOMB = lsmgpu.TOMBSTONE
MiB2 = 2 * 1024 * 1024


def lay_out(pairs, kv_layout, rng, align4=False):
    """Pairs as descriptors over one byte buffer, stored in shuffled order.
    kv_layout: KV records [klen][key][vlen][value] (value desc = None);
    else keys and values apart, each after 4 bytes of padding (IDX / V
    descriptor convention: bytes at rec_off + 4)."""
    n = len(pairs)
    place = list(range(n))
    rng.shuffle(place)
    parts, pos = [], 0
    kpos, vpos = np.zeros(n, np.uint64), np.zeros(n, np.uint64)
    kd = np.zeros(n, lsmgpu.DESC_DTYPE)
    vd = np.zeros(n, lsmgpu.DESC_DTYPE)
    for i in place:
        k, v = pairs[i]
        gap = 4 * rng.randint(0, 2) if align4 else rng.randint(0, 3)
        parts.append(bytes(gap))
        pos += gap
        if kv_layout:
            rec = len(k).to_bytes(4, "little") + k + len(v).to_bytes(4, "little") + v
            kd[i] = (pos, len(k), len(v))
            kpos[i], vpos[i] = pos + 4, pos + 8 + len(k)
            parts.append(rec)
            pos += len(rec)
        else:
            kd[i] = (pos, len(k), 0)
            kpos[i] = pos + 4
            parts.append(b"\xAA" * 4 + k)
            pos += 4 + len(k)
            vd[i] = (pos, 0, len(v))
            vpos[i] = pos + 4
            parts.append(b"\xBB" * 4 + v)
            pos += 4 + len(v)
    buf = np.frombuffer(b"".join(parts) + bytes(16), np.uint8)
    return buf, kd, (None if kv_layout else vd), kpos, vpos


def run(ctx, pairs, level, threshold, kv_layout=False, seed=0, align4=False, tie=0):
    rng = random.Random(seed)
    buf, kd, vd, kpos, vpos = lay_out(pairs, kv_layout, rng, align4)
    dev = ctx.torch_device
    d_buf = lsmgpu.to_device_bytes(buf, dev)
    d_kd = torch.from_numpy(kd.view(np.int32).reshape(-1, 4).copy()).to(dev)
    d_vd = None if vd is None else torch.from_numpy(vd.view(np.int32).reshape(-1, 4).copy()).to(dev)
    r = lsmgpu.merge_kvs(ctx, d_buf, d_kd, d_vd, level=level, threshold=threshold, tie=tie)
    torch.cuda.synchronize()
    got = r.out[:r.nout].cpu().numpy().view(np.uint32)
    starts = r.file_start[:r.nfiles + 1].cpu().numpy().view(np.uint64)
    klen = np.array([len(k) for k, _ in pairs], np.uint32)
    vlen = np.array([len(v) for _, v in pairs], np.uint32)
    want, wstarts = ora.merge_kvs(buf, kpos, klen, vpos, vlen, level, threshold,
                                  ora.TIE_GOHEAP if tie else ora.TIE_INPUT)
    assert np.array_equal(got, want), (level, threshold, got[:20], want[:20])
    assert np.array_equal(starts, wstarts), (level, threshold, starts, wstarts)
    return r, d_buf, d_kd, d_vd, got, starts


def random_pairs(rng, n, alphabet, maxlen, tomb=0.2, maxval=40):
    out = []
    for _ in range(n):
        k = bytes(rng.choice(alphabet) for _ in range(rng.randint(0, maxlen)))
        v = TOMB if rng.random() < tomb else bytes(rng.randint(0, 255) for _ in range(rng.randint(0, maxval)))
        out.append((k, v))
    return out


TIES = [lsmgpu.TIE_INPUT, lsmgpu.TIE_GOHEAP]


@pytest.mark.parametrize("tie", TIES)
def test_reference_vector(ctx, tie):
    pairs = [(b"alpha", b"A"), (b"beta", b"B"), (b"beta", b"B2"), (b"carrot", b"C"), (b"delta", b"D")]
    for kv in (False, True):
        _, _, _, _, got, starts = run(ctx, pairs, 1, MiB2, kv_layout=kv, tie=tie)
        assert list(got) == [0, 1, 3, 4] and list(starts) == [0, 4]


@pytest.mark.parametrize("tie", TIES)
def test_edge_sizes(ctx, tie):
    run(ctx, [(b"a", b"b")], 1, MiB2, tie=tie)
    run(ctx, [(b"", TOMB)], 6, MiB2, tie=tie)                      # nothing written: no file
    run(ctx, [(b"", b""), (b"", b"x"), (b"", TOMB)], 6, 1, tie=tie)
    run(ctx, [(b"", b"%d" % i) for i in range(40)] + [(b"q", b"1"), (b"", TOMB)], 1, 30, tie=tie)
    r = lsmgpu.merge_kvs(ctx, torch.zeros(16, dtype=torch.uint8, device=ctx.torch_device),
                         torch.zeros((0, 4), dtype=torch.int32, device=ctx.torch_device), None,
                         tie=tie)
    assert r.nout == 0 and r.nfiles == 0


@pytest.mark.parametrize("tie", TIES)
@pytest.mark.parametrize("level", [1, 6])
@pytest.mark.parametrize("threshold", [1, 60, 700, MiB2])
def test_random_duplicates_tombstones_flushes(ctx, level, threshold, tie):
    """Short keys over a 4-letter alphabet with zero bytes (prefix, padding
    and "a" < "a\\0" order), many duplicates, tombstones, and thresholds
    that flush inside duplicate groups."""
    rng = random.Random(level * 1000 + threshold % 997)
    pairs = random_pairs(rng, 3000, b"ab\x00\xff", 11)
    for kv in (False, True):
        run(ctx, pairs, level, threshold, kv_layout=kv, seed=level, tie=tie)


def test_long_keys_shared_prefixes(ctx):
    """Keys of 0..300 bytes sharing long prefixes: many 8-byte chunk passes."""
    rng = random.Random(4)
    stems = [bytes(rng.randint(0, 255) for _ in range(rng.randint(0, 200))) for _ in range(6)]
    pairs = []
    for _ in range(4000):
        k = rng.choice(stems) + bytes(rng.choice(b"\x00\x01xy") for _ in range(rng.randint(0, 100)))
        pairs.append((k, TOMB if rng.random() < 0.1 else b"v%d" % rng.randint(0, 99)))
    for level, threshold in ((1, MiB2), (6, 5000), (3, 1)):
        run(ctx, pairs, level, threshold)


@pytest.mark.parametrize("tie", TIES)
def test_compaction_shaped_runs(ctx, tie):
    """loadLevelData's shape (compaction.go:173-193): newest files first,
    each sorted and unique, overlapping key ranges; 2 MiB and 64 KiB files.
    Both tie orders against the oracle; they must differ somewhere (the
    heap keeps another pair of some duplicate groups)."""
    rng = np.random.default_rng(6)
    pairs = []
    for r in range(6):
        ids = np.unique(rng.integers(0, 120_000, 40_000))
        for i in ids:
            v = TOMB if (i * 7 + r) % 23 == 0 else b"r%d_" % r + b"x" * int(i % 90)
            pairs.append((b"key%012d" % i, v))
    outs = []
    for level, threshold in ((1, MiB2), (6, MiB2), (2, 64 * 1024)):
        outs.append(run(ctx, pairs, level, threshold, kv_layout=(level == 2), tie=tie)[4])
    if tie == lsmgpu.TIE_GOHEAP:
        inp = run(ctx, pairs, 1, MiB2)[4]
        assert not np.array_equal(outs[0], inp)


def test_gather_and_build_match_oracle_images(ctx):
    """merge -> gather -> lsm_build_sst: the .sst images equal the oracle's
    images of the oracle's merge (sstable.go:131-193 on merge.go's output)."""
    rng = random.Random(11)
    pairs = random_pairs(rng, 6000, b"abcdefgh", 14, tomb=0.1, maxval=300)
    r, d_buf, d_kd, d_vd, got, starts = run(ctx, pairs, 6, 200_000)
    kb = sum(len(k) for k, _ in pairs)
    vb = sum(len(v) for _, v in pairs)
    batch = lsmgpu.gather_kvs(ctx, d_buf, d_kd, d_vd, r.out, r.nout, kb, vb)
    torch.cuda.synchronize()
    keys = b"".join(pairs[i][0] for i in got)
    vals = b"".join(pairs[i][1] for i in got)
    koff = np.concatenate([[0], np.cumsum([len(pairs[i][0]) for i in got])]).astype(np.uint64)
    voff = np.concatenate([[0], np.cumsum([len(pairs[i][1]) for i in got])]).astype(np.uint64)
    assert np.array_equal(batch.koff.cpu().numpy().view(np.uint64), koff)
    assert np.array_equal(batch.voff.cpu().numpy().view(np.uint64), voff)
    assert batch.keys[:len(keys)].cpu().numpy().tobytes() == keys
    assert batch.vals[:len(vals)].cpu().numpy().tobytes() == vals
    assert r.max_recs == int(np.diff(starts.astype(np.int64)).max())
    sb = lsmgpu.prepare_sst_device(ctx, batch, r.file_start, r.nfiles, r.max_recs, m=20_000, k=5)
    lsmgpu.build_sst_into(ctx, batch, sb)
    torch.cuda.synchronize()
    img = sb.out.cpu().numpy()
    kn, vn = np.frombuffer(keys, np.uint8), np.frombuffer(vals, np.uint8)
    for f in range(r.nfiles):
        want, _ = ora.build_sst(kn, koff, vn, voff, int(starts[f]), int(starts[f + 1]), m=20_000, k=5)
        o = int(sb.file_off[f])
        assert int(sb.file_size[f]) == want.size
        assert np.array_equal(img[o:o + want.size], want), f
    # lsm_sst_layout: 16-byte aligned exclusive offsets, the total in the last
    # entry, inside the bound the buffer was sized by
    pad = (sb.file_size + np.uint64(15)) // np.uint64(16) * np.uint64(16)
    assert np.array_equal(sb.file_off, np.concatenate([[0], np.cumsum(pad)[:-1]]).astype(np.uint64))
    total = int(sb.d_file_off[r.nfiles].item())
    assert total == int(pad.sum()) and total <= sb.out.numel()
    # values read in place: keys-only gather + lsm_build_sst_views, same images
    for kv_layout in (False, True):
        r2, d_buf2, d_kd2, d_vd2, got2, _ = run(ctx, pairs, 6, 200_000, kv_layout=kv_layout)
        kb2 = lsmgpu.gather_kvs(ctx, d_buf2, d_kd2, d_vd2, r2.out, r2.nout, kb, None)
        sb2 = lsmgpu.prepare_sst_device(ctx, kb2, r2.file_start, r2.nfiles, r2.max_recs,
                                        val_bytes=vb, m=20_000, k=5)
        lsmgpu.build_sst_views_into(ctx, kb2, sb2, d_buf2, d_kd2, d_vd2, r2.out)
        torch.cuda.synchronize()
        img2 = sb2.out.cpu().numpy()
        for f in range(r2.nfiles):
            want, _ = ora.build_sst(kn, koff, vn, voff, int(starts[f]), int(starts[f + 1]), m=20_000, k=5)
            o = int(sb2.file_off[f])
            assert np.array_equal(img2[o:o + want.size], want), (kv_layout, f)


def test_build_views_dword_aligned_values(ctx):
    """lsm_build_sst_views when every value is dword-aligned in its source and
    in the image (16-byte keys, value lengths a multiple of 4, as go-lsm's
    benchmark records): the per-record copy path, against the oracle's images,
    including waves that mix aligned and unaligned records."""
    rng = random.Random(21)
    pairs = [(b"k%015d" % rng.randint(0, 5000),
              TOMB if rng.random() < 0.05 else bytes(rng.randint(0, 255) for _ in range(4 * rng.randint(0, 60))))
             for _ in range(5000)]
    mixed = pairs[:2500] + [(k, v + b"x") if i % 97 == 0 else (k, v) for i, (k, v) in enumerate(pairs[2500:])]
    for ps in (pairs, mixed):
        for kv_layout in (False, True):
            r, d_buf, d_kd, d_vd, got, starts = run(ctx, ps, 6, 100_000, kv_layout=kv_layout, align4=True)
            keys = b"".join(ps[i][0] for i in got)
            vals = b"".join(ps[i][1] for i in got)
            koff = np.concatenate([[0], np.cumsum([len(ps[i][0]) for i in got])]).astype(np.uint64)
            voff = np.concatenate([[0], np.cumsum([len(ps[i][1]) for i in got])]).astype(np.uint64)
            kb = lsmgpu.gather_kvs(ctx, d_buf, d_kd, d_vd, r.out, r.nout, len(keys), None)
            sb = lsmgpu.prepare_sst_device(ctx, kb, r.file_start, r.nfiles, r.max_recs,
                                           val_bytes=len(vals), m=20_000, k=5)
            lsmgpu.build_sst_views_into(ctx, kb, sb, d_buf, d_kd, d_vd, r.out)
            torch.cuda.synchronize()
            img = sb.out.cpu().numpy()
            kn, vn = np.frombuffer(keys, np.uint8), np.frombuffer(vals, np.uint8)
            for f in range(r.nfiles):
                want, _ = ora.build_sst(kn, koff, vn, voff, int(starts[f]), int(starts[f + 1]),
                                        m=20_000, k=5)
                o = int(sb.file_off[f])
                assert int(sb.file_size[f]) == want.size
                assert np.array_equal(img[o:o + want.size], want), (kv_layout, f)


def test_sst_pairs_join(ctx):
    """lsm_sst_pairs = loadLevelData's allPairs: every decoded file's
    (index key, data value) pairs in file order; failed files contribute
    nothing (their GetDataBlockFromFile error aborts the Go caller instead)."""
    rng = random.Random(13)
    images = []
    for f in range(5):
        keys = sorted({b"f%d_%05d" % (f % 3, rng.randint(0, 99999)) for _ in range(rng.randint(0, 400))})
        kb = b"".join(keys)
        ko = np.concatenate([[0], np.cumsum([len(k) for k in keys])]).astype(np.uint64)
        vals = [bytes(rng.randint(0, 255) for _ in range(rng.randint(0, 50))) for _ in keys]
        vo = np.concatenate([[0], np.cumsum([len(v) for v in vals])]).astype(np.uint64)
        img, _ = ora.build_sst(np.frombuffer(kb, np.uint8), ko, np.frombuffer(b"".join(vals) or b"\0", np.uint8),
                               vo, 0, len(keys), m=4096, k=3)
        images.append((img, keys, vals))
    bad = images[1][0].copy()
    bad[:4] = 255  # header length past the end: stage 1
    images[1] = (bad, [], [])
    offs, pos, parts = [], 0, []
    for img, _, _ in images:
        gap = rng.randint(0, 40)
        parts += [np.zeros(gap, np.uint8), img]
        pos += gap
        offs.append(pos)
        pos += img.size
    buf = np.concatenate(parts)
    d_img = lsmgpu.to_device_bytes(buf, ctx.torch_device)
    r = lsmgpu.decode_sst(ctx, d_img, np.array(offs, np.uint64),
                          np.array([im.size for im, _, _ in images], np.uint64))
    kd, vd, prefix = lsmgpu.sst_pairs(ctx, r)
    torch.cuda.synchronize()
    kd = kd.cpu().numpy().view(lsmgpu.DESC_DTYPE).reshape(-1)
    vd = vd.cpu().numpy().view(lsmgpu.DESC_DTYPE).reshape(-1)
    want = [(k, v) for _, keys, vals in images for k, v in zip(keys, vals)]
    got = [(buf[d["rec_off"] + 4:d["rec_off"] + 4 + d["key_len"]].tobytes(),
            buf[e["rec_off"] + 4:e["rec_off"] + 4 + e["val_len"]].tobytes()) for d, e in zip(kd, vd)]
    assert got == want
    counts = [0 if i == 1 else len(images[i][1]) for i in range(5)]
    assert list(prefix.cpu().numpy()) == list(np.concatenate([[0], np.cumsum(counts)]))


def test_full_size_compaction_merge(ctx):
    """The compact bench's workload at full size (216 images: 8 level-0 update
    flushes + 208 level-1 files, 3.43M pairs) through lsm_decode_sst ->
    lsm_sst_pairs -> lsm_merge_kvs, against ora_merge_kvs on the same views."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench_compact import build_images, level0_runs
    from lsmgpu import synth
    n1 = 100_000 * 33
    img, file_off, file_size = build_images(ctx, level0_runs(n1, 0, 0) + [synth.kv_stream(n1)])
    r = lsmgpu.alloc_sst_decode(ctx, file_off, file_size, int(img.numel()))
    lsmgpu.decode_sst_into(ctx, img, r)
    kd, vd, prefix = lsmgpu.sst_pairs(ctx, r)
    for level in (1, 6):
        m = lsmgpu.merge_kvs(ctx, img, kd, vd, level=level)
        torch.cuda.synchronize()
        got = m.out[:m.nout].cpu().numpy().view(np.uint32)
        starts = m.file_start[:m.nfiles + 1].cpu().numpy().view(np.uint64)
        k = kd.cpu().numpy().view(lsmgpu.DESC_DTYPE).reshape(-1)
        v = vd.cpu().numpy().view(lsmgpu.DESC_DTYPE).reshape(-1)
        want, wstarts = ora.merge_kvs(img.cpu().numpy(), k["rec_off"] + 4, k["key_len"],
                                      v["rec_off"] + 4, v["val_len"], level, MiB2, ora.TIE_INPUT)
        assert np.array_equal(got, want) and np.array_equal(starts, wstarts), level
        assert m.nfiles >= 200


def test_full_size_compaction_merge_goheap(ctx):
    """LSM_TIE_GOHEAP at the compact bench's full size (3.43M pairs): the
    reference's exact output (container/heap's own tie order) against
    ora_merge_kvs(ORA_TIE_GOHEAP); prints the call's cost beside the
    input-order path."""
    import os
    import sys
    import time
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench_compact import build_images, level0_runs
    from lsmgpu import synth
    n1 = 100_000 * 33
    img, file_off, file_size = build_images(ctx, level0_runs(n1, 0, 0) + [synth.kv_stream(n1)])
    r = lsmgpu.alloc_sst_decode(ctx, file_off, file_size, int(img.numel()))
    lsmgpu.decode_sst_into(ctx, img, r)
    kd, vd, prefix = lsmgpu.sst_pairs(ctx, r)
    m = lsmgpu.alloc_merge(ctx, int(kd.shape[0]))
    t = {}
    for tie in (lsmgpu.TIE_INPUT, lsmgpu.TIE_GOHEAP):
        lsmgpu.merge_kvs_into(ctx, img, kd, vd, m, level=1, tie=tie)  # warm
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        lsmgpu.merge_kvs_into(ctx, img, kd, vd, m, level=1, tie=tie)
        torch.cuda.synchronize()
        t[tie] = time.perf_counter() - t0
    got = m.out[:m.nout].cpu().numpy().view(np.uint32)
    starts = m.file_start[:m.nfiles + 1].cpu().numpy().view(np.uint64)
    k = kd.cpu().numpy().view(lsmgpu.DESC_DTYPE).reshape(-1)
    v = vd.cpu().numpy().view(lsmgpu.DESC_DTYPE).reshape(-1)
    want, wstarts = ora.merge_kvs(img.cpu().numpy(), k["rec_off"] + 4, k["key_len"],
                                  v["rec_off"] + 4, v["val_len"], 1, MiB2, ora.TIE_GOHEAP)
    assert np.array_equal(got, want) and np.array_equal(starts, wstarts)
    print(f"merge of {k.size} pairs: TIE_INPUT {t[0] * 1e3:.2f} ms, TIE_GOHEAP {t[1] * 1e3:.2f} ms")


def test_full_size_compaction_build(ctx):
    """Exactly what the compact bench times, at full size: decode -> join ->
    merge -> keys-only gather -> lsm_sst_layout -> lsm_build_sst_views, whose
    data regions are copied as runs of whole source records.  The images must
    equal, byte for byte, those lsm_build_sst writes from a gathered copy of
    the values, and three files must equal the oracle's build."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench_compact import build_images, level0_runs
    from lsmgpu import synth
    n1 = 100_000 * 33
    img, file_off, file_size = build_images(ctx, level0_runs(n1, 0, 0) + [synth.kv_stream(n1)])
    r = lsmgpu.alloc_sst_decode(ctx, file_off, file_size, int(img.numel()))
    lsmgpu.decode_sst_into(ctx, img, r)
    kd, vd, prefix = lsmgpu.sst_pairs(ctx, r)
    meta = r.meta_numpy()
    key_bytes = int(meta["idx_size"].astype(np.int64).sum())
    val_bytes = int(meta["data_size"].astype(np.int64).sum())
    m = lsmgpu.merge_kvs(ctx, img, kd, vd, level=1)
    kb = lsmgpu.gather_kvs(ctx, img, kd, vd, m.out, m.nout, key_bytes, None)
    sb = lsmgpu.prepare_sst_device(ctx, kb, m.file_start, m.nfiles, m.max_recs, val_bytes=val_bytes)
    lsmgpu.build_sst_views_into(ctx, kb, sb, img, kd, vd, m.out)
    full = lsmgpu.gather_kvs(ctx, img, kd, vd, m.out, m.nout, key_bytes, val_bytes)
    sb2 = lsmgpu.prepare_sst_device(ctx, full, m.file_start, m.nfiles, m.max_recs)
    lsmgpu.build_sst_into(ctx, full, sb2)
    torch.cuda.synchronize()
    assert m.nfiles >= 200 and m.max_recs == int(np.diff(sb.file_start.astype(np.int64)).max())
    assert np.array_equal(sb.file_off, sb2.file_off) and np.array_equal(sb.file_size, sb2.file_size)
    total = int(sb.d_file_off[m.nfiles].item())
    for f in range(m.nfiles):  # image bytes only: the alignment padding is never written
        o, n = int(sb.file_off[f]), int(sb.file_size[f])
        assert torch.equal(sb.out[o:o + n], sb2.out[o:o + n]), f
    koff = full.koff[:m.nout + 1].cpu().numpy().view(np.uint64)
    voff = full.voff[:m.nout + 1].cpu().numpy().view(np.uint64)
    keys = full.keys[:int(koff[-1]) + 16].cpu().numpy()
    vals = full.vals[:int(voff[-1]) + 16].cpu().numpy()
    out = sb.out[:total].cpu().numpy()
    for f in (0, m.nfiles // 2, m.nfiles - 1):
        want, _ = ora.build_sst(keys, koff, vals, voff, int(sb.file_start[f]), int(sb.file_start[f + 1]))
        o = int(sb.file_off[f])
        assert int(sb.file_size[f]) == want.size
        assert np.array_equal(out[o:o + want.size], want), f


@pytest.mark.parametrize("tie", TIES)
@pytest.mark.parametrize("shape", ["run_last", "run_first", "run_middle", "sorted", "two_runs"])
def test_merge_path_one_long_run(ctx, tie, shape):
    """The merge path (one sorted run holds at least half the pairs): level-0
    style updates (sorted per file, newest first, duplicates of run keys and
    of each other, tombstones, empty keys, a key that is a prefix of
    another) beside one long sorted run; the run at the end, the start or in
    the middle of the input, a fully sorted input (no others) and two runs
    of equal length.  Levels 1 and 6, thresholds that flush inside
    duplicate groups; both tie modes."""
    rng = random.Random(hash(shape) & 0xFFFF)
    base = sorted({b"key%05d" % rng.randint(0, 99999) for _ in range(6000)})
    runp = [(k, b"v" * rng.randint(0, 30)) for k in base]
    l0 = []
    for f in range(4):
        ks = sorted({rng.choice(base) if rng.random() < 0.7 else b"key%05d" % rng.randint(0, 99999)
                     for _ in range(300)})
        l0 += [(k, TOMB if rng.random() < 0.1 else b"u%d" % f) for k in ks]
    l0 += [(b"", b"e"), (b"key0", b"p"), (b"key00000", b"q")]
    if shape == "run_last":
        pairs = l0 + runp
    elif shape == "run_first":
        pairs = runp + l0
    elif shape == "run_middle":
        pairs = l0[:600] + runp + l0[600:]
    elif shape == "sorted":
        pairs = runp
    else:
        half = len(runp) // 2
        pairs = runp[half:] + runp[:half]
    for level in (1, 6):
        for thr in (MiB2, 4000, 257):
            run(ctx, pairs, level, thr, seed=level, tie=tie)


@pytest.mark.parametrize("tie", TIES)
@pytest.mark.parametrize("nfiles", [1, 2, 7, 9, 10, 11, 12, 16, 40])
def test_merge_path_kway_runs(ctx, tie, nfiles):
    """The merge path's others as a k-way merge of their sorted runs (at most
    12, bounded by the input's descent count; more take the radix sort):
    nfiles sorted, overlapping update files before and after one long run,
    keys repeated across the files and with the run (the stable order: the
    earlier file's pair first), tombstones, and file counts on both sides of
    the bound."""
    rng = random.Random(977 + nfiles)
    base = sorted({b"k%06d" % rng.randint(0, 999999) for _ in range(5000)})
    runp = [(k, b"r" * rng.randint(0, 20)) for k in base]
    files = []
    for f in range(nfiles):
        ks = sorted({rng.choice(base) if rng.random() < 0.5 else b"k%06d" % rng.randint(0, 999999)
                     for _ in range(rng.randint(1, 120))})
        files.append([(k, TOMB if rng.random() < 0.1 else b"f%d" % f) for k in ks])
    cut = rng.randint(0, nfiles)
    pairs = [p for fl in files[:cut] for p in fl] + runp + [p for fl in files[cut:] for p in fl]
    for level, thr in ((1, MiB2), (6, 3000)):
        run(ctx, pairs, level, thr, seed=nfiles, tie=tie)


@pytest.mark.parametrize("tie", TIES)
def test_async_merge_and_device_count_gather(ctx, tie):
    """lsm_merge_kvs_async (counts left on the device) + lsm_gather_kvs_dev
    (the gather on that device count, launched on a bound) equal the
    read-back forms: the same written pairs, file starts and counts, and the
    same packed keys, values and offsets."""
    rng = random.Random(31 + tie)
    pairs = random_pairs(rng, 6000, b"abc\x00", 9)
    buf, kd, vd, kpos, vpos = lay_out(pairs, False, random.Random(5))
    dev = ctx.torch_device
    d_buf = lsmgpu.to_device_bytes(buf, dev)
    d_kd = torch.from_numpy(kd.view(np.int32).reshape(-1, 4).copy()).to(dev)
    d_vd = torch.from_numpy(vd.view(np.int32).reshape(-1, 4).copy()).to(dev)
    n = len(pairs)
    for level, threshold in ((1, 900), (6, 4000), (1, MiB2)):
        want = lsmgpu.merge_kvs(ctx, d_buf, d_kd, d_vd, level=level, threshold=threshold, tie=tie)
        got = lsmgpu.alloc_merge(ctx, n)
        d_counts = torch.full((3,), -1, dtype=torch.int64, device=dev)
        lsmgpu.merge_kvs_into(ctx, d_buf, d_kd, d_vd, got, level=level, threshold=threshold,
                              tie=tie, d_counts=d_counts)
        torch.cuda.synchronize()
        cnt = d_counts.cpu().tolist()
        assert cnt == [want.nout, want.nfiles, want.max_recs], (level, threshold)
        assert torch.equal(got.out[:want.nout], want.out[:want.nout])
        assert torch.equal(got.file_start[:want.nfiles + 1], want.file_start[:want.nfiles + 1])
        kb = buf.size + 64  # the input's bytes bound the selected keys and values
        for vb in (None, buf.size + 64):
            a = lsmgpu.gather_kvs(ctx, d_buf, d_kd, d_vd, want.out, want.nout, kb, vb)
            b = lsmgpu.gather_kvs(ctx, d_buf, d_kd, d_vd, got.out, n, kb, vb, d_nout=d_counts)
            torch.cuda.synchronize()
            m = want.nout
            assert torch.equal(a.koff[:m + 1], b.koff[:m + 1]) and torch.equal(a.voff[:m + 1], b.voff[:m + 1])
            kbytes = int(a.koff[m])
            assert torch.equal(a.keys[:kbytes], b.keys[:kbytes])
            if vb is not None:
                vbytes = int(a.voff[m])
                assert torch.equal(a.vals[:vbytes], b.vals[:vbytes])


def test_device_count_above_bound_is_capped(ctx):
    """lsm_gather_kvs_dev with a device count larger than its bound gathers
    exactly `bound` pairs: the offsets, keys and values equal the host-count
    gather of those pairs, and nothing past the bound's koff / voff slot or
    the gathered bytes is written (the count is capped on the
    device, gather_count in merge.hip)."""
    rng = random.Random(77)
    pairs = random_pairs(rng, 3000, b"abc\x00", 9)
    buf, kd, vd, kpos, vpos = lay_out(pairs, False, random.Random(6))
    dev = ctx.torch_device
    d_buf = lsmgpu.to_device_bytes(buf, dev)
    d_kd = torch.from_numpy(kd.view(np.int32).reshape(-1, 4).copy()).to(dev)
    d_vd = torch.from_numpy(vd.view(np.int32).reshape(-1, 4).copy()).to(dev)
    want = lsmgpu.merge_kvs(ctx, d_buf, d_kd, d_vd, level=1)
    bound = want.nout // 2
    idx = torch.zeros(len(pairs), dtype=want.out.dtype, device=dev)  # valid pair ids past the bound
    idx[:bound] = want.out[:bound]
    kb = vb = buf.size + 64
    a = lsmgpu.gather_kvs(ctx, d_buf, d_kd, d_vd, idx, bound, kb, vb)
    guard = 64
    reuse = lsmgpu.codec.RecordBatch(
        keys=torch.full((lsmgpu.pad16(kb) + 4096,), 0xEE, dtype=torch.uint8, device=dev),
        koff=torch.full((bound + 1 + guard,), -7, dtype=torch.int64, device=dev),
        vals=torch.full((lsmgpu.pad16(vb) + 4096,), 0xEE, dtype=torch.uint8, device=dev),
        voff=torch.full((bound + 1 + guard,), -7, dtype=torch.int64, device=dev),
        n=0, koff_host=None, voff_host=None)
    reuse._ws = torch.empty(int(ctx.lib.lsm_gather_kvs_workspace_bytes(bound)), dtype=torch.uint8,
                            device=dev)
    d_nout = torch.tensor([bound + 500], dtype=torch.int64, device=dev)
    b = lsmgpu.gather_kvs(ctx, d_buf, d_kd, d_vd, idx, bound, kb, vb, reuse=reuse, d_nout=d_nout)
    torch.cuda.synchronize()
    assert b.koff.data_ptr() == reuse.koff.data_ptr()
    assert torch.equal(a.koff[:bound + 1], b.koff[:bound + 1])
    assert torch.equal(a.voff[:bound + 1], b.voff[:bound + 1])
    assert bool((b.koff[bound + 1:] == -7).all()) and bool((b.voff[bound + 1:] == -7).all())
    kbytes, vbytes = int(a.koff[bound]), int(a.voff[bound])
    assert torch.equal(a.keys[:kbytes], b.keys[:kbytes]) and torch.equal(a.vals[:vbytes], b.vals[:vbytes])
    assert bool((b.keys[kbytes:] == 0xEE).all()) and bool((b.vals[vbytes:] == 0xEE).all())


def _decode_level(ctx, images, rng):
    offs, pos, parts = [], 0, []
    for im in images:
        gap = 16 * int(rng.integers(0, 3))
        parts += [np.zeros(gap, np.uint8), im]
        pos += gap
        offs.append(pos)
        pos += im.size
        pad = (-pos) % 16
        parts.append(np.zeros(pad, np.uint8))
        pos += pad
    buf = np.concatenate(parts)
    d_img = lsmgpu.to_device_bytes(buf, ctx.torch_device)
    r = lsmgpu.decode_sst(ctx, d_img, np.array(offs, np.uint64), np.array([im.size for im in images], np.uint64))
    return d_img, r


def _compare_compact_merge(ctx, d_img, r, level, threshold, tie):
    """lsm_compact_merge_async against lsm_sst_pairs + lsm_merge_kvs_async."""
    kd, vd, prefix = lsmgpu.sst_pairs(ctx, r)
    n = int(kd.shape[0])
    want = lsmgpu.alloc_merge(ctx, n)
    dc_w = torch.full((3,), -1, dtype=torch.int64, device=ctx.torch_device)
    lsmgpu.merge_kvs_into(ctx, d_img, kd, vd, want, level=level, threshold=threshold, tie=tie, d_counts=dc_w)
    cap = int(r.idx_desc.shape[0])
    kd2 = torch.full((cap, 4), -3, dtype=torch.int32, device=ctx.torch_device)
    vd2 = torch.full((cap, 4), -3, dtype=torch.int32, device=ctx.torch_device)
    pre2 = torch.full((r.nfile + 1,), -3, dtype=torch.int64, device=ctx.torch_device)
    got = lsmgpu.alloc_merge(ctx, n)
    dc_g = torch.full((3,), -1, dtype=torch.int64, device=ctx.torch_device)
    lsmgpu.compact_merge_into(ctx, d_img, r, kd2, vd2, pre2, got, dc_g, level=level, threshold=threshold, tie=tie)
    torch.cuda.synchronize()
    assert torch.equal(pre2, prefix)
    assert torch.equal(kd2[:n], kd) and torch.equal(vd2[:n], vd)
    c = dc_w.cpu().tolist()
    assert dc_g.cpu().tolist() == c
    assert torch.equal(got.out[:c[0]], want.out[:c[0]])
    assert torch.equal(got.file_start[:c[1] + 1], want.file_start[:c[1] + 1])
    return c


@pytest.mark.parametrize("tie", TIES)
def test_compact_merge_matches_two_calls_small(ctx, tie):
    """Images of random sorted runs (tombstones, duplicates across files,
    an empty file and one whose header does not decode -- both contribute no
    pairs, so the statistics' file lookup must step over them) through the
    one-call join + merge and through the two calls: identical join, pairs,
    file starts and counts."""
    rng = np.random.default_rng(808 + tie)
    images = []
    for f in range(9):
        keys = sorted({b"m%05d" % int(x) for x in rng.integers(0, 3000, int(rng.integers(50, 400)))})
        vals = [TOMB if rng.random() < 0.1 else b"v%d" % f * int(rng.integers(1, 5)) for _ in keys]
        kb = np.frombuffer(b"".join(keys), np.uint8)
        ko = np.concatenate([[0], np.cumsum([len(k) for k in keys])]).astype(np.uint64)
        vb = np.frombuffer(b"".join(vals), np.uint8)
        vo = np.concatenate([[0], np.cumsum([len(v) for v in vals])]).astype(np.uint64)
        img, _ = ora.build_sst(kb, ko, vb, vo, 0, len(keys))
        images.append(img.copy())
    empty, _ = ora.build_sst(np.zeros(1, np.uint8), np.zeros(1, np.uint64), np.zeros(1, np.uint8),
                             np.zeros(1, np.uint64), 0, 0)
    broken = images[4].copy()
    broken[0:4] = 255  # header key length past the file: stage 1
    images = images[:2] + [empty] + images[2:4] + [broken] + images[4:]
    d_img, r = _decode_level(ctx, images, rng)
    for level, thr in ((1, MiB2), (6, 3000), (1, 700)):
        _compare_compact_merge(ctx, d_img, r, level, thr, tie)
    # n is an exact precondition: a count other than the join's own
    # (d_prefix[nfile], read back with the key statistics) is refused
    kd, vd, prefix = lsmgpu.sst_pairs(ctx, r)
    n = int(kd.shape[0])
    cap = int(r.idx_desc.shape[0])
    for bad in (n + 1, n - 1, 0):
        kd2 = torch.empty((cap, 4), dtype=torch.int32, device=ctx.torch_device)
        vd2 = torch.empty((cap, 4), dtype=torch.int32, device=ctx.torch_device)
        pre2 = torch.empty((r.nfile + 1,), dtype=torch.int64, device=ctx.torch_device)
        mg = lsmgpu.alloc_merge(ctx, max(bad, 1))
        mg.n = bad
        dc = torch.zeros((3,), dtype=torch.int64, device=ctx.torch_device)
        with pytest.raises(RuntimeError, match="code -1"):
            lsmgpu.compact_merge_into(ctx, d_img, r, kd2, vd2, pre2, mg, dc, tie=tie)


def test_compact_merge_matches_two_calls_full_size(ctx):
    """The compact bench's input (216 images, 3.43M pairs), both tie modes."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench_compact import build_images, level0_runs
    from lsmgpu import synth
    n1 = 100_000 * 33
    img, file_off, file_size = build_images(ctx, level0_runs(n1, 0, 0) + [synth.kv_stream(n1)])
    r = lsmgpu.alloc_sst_decode(ctx, file_off, file_size, int(img.numel()))
    lsmgpu.decode_sst_into(ctx, img, r)
    for tie in TIES:
        c = _compare_compact_merge(ctx, img, r, 1, MiB2, tie)
        assert c[1] >= 200


def test_goheap_distinct_keys_skip_the_replay(ctx):
    """LSM_TIE_GOHEAP on distinct keys: the device's group count equals n, the
    heap would pop in key order, so the host replay is skipped
    (lsm_goheap_replays unchanged) and the output equals both oracle modes
    bit for bit; one duplicate key brings the replay back."""
    rng = random.Random(77)
    keys = rng.sample(range(10 ** 6), 5000)
    pairs = [(b"dk%07d" % k, bytes(rng.randint(0, 255) for _ in range(rng.randint(0, 30)))) for k in keys]
    for level, threshold in ((1, MiB2), (6, 700), (1, 1)):
        before = ctx.lib.lsm_goheap_replays(ctx.handle)
        _, _, _, _, got, starts = run(ctx, pairs, level, threshold, tie=lsmgpu.TIE_GOHEAP)
        assert ctx.lib.lsm_goheap_replays(ctx.handle) == before, "a replay ran on distinct keys"
        _, _, _, _, got_in, starts_in = run(ctx, pairs, level, threshold, tie=lsmgpu.TIE_INPUT)
        assert np.array_equal(got, got_in) and np.array_equal(starts, starts_in)
    dup = pairs + [(pairs[17][0], b"newer")]
    before = ctx.lib.lsm_goheap_replays(ctx.handle)
    run(ctx, dup, 1, MiB2, tie=lsmgpu.TIE_GOHEAP)
    assert ctx.lib.lsm_goheap_replays(ctx.handle) == before + 1
