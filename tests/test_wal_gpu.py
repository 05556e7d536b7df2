"""GPU parity of lsm_wal_replay (wal.Recover, wal/wal.go:95-121; SURVEY.md
§8(f) row f4) against the oracle's KV-grammar restatement.

Logs are shaped by go-lsm's benchmark (keys "k_<i>_<1-10 letters>", values
"v_<i>_<2-20 letters>", Delete tombstones), memtable-sized, and cut or
corrupted the way a crash mid-append or a damaged file leaves them: records
before the error are delivered (Recover already called back for them), the
status names the error.
"""
import struct

import numpy as np
import pytest
import torch

import lsmgpu
import pyoracle as ora
from lsmgpu import synth

pytestmark = pytest.mark.gpu


def replay_and_check(ctx, logs):
    offs, pos, parts = [], 0, []
    for lg in logs:
        offs.append(pos)
        pad = (16 - len(lg) % 16) % 16 + 16
        parts.append(np.frombuffer(lg, np.uint8))
        parts.append(np.zeros(pad, np.uint8))
        pos += len(lg) + pad
    buf = np.concatenate(parts)
    dev = ctx.torch_device
    d = lsmgpu.to_device_bytes(buf, dev)
    off = torch.tensor(np.array(offs, np.uint64).view(np.int64), device=dev)
    ln = torch.tensor(np.array([len(x) for x in logs], np.uint32).view(np.int32), device=dev)
    r = lsmgpu.wal_replay(ctx, d, off, ln)
    torch.cuda.synchronize()
    nrec, status = r.nrec.cpu().numpy(), r.status.cpu().numpy()
    desc = r.desc_numpy()
    bases = r.bases(np.array(offs, np.uint64)).astype(np.int64)
    for w, o in enumerate(offs):
        st, od, _ = ora.decode_block(lsmgpu.GRAMMAR_KV, buf, o, len(logs[w]))
        assert status[w] == st and nrec[w] == len(od), (w, status[w], st, nrec[w], len(od))
        assert np.array_equal(desc[bases[w]:bases[w] + nrec[w]], od), w
    return status, nrec


def test_benchmark_shaped_logs(ctx):
    buf, off, ln, nrec = synth.wal_logs(3, memtable_bytes=96 * 1024)
    logs = [buf[o:o + l].tobytes() for o, l in zip(off, ln)]
    status, got = replay_and_check(ctx, logs)
    assert (status == 0).all() and np.array_equal(got, nrec)
    assert synth.TOMBSTONE in logs[0]


def test_crashed_and_damaged_logs(ctx):
    rng = np.random.default_rng(9)
    buf, off, ln, _ = synth.wal_logs(1, memtable_bytes=32 * 1024, seed=3)
    base = buf[off[0]:off[0] + ln[0]].tobytes()
    logs = [base[:int(rng.integers(1, len(base)))] for _ in range(12)]  # crash mid-append
    logs += [base + bytes(int(rng.integers(1, 4)))]                   # 1-3 stray bytes
    for bad in (2 ** 20 + 1, 2 ** 31, 0xFFFFFFFF):                    # key length over the cap
        at = int(rng.integers(0, 400)) * 0  # first record
        logs.append(base[:at] + struct.pack("<I", bad) + base[at + 4:])
    v = bytearray(base)
    v[len(base) // 2:len(base) // 2 + 4] = b"\xff\xff\xff\x7f"         # garbage mid-log
    logs.append(bytes(v))
    logs.append(b"")                                                  # empty log
    status, _ = replay_and_check(ctx, logs)
    assert status[-1] == 0 and (status[:12] != 0).any()


def test_memtable_sized_logs(ctx):
    """Two full 2 MiB-memtable logs (~44k records each)."""
    buf, off, ln, nrec = synth.wal_logs(2)
    logs = [buf[o:o + l].tobytes() for o, l in zip(off, ln)]
    status, got = replay_and_check(ctx, logs)
    assert (status == 0).all() and np.array_equal(got, nrec)


def test_segments_inside_large_values_and_bad_guesses(ctx):
    """Records longer than a 16 KiB segment (segments with no record start),
    values that look like record headers (the guess of the next segment is
    wrong and the stitch re-chases), and a log longer than max_wal_len."""
    rng = np.random.default_rng(12)
    recs = []
    for i in range(300):
        k = b"key%05d" % i
        if i % 50 == 7:
            v = rng.integers(0, 256, 40_000, dtype=np.uint8).tobytes()  # spans segments
        elif i % 9 == 3:
            # a value made of fake 8-byte KV headers: plausible chains everywhere
            v = (struct.pack("<I", 2) + b"zz" + struct.pack("<I", 6) + b"abcdef") * 30
        else:
            v = rng.integers(97, 123, int(rng.integers(0, 300)), dtype=np.uint8).tobytes()
        recs.append(struct.pack("<I", len(k)) + k + struct.pack("<I", len(v)) + v)
    log = b"".join(recs)
    logs = [log, log[:len(log) // 3], log[: len(log) - 5]]
    replay_and_check(ctx, logs)
    # a log over max_wal_len is chased by one wave
    buf, off, ln, nrec = synth.wal_logs(1, memtable_bytes=64 * 1024, seed=5)
    small = buf[off[0]:off[0] + ln[0]].tobytes()
    dev = ctx.torch_device
    both = [small, log]
    offs = [0, (len(small) + 31) // 16 * 16]
    allb = np.zeros(offs[1] + len(log) + 32, np.uint8)
    allb[:len(small)] = np.frombuffer(small, np.uint8)
    allb[offs[1]:offs[1] + len(log)] = np.frombuffer(log, np.uint8)
    d = lsmgpu.to_device_bytes(allb, dev)
    o = torch.tensor(np.array(offs, np.uint64).view(np.int64), device=dev)
    ln2 = torch.tensor(np.array([len(x) for x in both], np.uint32).view(np.int32), device=dev)
    r = lsmgpu.wal_replay(ctx, d, o, ln2, max_len=len(small))
    torch.cuda.synchronize()
    desc = r.desc_numpy()
    bases = r.bases(np.array(offs, np.uint64)).astype(np.int64)
    for w in range(2):
        st, od, _ = ora.decode_block(lsmgpu.GRAMMAR_KV, allb, offs[w], len(both[w]))
        assert int(r.status[w]) == st and int(r.nrec[w]) == len(od)
        assert np.array_equal(desc[bases[w]:bases[w] + len(od)], od)


def test_bench_sized_replay(ctx):
    """The wal bench's workload at full size: 64 memtable-sized logs, every
    descriptor equal to the oracle's serial chase of each log."""
    buf, off, ln, nrec = synth.wal_logs(64)
    dev = ctx.torch_device
    d = lsmgpu.to_device_bytes(buf, dev)
    o = torch.tensor(np.asarray(off, np.uint64).view(np.int64), device=dev)
    l2 = torch.tensor(np.asarray(ln, np.uint32).view(np.int32), device=dev)
    r = lsmgpu.wal_replay(ctx, d, o, l2)
    torch.cuda.synchronize()
    assert (r.status.cpu().numpy() == 0).all()
    assert np.array_equal(r.nrec.cpu().numpy(), nrec)
    desc = r.desc_numpy()
    bases = r.bases(np.asarray(off, np.uint64)).astype(np.int64)
    for w in range(64):
        st, od, _ = ora.decode_block(lsmgpu.GRAMMAR_KV, buf, int(off[w]), int(ln[w]))
        assert st == 0 and np.array_equal(desc[bases[w]:bases[w] + nrec[w]], od), w


def test_record_spanning_last_share_of_a_segment(ctx):
    """A segment's last lane share (the 64 bytes before a 16 KiB boundary)
    holding a record's value-length field but no record start: the guess
    from that field (phase 1 of the share) leads exactly to the next record
    start, past the share.  That chain has no records and must pass the
    position through (it once reported exit 0 and the log was over-counted).
    Records of 8 B keys and 90-140 B ASCII values make the case common."""
    rng = np.random.Generator(np.random.PCG64(77))
    logs, hits = [], 0
    for _ in range(3):
        parts, pos, vfields, starts = [], 0, [], []
        while pos < 256 * 1024:
            i = len(starts)
            k = b"key%05d" % (i % 100000)
            v = bytes(rng.integers(97, 123, int(rng.integers(90, 141))).astype(np.uint8))
            starts.append(pos)
            vfields.append(pos + 4 + len(k))
            parts.append(struct.pack("<I", len(k)) + k + struct.pack("<I", len(v)) + v)
            pos += 8 + len(k) + len(v)
        lg = b"".join(parts)
        st, vf = np.array(starts), np.array(vfields)
        for b in range(16384, len(lg) - 16384, 16384):
            if not ((st >= b - 64) & (st < b)).any() and ((vf >= b - 64) & (vf < b)).any():
                hits += 1
        logs.append(lg)
    assert hits >= 3, hits  # the case is exercised
    status, got = replay_and_check(ctx, logs)
    assert (status == 0).all()


def _fuzz_log(rng, nbytes, kmax, vmax, ascii_bytes, vbig):
    parts, pos = [], 0
    while pos < nbytes:
        k = int(rng.integers(0, kmax + 1))
        v = int(rng.integers(0, vmax + 1))
        if vbig and rng.random() < 0.02:
            v = int(rng.integers(4096, 40000))  # values spanning whole shares/segments
        lo, hi = (97, 123) if ascii_bytes else (0, 256)
        kb = rng.integers(lo, hi, k).astype(np.uint8).tobytes()
        vb = rng.integers(lo, hi, v).astype(np.uint8).tobytes()
        parts.append(struct.pack("<I", k) + kb + struct.pack("<I", v) + vb)
        pos += 8 + k + v
    return b"".join(parts)


@pytest.mark.parametrize("profile", [
    (16, 100, True, False),    # config-2 record shape
    (24, 300, True, False),    # records near a share's width
    (8, 70, False, False),     # binary lengths-look-alike bytes
    (40, 1200, True, True),    # large values, multi-segment records
    (4, 12, False, False),     # tiny records (dense guesses)
])
def test_fuzz_record_shapes(ctx, profile):
    """Randomized record shapes against the oracle, intact and cut at a
    random point (a crash mid-append), so the share guesses, both stitch
    levels and their fallbacks meet many layouts."""
    kmax, vmax, ascii_bytes, vbig = profile
    rng = np.random.Generator(np.random.PCG64(1000 + kmax * 7 + vmax))
    logs = []
    for i in range(6):
        lg = _fuzz_log(rng, int(rng.integers(20_000, 180_000)), kmax, vmax, ascii_bytes, vbig)
        if i % 2:
            lg = lg[:int(rng.integers(1, len(lg)))]
        logs.append(lg)
    replay_and_check(ctx, logs)


def test_escaped_key_lengths(ctx):
    """Keys of 2^18 - 1 bytes and more: the segment kernel's 4-byte scratch
    entry holds an escape value for such a key length and the compact pass
    re-reads it from the log, the value length from the next record's start.
    Logs long enough for the segment grid (many 16 KiB segments), the long
    keys between ordinary records, intact and cut inside a long key, inside
    its value length and inside the record after it."""
    rng = np.random.default_rng(21)

    def rec(k, v):
        return struct.pack("<I", len(k)) + k + struct.pack("<I", len(v)) + v

    small = [rec(b"k_%d_ab" % i, b"v_%d_xyz" % i) for i in range(3000)]
    longs = [(1 << 18) - 1, 1 << 18, 300_000, (1 << 20)]  # the escape boundary, up to kv.go's cap
    parts, cuts = [], []
    for j, L in enumerate(longs):
        parts += small[j * 500:(j + 1) * 500]
        key = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
        val = rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8).tobytes()
        start = sum(len(p) for p in parts)
        parts.append(rec(key, val))
        cuts += [start + 4 + L // 2, start + 4 + L + 2, start + len(parts[-1]) + 3]
    parts += small[2000:]
    log = b"".join(parts)
    logs = [log] + [log[:c] for c in cuts]
    status, nrec = replay_and_check(ctx, logs)
    assert status[0] == 0 and nrec[0] == 3000 + len(longs)
    assert (status[1:] != 0).all()
