"""Seeded synthetic workloads of BASELINE.json's configs.

Keys are 16 bytes, b"k" + the 15-digit global record index (sorted, unique);
values are splitmix64 bytes of (seed, global record index), so any subset of
blocks (e.g. one rank's round-robin share) is generated independently and
identically.  Seed 0x5EED.
"""
import numpy as np

SEED = 0x5EED
KEY_LEN = 16
VAL_LEN = 100
RECS_PER_4K = 33          # 33 x (8+16+100) = 4092 bytes
SLOT_4K = 4096

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x: np.ndarray) -> np.ndarray:
    """Vectorized splitmix64 finalizer over uint64 counters."""
    with np.errstate(over="ignore"):
        z = x.astype(np.uint64) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def keys_for(idx: np.ndarray) -> np.ndarray:
    """(n, 16) uint8 keys b"k%015d" % idx."""
    idx = np.asarray(idx, dtype=np.int64)
    out = np.empty((idx.size, KEY_LEN), dtype=np.uint8)
    out[:, 0] = ord("k")
    v = idx.copy()
    for d in range(KEY_LEN - 1, 0, -1):
        out[:, d] = ord("0") + (v % 10)
        v //= 10
    return out


def value_bytes(gidx: np.ndarray, vlen: int, seed: int = SEED) -> np.ndarray:
    """(n, vlen) uint8 pseudo-random value bytes of global records gidx."""
    gidx = np.asarray(gidx, dtype=np.uint64)
    nw = (vlen + 7) // 8
    with np.errstate(over="ignore"):
        ctr = (np.uint64(seed) << np.uint64(40)) + gidx[:, None] * np.uint64(64) + \
            np.arange(nw, dtype=np.uint64)[None, :]
    words = splitmix64(ctr)
    return words.view(np.uint8).reshape(gidx.size, nw * 8)[:, :vlen]


def uniform_kv_blocks(block_ids, recs: int = RECS_PER_4K, klen: int = KEY_LEN,
                      vlen: int = VAL_LEN, slot: int = SLOT_4K, seed: int = SEED):
    """KV-grammar blocks in fixed slots (config 2 / 4).

    Returns (buf uint8[nblk*slot], blk_off uint64[nblk], blk_len uint32[nblk]).
    Block b holds global records block_ids[b]*recs + (0..recs-1)."""
    block_ids = np.asarray(block_ids, dtype=np.int64)
    nblk = block_ids.size
    rs = 8 + klen + vlen
    used = recs * rs
    assert used <= slot
    buf = np.zeros((nblk, slot), dtype=np.uint8)
    g = (block_ids[:, None] * recs + np.arange(recs)[None, :]).reshape(-1)
    r = buf[:, :used].reshape(nblk, recs, rs)
    r[:, :, 0:4] = np.frombuffer(np.uint32(klen).tobytes(), dtype=np.uint8)
    if klen:
        r[:, :, 4:4 + klen] = keys_for(g).reshape(nblk, recs, KEY_LEN)[:, :, :klen]
    r[:, :, 4 + klen:8 + klen] = np.frombuffer(np.uint32(vlen).tobytes(), dtype=np.uint8)
    if vlen:
        r[:, :, 8 + klen:] = value_bytes(g, vlen, seed).reshape(nblk, recs, vlen)
    blk_off = (np.arange(nblk, dtype=np.uint64) * np.uint64(slot))
    blk_len = np.full(nblk, used, dtype=np.uint32)
    return buf.reshape(-1), blk_off, blk_len


def kv_stream(n: int, first: int = 0, klen: int = KEY_LEN, vlen: int = VAL_LEN,
              seed: int = SEED):
    """Columnar sorted record stream (config 3): keys, koff, vals, voff."""
    g = np.arange(first, first + n, dtype=np.int64)
    keys = keys_for(g)[:, :klen].reshape(-1).copy()
    vals = value_bytes(g, vlen, seed).reshape(-1).copy()
    koff = np.arange(n + 1, dtype=np.uint64) * np.uint64(klen)
    voff = np.arange(n + 1, dtype=np.uint64) * np.uint64(vlen)
    return keys, koff, vals, voff


def mixed_kv_blocks(total_bytes: int, seed: int = SEED, sizes=(4096, 16384, 65536),
                    vmin: int = 8, vmax: int = 4096):
    """Config 5: block sizes uniform over {4,16,64} KiB, value sizes
    log-uniform on [8, 4096] (capped at blk_size-24), 16-byte keys, records
    packed greedily until the next one does not fit.  Blocks sit in slots of
    their own size; blk_len counts the packed bytes.

    Returns (buf, blk_off, blk_len, nrec)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    # draw blocks until the slot bytes reach total_bytes
    nblk_est = max(1, int(total_bytes / (sum(sizes) / len(sizes))) + 1)
    bsz = rng.choice(np.asarray(sizes, dtype=np.int64), size=nblk_est)
    bsz = bsz[: max(1, int(np.searchsorted(np.cumsum(bsz), total_bytes)) + 1)]
    nblk = bsz.size
    buf = np.zeros(int(bsz.sum()), dtype=np.uint8)
    blk_off = np.zeros(nblk, dtype=np.uint64)
    blk_off[1:] = np.cumsum(bsz)[:-1].astype(np.uint64)
    blk_len = np.zeros(nblk, dtype=np.uint32)
    nrec = np.zeros(nblk, dtype=np.int64)
    g = 0
    lo, hi = np.log(vmin), np.log(vmax)
    pool = np.exp(rng.uniform(lo, hi, size=1 << 20)).astype(np.int64)
    pp = 0
    for b in range(nblk):
        cap = int(bsz[b])
        need = cap // (8 + KEY_LEN + vmin) + 2
        if pp + need > pool.size:
            pool = np.exp(rng.uniform(lo, hi, size=1 << 20)).astype(np.int64)
            pp = 0
        v = np.minimum(pool[pp:pp + need], cap - 24)
        rsz = 8 + KEY_LEN + v
        c = np.cumsum(rsz)
        cnt = int(np.searchsorted(c, cap, side="right"))
        pp += cnt + 1
        v = v[:cnt]
        rsz = rsz[:cnt]
        starts = np.concatenate([[0], np.cumsum(rsz)[:-1]]).astype(np.int64)
        gi = np.arange(g, g + cnt, dtype=np.int64)
        keys = keys_for(gi)
        base = int(blk_off[b])
        blk = buf[base:base + cap]
        for j in range(cnt):
            s = int(starts[j])
            vl = int(v[j])
            blk[s:s + 4] = np.frombuffer(np.uint32(KEY_LEN).tobytes(), dtype=np.uint8)
            blk[s + 4:s + 20] = keys[j]
            blk[s + 20:s + 24] = np.frombuffer(np.uint32(vl).tobytes(), dtype=np.uint8)
            blk[s + 24:s + 24 + vl] = value_bytes(np.array([g + j]), vl, seed)[0]
        blk_len[b] = int(rsz.sum())
        nrec[b] = cnt
        g += cnt
    return buf, blk_off, blk_len, nrec


TOMBSTONE = "～DELETED～".encode()  # kv.DeletedValue, kv/kv.go:30 (13 bytes)


def wal_logs(nwal: int, seed: int = SEED, memtable_bytes: int = 2 * 1024 * 1024,
             delete_every: int = 16):
    """Write-ahead logs shaped by go-lsm's own benchmark (benchmark.go:30-43):
    Put keys "k_<i>_<1-10 random letters>", values "v_<i>_<2-20 random
    letters>", every delete_every-th record a Delete (the tombstone value,
    memtable Delete -> WAL.Append).  Each log holds the records of one
    memtable: appended until the EstimateSize sum (kv.go:118-121) reaches
    memtable_bytes (memtable.go:119-121).  A log is KeyValuePair.EncodeTo of
    each record (kv.go:46-74).

    Returns (buf uint8, wal_off uint64[nwal], wal_len uint32[nwal], nrec[nwal])."""
    rng = np.random.Generator(np.random.PCG64(seed))
    letters = np.frombuffer(b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ", np.uint8)
    logs, nrec = [], []
    g = 0
    for _ in range(nwal):
        parts, est, cnt = [], 0, 0
        while est < memtable_bytes:
            k = b"k_%d_" % g + letters[rng.integers(0, 52, int(rng.integers(1, 11)))].tobytes()
            if delete_every and g % delete_every == delete_every - 1:
                v = TOMBSTONE
            else:
                v = b"v_%d_" % g + letters[rng.integers(0, 52, int(rng.integers(2, 21)))].tobytes()
            parts.append(np.uint32(len(k)).tobytes() + k + np.uint32(len(v)).tobytes() + v)
            est += 4 + len(k) + 4 + len(v) + 8
            cnt += 1
            g += 1
        logs.append(b"".join(parts))
        nrec.append(cnt)
    # 16-byte aligned starts, as files read into one device buffer
    off, pos = [], 0
    for lg in logs:
        off.append(pos)
        pos += (len(lg) + 15) // 16 * 16
    buf = np.zeros(pos, dtype=np.uint8)
    for o, lg in zip(off, logs):
        buf[o:o + len(lg)] = np.frombuffer(lg, np.uint8)
    return (buf, np.array(off, dtype=np.uint64), np.array([len(x) for x in logs], dtype=np.uint32),
            np.array(nrec, dtype=np.int64))
