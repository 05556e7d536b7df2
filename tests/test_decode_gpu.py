"""GPU parity: lsm_decode_blocks vs the CPU restatement (bit-exact).

Translates sstable/block/data_test.go, index_test.go and kv/kv_test.go cases
into device batches, fuzzes every grammar with corruptions, odd alignments
and large blocks, and checks BASELINE config 2 / 5 at full size through
size-independent properties plus a sampled oracle comparison.
"""
import json
import os
import struct

import numpy as np
import pytest
import torch

import lsmgpu
import pyoracle as ora
from lsmgpu import synth

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
REF = json.load(open(os.path.join(HERE, "golden", "reference_vectors.json")))


def dev_batch(ctx, blocks, align_pad=None, rng=None):
    """Pack byte blocks into one buffer (optionally at odd offsets)."""
    parts, offs, lens = [], [], []
    pos = 0
    for i, b in enumerate(blocks):
        b = np.frombuffer(bytes(b), np.uint8) if not isinstance(b, np.ndarray) else b
        gap = 0
        if align_pad is not None:
            gap = int(rng.integers(0, align_pad)) if rng is not None else align_pad
        parts.append(np.zeros(gap, np.uint8))
        pos += gap
        offs.append(pos)
        lens.append(b.size)
        parts.append(b)
        pos += b.size
    buf = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
    dev = ctx.torch_device
    return (buf, lsmgpu.to_device_bytes(buf, dev),
            torch.tensor(np.array(offs, np.uint64).view(np.int64), device=dev),
            torch.tensor(np.array(lens, np.uint32).view(np.int32), device=dev))


def check_against_oracle(grammar, buf, blk_off, blk_len, r, arena=False, arena_fill=0):
    nrec = r.nrec.cpu().numpy()
    status = r.status.cpu().numpy()
    rec_base = r.bases(blk_off).astype(np.int64)
    desc = r.desc_numpy()
    iv = r.idx_value.cpu().numpy() if r.idx_value is not None else None
    if arena:
        ka = r.key_arena.cpu().numpy() if r.key_arena is not None else None
        va = r.val_arena.cpu().numpy() if r.val_arena is not None else None
        ab = r.arena_bases(blk_off).astype(np.int64)
        # every arena byte outside the blocks' packed ranges keeps its initial
        # value (arena_fill): no emitter writes past a run or a batch
        ek = np.full_like(ka, arena_fill) if ka is not None else None
        ev = np.full_like(va, arena_fill) if va is not None else None
    for b, (o, l) in enumerate(zip(blk_off, blk_len)):
        st, d, oiv = ora.decode_block(grammar, buf, int(o), int(l))
        assert status[b] == st, (b, status[b], st)
        assert nrec[b] == len(d), (b, nrec[b], len(d))
        got = desc[rec_base[b]:rec_base[b] + nrec[b]]
        assert np.array_equal(got, d), b
        if grammar == lsmgpu.GRAMMAR_IDX:
            assert np.array_equal(iv[rec_base[b]:rec_base[b] + nrec[b]], oiv), b
        if arena:
            ok, ov = ora.materialize(grammar, buf, d)
            if ka is not None:
                assert ka[ab[b]:ab[b] + ok.size].tobytes() == ok.tobytes(), b
            if va is not None:
                assert va[ab[b]:ab[b] + ov.size].tobytes() == ov.tobytes(), b
                ev[ab[b]:ab[b] + ov.size] = ov
            if ka is not None:
                ek[ab[b]:ab[b] + ok.size] = ok
    if arena:
        for got, exp in ((ka, ek), (va, ev)):
            if got is not None:
                bad = np.nonzero(got != exp)[0]
                assert bad.size == 0, ("arena bytes written outside the packed ranges", bad[:8])


def check_compaction(ctx, grammar, blk_off_host, d_off, r):
    """lsm_compact_records: the same records, dense, in block order."""
    nrec = r.nrec.cpu().numpy().astype(np.int64)[: d_off.numel()]
    d = lsmgpu.alloc_dense(ctx, grammar, int(d_off.numel()), int(nrec.sum()))
    lsmgpu.compact_into(ctx, grammar, d_off, r, d)
    torch.cuda.synchronize()
    base = d.base.cpu().numpy()
    assert np.array_equal(base, np.concatenate([[0], np.cumsum(nrec)]))
    dense = d.desc.cpu().numpy().view(np.uint8).view(lsmgpu.DESC_DTYPE).reshape(-1)
    sparse = r.desc_numpy()
    rb = r.bases(blk_off_host).astype(np.int64)
    for b in range(len(nrec)):
        assert np.array_equal(dense[base[b]:base[b + 1]], sparse[rb[b]:rb[b] + nrec[b]]), b
    if d.idx_value is not None:
        iv, div = r.idx_value.cpu().numpy(), d.idx_value.cpu().numpy()
        for b in range(len(nrec)):
            assert np.array_equal(div[base[b]:base[b + 1]], iv[rb[b]:rb[b] + nrec[b]]), b


def run(ctx, grammar, blocks, arena=False, align_pad=None, seed=0, placement="plan",
        compact=False):
    rng = np.random.default_rng(seed)
    buf, d_in, d_off, d_len = dev_batch(ctx, blocks, align_pad=align_pad, rng=rng)
    r = lsmgpu.decode_blocks(ctx, grammar, d_in, d_off, d_len, arena=arena, arena_offsets=arena,
                             placement=placement)
    torch.cuda.synchronize()
    blk_off = d_off.cpu().numpy().view(np.uint64)
    check_against_oracle(grammar, buf, blk_off, d_len.cpu().numpy().view(np.uint32), r,
                         arena=arena)
    if compact:
        check_compaction(ctx, grammar, blk_off, d_off, r)
    return r


def v_block(values):
    return b"".join(struct.pack("<I", len(v)) + v for v in values)


def kv_block(pairs):
    return b"".join(struct.pack("<I", len(k)) + k + struct.pack("<I", len(v)) + v for k, v in pairs)


def idx_block(entries):
    return b"".join(struct.pack("<I", len(k)) + k + struct.pack("<q", o) for k, o in entries)


# ---- reference test vectors as device batches ---------------------------------

def test_data_test_vectors(ctx):
    blocks = []
    for case in REF["data_block_roundtrip"]:
        b = v_block([e.encode() for e in case["entries"]])
        n = len(b) if case["size"] <= 0 else min(case["size"], len(b))
        blocks.append(b[:n])
    sl = REF["data_block_size_limit"]
    full = v_block([e.encode() for e in sl["entries"]])
    blocks.append(full[:sl["insufficient"]["size"]])
    blocks.append(full[:sl["partial"]["size"]])
    for case in REF["data_block_corrupt"]:
        blocks.append(bytes.fromhex(case["bytes"]))
    r = run(ctx, lsmgpu.GRAMMAR_V, blocks)
    st = r.status.cpu().numpy()
    assert list(st[:5]) == [0] * 5 and st[5] != 0 and st[6] == 0 and st[7] != 0 and st[8] != 0
    assert list(r.nrec.cpu().numpy()[:7]) == [0, 1, 3, 2, 2, 0, 2]


def test_kv_test_vectors(ctx):
    pairs = [(bytes.fromhex(c["key"]), bytes.fromhex(c["value"])) for c in REF["kv_pairs"]]
    blocks = [kv_block([p]) for p in pairs] + [kv_block(pairs)]
    r = run(ctx, lsmgpu.GRAMMAR_KV, blocks, arena=True)
    assert list(r.nrec.cpu().numpy()) == [1] * len(pairs) + [len(pairs)]


def test_index_test_vectors(ctx):
    ib = REF["index_block"]
    ent = [(k.encode(), o) for k, o in ib["entries"]]
    full = idx_block(ent)
    two = idx_block(ent[:2])
    f = ib["partial_size_first_entry"]
    blocks = [full, two[:f], two[: f - ib["truncate_by"]], b""]
    for case in REF["index_entry_encode"]:
        blocks.append(bytes.fromhex(case["bytes"]))
    r = run(ctx, lsmgpu.GRAMMAR_IDX, blocks)
    assert list(r.nrec.cpu().numpy()) == [3, 1, 0, 0, 1, 1]
    assert list(r.idx_value.cpu().numpy()[r.rec_base.cpu().numpy()[0]:][:3]) == [100, 200, 300]


def test_index_block_cut_inside_last_entry(ctx):
    """An IDX block whose size ends inside its last entry: inside the key
    length, the key, or the i64 offset, with the entry's remaining bytes
    present past the block (the .sst's reader) or not (the block ends the
    buffer).  Go appends the entries before it and fails on that entry
    (index.go:61-101, one of three messages by what the reader holds past the
    block: include/lsm_gpu.h); the library and the oracle both report
    LSM_ST_IDX_OVERRUN with the same records."""
    ent = [(b"alpha", 100), (b"bravo-key", -7), (b"charlie-longer-key", 2**40)]
    full = idx_block(ent)
    last = len(idx_block(ent[:2]))
    klen_cut = [last + 1, last + 2, last + 3]                 # inside the key length
    key_cut = [last + 4, last + 4 + 7, last + 4 + 17]         # inside the key
    off_cut = [last + 4 + 18 + j for j in (0, 1, 4, 7)]       # inside the offset
    blocks = [full[:c] for c in klen_cut + key_cut + off_cut]
    # the same cuts with the rest of the entry present past the block
    buf = np.frombuffer(full, np.uint8)
    dev = ctx.torch_device
    cuts = klen_cut + key_cut + off_cut
    d_in = lsmgpu.to_device_bytes(buf, dev)
    d_off = torch.zeros(len(cuts), dtype=torch.int64, device=dev)
    d_len = torch.tensor(np.array(cuts, np.uint32).view(np.int32), device=dev)
    r = lsmgpu.decode_blocks(ctx, lsmgpu.GRAMMAR_IDX, d_in, d_off, d_len)
    torch.cuda.synchronize()
    check_against_oracle(lsmgpu.GRAMMAR_IDX, buf, np.zeros(len(cuts), np.uint64),
                         np.array(cuts, np.uint32), r)
    assert (r.status.cpu().numpy() == 7).all() and (r.nrec.cpu().numpy() == 2).all()
    r2 = run(ctx, lsmgpu.GRAMMAR_IDX, blocks)
    assert (r2.status.cpu().numpy() == 7).all() and (r2.nrec.cpu().numpy() == 2).all()


# ---- fuzz ---------------------------------------------------------------------------

def rand_records(rng, grammar, n, kmax=40, vmax=300):
    out = []
    for _ in range(n):
        k = rng.integers(0, 256, int(rng.integers(0, kmax + 1)), dtype=np.uint8).tobytes()
        v = rng.integers(0, 256, int(rng.integers(0, vmax + 1)), dtype=np.uint8).tobytes()
        if grammar == 0:
            out.append(struct.pack("<I", len(v)) + v)
        elif grammar == 1:
            out.append(struct.pack("<I", len(k)) + k + struct.pack("<I", len(v)) + v)
        else:
            out.append(struct.pack("<I", len(k)) + k + struct.pack("<q", int(rng.integers(-2**62, 2**62))))
    return b"".join(out)


def corrupt(rng, b):
    kind = int(rng.integers(0, 6))
    if kind == 0 or len(b) == 0:
        return b
    if kind == 1:  # truncate anywhere
        return b[: int(rng.integers(0, len(b)))]
    if kind == 2:  # trailing 1-3 bytes
        return b + bytes(int(rng.integers(1, 4)))
    if kind == 3:  # giant length somewhere at a record start (first 4 bytes)
        return struct.pack("<I", int(rng.choice([2**20 + 1, 2**30 + 1, 2**32 - 1, 999999]))) + b[4:]
    if kind == 4:  # random bytes
        return rng.integers(0, 256, len(b), dtype=np.uint8).tobytes()
    return b[: len(b) // 2] + bytes(3)


@pytest.mark.parametrize("grammar", [0, 1, 2])
@pytest.mark.parametrize("arena", [False, True])
@pytest.mark.parametrize("placement", ["plan", "offset"])
def test_fuzz_small_blocks(ctx, grammar, arena, placement):
    rng = np.random.default_rng(100 + grammar * 2 + arena)
    blocks = []
    for i in range(300):
        b = rand_records(rng, grammar, int(rng.integers(0, 40)), kmax=24, vmax=120)
        blocks.append(corrupt(rng, b))
    run(ctx, grammar, blocks, arena=arena, align_pad=19, seed=grammar, placement=placement,
        compact=not arena)


@pytest.mark.parametrize("grammar", [0, 1, 2])
def test_large_and_many_record_blocks(ctx, grammar):
    rng = np.random.default_rng(7 + grammar)
    blocks = [
        rand_records(rng, grammar, 1500, kmax=8, vmax=8),        # thousands of tiny records
        rand_records(rng, grammar, 40, kmax=64, vmax=4000),      # 64 KiB-ish, long values
        rand_records(rng, grammar, 300, kmax=40, vmax=1500),     # ~200 KiB
        rand_records(rng, grammar, 5, kmax=2000, vmax=20000),    # values larger than the ring
        b"",
    ]
    blocks.append(corrupt(rng, blocks[1]))
    # a mixed-shape block far larger than the 4 KiB ring, then a uniform one:
    # the DESC path streams both through counted-wait ring refills
    blocks.append(rand_records(rng, grammar, 400, kmax=30, vmax=700))
    blocks.append(rand_records(np.random.default_rng(0), grammar, 1, kmax=16, vmax=100) * 900)
    run(ctx, grammar, blocks, arena=True, align_pad=13, seed=3)
    run(ctx, grammar, blocks, arena=True, align_pad=13, seed=3, placement="offset")
    run(ctx, grammar, blocks, arena=False, align_pad=13, seed=3, compact=True)
    run(ctx, grammar, blocks, arena=False, align_pad=13, seed=4, placement="offset")


def test_capacity_status(ctx):
    # A caller-provided rec_base with too little room: LSM_ST_CAPACITY, nrec = cap.
    b = kv_block([(b"k%d" % i, b"v" * i) for i in range(10)])
    buf, d_in, d_off, d_len = dev_batch(ctx, [b, b])
    p = lsmgpu.plan(ctx, lsmgpu.GRAMMAR_KV, d_len)
    p.rec_base.copy_(torch.tensor([0, 4, 14], device=ctx.torch_device))
    r = lsmgpu.alloc_decode(ctx, lsmgpu.GRAMMAR_KV, 2, p)
    lsmgpu.decode_into(ctx, lsmgpu.GRAMMAR_KV, d_in, d_off, d_len, r)
    assert r.status.cpu().tolist() == [8, 0]
    assert r.nrec.cpu().tolist() == [4, 10]


def test_plan_matches_host(ctx):
    rng = np.random.default_rng(5)
    lens = rng.integers(0, 70000, 10000).astype(np.uint32)
    d_len = torch.tensor(lens.view(np.int32), device=ctx.torch_device)
    for g, div in ((0, 4), (1, 8), (2, 12)):
        p = lsmgpu.plan(ctx, g, d_len, arena=True)
        want = np.zeros(lens.size + 1, np.uint64)
        want[1:] = np.cumsum(lens // div)
        assert np.array_equal(p.rec_base.cpu().numpy().view(np.uint64), want)
        wa = np.zeros(lens.size + 1, np.uint64)
        wa[1:] = np.cumsum(lens.astype(np.uint64))
        assert np.array_equal(p.arena_base.cpu().numpy().view(np.uint64), wa)


# ---- BASELINE configs at full size ----------------------------------------------------

def test_config2_full_size(ctx):
    """100k x 4 KiB KV blocks (16 B keys / 100 B values): every descriptor is
    closed-form; a sample of blocks is compared with the oracle, and the
    materialized arenas checksum against the generator's columns."""
    nblk = 100_000
    buf, blk_off, blk_len = synth.uniform_kv_blocks(np.arange(nblk))
    dev = ctx.torch_device
    d_in = lsmgpu.to_device_bytes(buf, dev)
    d_off = torch.tensor(blk_off.view(np.int64), device=dev)
    d_len = torch.tensor(blk_len.view(np.int32), device=dev)
    r = lsmgpu.decode_blocks(ctx, lsmgpu.GRAMMAR_KV, d_in, d_off, d_len, arena=True)
    torch.cuda.synchronize()
    assert int((r.status != 0).sum()) == 0
    assert bool((r.nrec == 33).all())
    rb = r.rec_base.cpu().numpy()
    assert np.array_equal(rb, np.arange(nblk + 1) * 511)
    desc = r.desc.view(-1, 4)
    idx = (torch.arange(nblk, device=dev)[:, None] * 511 + torch.arange(33, device=dev)[None, :]).reshape(-1)
    d = desc[idx].cpu().numpy().view(np.uint8).view(lsmgpu.DESC_DTYPE).reshape(-1)
    want_off = (np.arange(nblk)[:, None] * 4096 + np.arange(33)[None, :] * 124).reshape(-1)
    assert np.array_equal(d["rec_off"], want_off.astype(np.uint64))
    assert (d["key_len"] == 16).all() and (d["val_len"] == 100).all()
    # arenas: block b's keys are packed at arena_base[b] = 4092*b
    ka = r.key_arena[: nblk * 4092].view(nblk, 4092)[:, : 33 * 16].cpu().numpy()
    va = r.val_arena[: nblk * 4092].view(nblk, 4092)[:, : 33 * 100].cpu().numpy()
    keys, _, vals, _ = synth.kv_stream(nblk * 33)
    assert np.array_equal(ka.reshape(-1), keys)
    assert np.array_equal(va.reshape(-1), vals)
    # oracle on a sample of blocks
    sample = np.random.default_rng(0).choice(nblk, 64, replace=False)
    for b in sample:
        st, od, _ = ora.decode_block(1, buf, int(blk_off[b]), int(blk_len[b]))
        assert st == 0 and np.array_equal(d[b * 33:(b + 1) * 33], od)


def test_bench_path_config2_full_size(ctx):
    """Exactly what bench.py times (alloc_decode_offset + decode_into, DESC,
    offset placement: decode_v2_kernel<KV,8>) on the full 100k config-2 batch:
    every descriptor in closed form, 256 sampled blocks against the oracle
    (kv/kv.go:77-115), and repeated launches into the same outputs."""
    nblk = 100_000
    buf, blk_off, blk_len = synth.uniform_kv_blocks(np.arange(nblk))
    dev = ctx.torch_device
    d_in = lsmgpu.to_device_bytes(buf, dev)
    d_off = torch.tensor(blk_off.view(np.int64), device=dev)
    d_len = torch.tensor(blk_len.view(np.int32), device=dev)
    r = lsmgpu.alloc_decode_offset(ctx, lsmgpu.GRAMMAR_KV, nblk, int(d_in.numel()))
    r.desc.fill_(-1)
    for _ in range(3):
        lsmgpu.decode_into(ctx, lsmgpu.GRAMMAR_KV, d_in, d_off, d_len, r)
    torch.cuda.synchronize()
    assert int((r.status[:nblk] != 0).sum()) == 0
    assert bool((r.nrec[:nblk] == 33).all())
    # offset placement: block b's records at slots blk_off[b] / 8 = 512 b
    idx = (torch.arange(nblk, device=dev)[:, None] * 512
           + torch.arange(33, device=dev)[None, :]).reshape(-1)
    d = r.desc[idx].cpu().numpy().view(np.uint8).view(lsmgpu.DESC_DTYPE).reshape(-1)
    want_off = (np.arange(nblk)[:, None] * 4096 + np.arange(33)[None, :] * 124).reshape(-1)
    assert np.array_equal(d["rec_off"], want_off.astype(np.uint64))
    assert (d["key_len"] == 16).all() and (d["val_len"] == 100).all()
    sample = np.random.default_rng(2).choice(nblk, 256, replace=False)
    for b in sample:
        st, od, _ = ora.decode_block(1, buf, int(blk_off[b]), int(blk_len[b]))
        assert st == 0 and np.array_equal(d[b * 33:(b + 1) * 33], od), b
    # the bench's own post-run check accepts it and rejects a single bad record
    import bench
    import argparse
    bench.lsmgpu = lsmgpu
    args = argparse.Namespace(config="decode4k")
    bench.verify_decode(args, r, d_off, d_len, nblk)
    r.desc[512 * 777 + 5, 3] = 101
    with pytest.raises(AssertionError):
        bench.verify_decode(args, r, d_off, d_len, nblk)


def test_large_launch_closed_form(ctx):
    """A launch above kBigLaunch blocks (450k x 4 KiB config-2 blocks, 1.8 GB)
    takes the large-launch instantiation (blocks loaded with the default
    cache policy): every descriptor in closed form on the device, 64 sampled
    blocks against the oracle."""
    nblk = 450_000
    buf, blk_off, blk_len = synth.uniform_kv_blocks(np.arange(nblk))
    dev = ctx.torch_device
    d_in = lsmgpu.to_device_bytes(buf, dev)
    d_off = torch.tensor(blk_off.view(np.int64), device=dev)
    d_len = torch.tensor(blk_len.view(np.int32), device=dev)
    r = lsmgpu.alloc_decode_offset(ctx, lsmgpu.GRAMMAR_KV, nblk, int(d_in.numel()))
    r.desc.fill_(-1)
    lsmgpu.decode_into(ctx, lsmgpu.GRAMMAR_KV, d_in, d_off, d_len, r)
    torch.cuda.synchronize()
    assert int((r.status[:nblk] != 0).sum()) == 0
    assert bool((r.nrec[:nblk] == 33).all())
    idx = (torch.arange(nblk, device=dev)[:, None] * 512
           + torch.arange(33, device=dev)[None, :]).reshape(-1)
    d = r.desc[idx].view(torch.int32).reshape(-1, 4).to(torch.int64)
    want = (torch.arange(nblk, device=dev)[:, None] * 4096
            + torch.arange(33, device=dev)[None, :] * 124).reshape(-1)
    got = d[:, 0] + (d[:, 1] << 32)
    assert torch.equal(got, want)
    assert bool((d[:, 2] == 16).all()) and bool((d[:, 3] == 100).all())
    sample = np.random.default_rng(3).choice(nblk, 64, replace=False)
    for b in sample:
        st, od, _ = ora.decode_block(1, buf, int(blk_off[b]), int(blk_len[b]))
        rows = r.desc[b * 512: b * 512 + 33].cpu().numpy().view(np.uint8).view(lsmgpu.DESC_DTYPE).reshape(-1)
        assert st == 0 and np.array_equal(rows, od), b


def test_config5_mixed_sample(ctx):
    buf, blk_off, blk_len, nrec = synth.mixed_kv_blocks(24 << 20, seed=11)
    dev = ctx.torch_device
    d_in = lsmgpu.to_device_bytes(buf, dev)
    d_off = torch.tensor(blk_off.view(np.int64), device=dev)
    d_len = torch.tensor(blk_len.view(np.int32), device=dev)
    r = lsmgpu.decode_blocks(ctx, lsmgpu.GRAMMAR_KV, d_in, d_off, d_len, arena=True)
    torch.cuda.synchronize()
    assert int((r.status != 0).sum()) == 0
    assert np.array_equal(r.nrec.cpu().numpy(), nrec)
    check_against_oracle(lsmgpu.GRAMMAR_KV, buf, blk_off, blk_len, r, arena=True)
    # DESC output, offset placement
    r = lsmgpu.decode_blocks(ctx, lsmgpu.GRAMMAR_KV, d_in, d_off, d_len, placement="offset")
    torch.cuda.synchronize()
    assert int((r.status != 0).sum()) == 0
    check_against_oracle(lsmgpu.GRAMMAR_KV, buf, blk_off, blk_len, r)
    # the bench's path: lsm_decode_blocks_scheduled (largest first), twice
    # into the same outputs, then the bench's own post-run check
    rs = lsmgpu.alloc_decode_offset(ctx, lsmgpu.GRAMMAR_KV, blk_off.size, int(d_in.numel()))
    ws = lsmgpu.schedule_workspace(ctx, blk_off.size)
    for _ in range(2):
        lsmgpu.decode_into(ctx, lsmgpu.GRAMMAR_KV, d_in, d_off, d_len, rs, schedule=ws)
    torch.cuda.synchronize()
    check_against_oracle(lsmgpu.GRAMMAR_KV, buf, blk_off, blk_len, rs)
    import argparse
    import bench
    bench.lsmgpu = lsmgpu
    args = argparse.Namespace(config="mixed", arena=False, _d_in=d_in)
    bench.verify_decode(args, rs, d_off, d_len, blk_off.size)


@pytest.mark.parametrize("grammar", [0, 1, 2])
@pytest.mark.parametrize("arena", [False, True])
def test_scheduled_matches_unscheduled(ctx, grammar, arena):
    """lsm_decode_blocks_scheduled launches blocks largest first; every
    output (status, counts, descriptors, arenas) equals lsm_decode_blocks' on
    fuzzed blocks of 0 B to ~200 KiB, corrupted ones included."""
    rng = np.random.default_rng(40 + grammar)
    blocks = []
    for i in range(700):
        n = int(rng.choice([0, 1, 3, 20, 60, 300]))
        b = rand_records(rng, grammar, n, kmax=24, vmax=int(rng.choice([8, 120, 700])))
        blocks.append(corrupt(rng, b) if i % 3 == 0 else b)
    buf, d_in, d_off, d_len = dev_batch(ctx, blocks)
    outs = []
    for sched in (None, lsmgpu.schedule_workspace(ctx, len(blocks))):
        r = lsmgpu.alloc_decode_offset(ctx, grammar, len(blocks), int(d_in.numel()), arena=arena)
        for t in (r.desc, r.idx_value, r.key_arena, r.val_arena):
            if t is not None:
                t.fill_(-1)  # slots no block writes compare equal
        lsmgpu.decode_into(ctx, grammar, d_in, d_off, d_len, r, schedule=sched)
        torch.cuda.synchronize()
        outs.append(r)
    a, b = outs
    assert torch.equal(a.status, b.status) and torch.equal(a.nrec, b.nrec)
    assert torch.equal(a.desc, b.desc)
    if grammar == 2:
        assert torch.equal(a.idx_value, b.idx_value)
    if arena:
        for x, y in ((a.key_arena, b.key_arena), (a.val_arena, b.val_arena)):
            if x is not None:
                assert torch.equal(x, y)
    check_against_oracle(grammar, buf, d_off.cpu().numpy().view(np.uint64),
                         d_len.cpu().numpy().view(np.uint32), b, arena=arena, arena_fill=0xFF)


def test_decode64k_full_size(ctx):
    """6,400 x 64 KiB uniform KV blocks (the bench's decode64k): closed-form
    descriptors, every block's records streamed through the ring."""
    nblk, recs = 6400, 528
    buf, blk_off, blk_len = synth.uniform_kv_blocks(np.arange(nblk), recs=recs, slot=65536)
    dev = ctx.torch_device
    d_in = lsmgpu.to_device_bytes(buf, dev)
    d_off = torch.tensor(blk_off.view(np.int64), device=dev)
    d_len = torch.tensor(blk_len.view(np.int32), device=dev)
    r = lsmgpu.decode_blocks(ctx, lsmgpu.GRAMMAR_KV, d_in, d_off, d_len, placement="offset")
    torch.cuda.synchronize()
    assert int((r.status != 0).sum()) == 0 and bool((r.nrec == recs).all())
    per = 65536 // 8
    idx = (torch.arange(nblk, device=dev)[:, None] * per + torch.arange(recs, device=dev)[None, :]).reshape(-1)
    d = r.desc.view(-1, 4)[idx].cpu().numpy().view(np.uint8).view(lsmgpu.DESC_DTYPE).reshape(-1)
    want = (np.arange(nblk)[:, None] * 65536 + np.arange(recs)[None, :] * 124).reshape(-1)
    assert np.array_equal(d["rec_off"], want.astype(np.uint64))
    assert (d["key_len"] == 16).all() and (d["val_len"] == 100).all()
    # the bench's path: lsm_decode_blocks_hinted with the 64 KiB bound (16 KiB
    # ring), identical outputs, and the bench's own post-run check
    rh = lsmgpu.alloc_decode_offset(ctx, lsmgpu.GRAMMAR_KV, nblk, int(d_in.numel()))
    lsmgpu.decode_into(ctx, lsmgpu.GRAMMAR_KV, d_in, d_off, d_len, rh, max_blk_len=65536)
    torch.cuda.synchronize()
    assert torch.equal(rh.desc.view(-1, 4)[idx], r.desc.view(-1, 4)[idx])
    assert torch.equal(rh.nrec[:nblk], r.nrec[:nblk]) and torch.equal(rh.status[:nblk], r.status[:nblk])
    import argparse
    import bench
    bench.lsmgpu = lsmgpu
    bench.verify_decode(argparse.Namespace(config="decode64k", arena=False, _d_in=d_in), rh, d_off,
                        d_len, nblk)


@pytest.mark.parametrize("grammar", [0, 1, 2])
@pytest.mark.parametrize("arena", [False, True])
def test_hinted_matches_plain(ctx, grammar, arena):
    """lsm_decode_blocks_hinted only picks the ring: with a large-block hint
    (16 KiB ring) every output equals lsm_decode_blocks', also for blocks
    longer than the hint and for corrupted ones."""
    rng = np.random.default_rng(70 + grammar)
    blocks = []
    for i in range(300):
        n = int(rng.choice([0, 2, 40, 300, 900]))
        b = rand_records(rng, grammar, n, kmax=40, vmax=int(rng.choice([8, 200, 2000])))
        blocks.append(corrupt(rng, b) if i % 4 == 0 else b)
    blocks += [rand_records(rng, grammar, 1500, kmax=200, vmax=2000) for _ in range(3)]
    buf, d_in, d_off, d_len = dev_batch(ctx, blocks, align_pad=7, rng=rng)
    outs = []
    for hint in (None, 40000):
        r = lsmgpu.alloc_decode_offset(ctx, grammar, len(blocks), int(d_in.numel()), arena=arena)
        for t in (r.desc, r.idx_value, r.key_arena, r.val_arena):
            if t is not None:
                t.fill_(-1)
        lsmgpu.decode_into(ctx, grammar, d_in, d_off, d_len, r, max_blk_len=hint)
        torch.cuda.synchronize()
        outs.append(r)
    a, b = outs
    assert int(d_len.max()) > 40000  # some blocks exceed the hint
    assert torch.equal(a.status, b.status) and torch.equal(a.nrec, b.nrec)
    assert torch.equal(a.desc, b.desc)
    for x, y in ((a.idx_value, b.idx_value), (a.key_arena, b.key_arena), (a.val_arena, b.val_arena)):
        if x is not None:
            assert torch.equal(x, y)
    check_against_oracle(grammar, buf, d_off.cpu().numpy().view(np.uint64),
                         d_len.cpu().numpy().view(np.uint32), b, arena=arena, arena_fill=0xFF)


@pytest.mark.parametrize("grammar", [0, 1, 2])
def test_arena_uniform_runs(ctx, grammar):
    """ARENA through the speculative-run emitter: blocks of equal-shape records
    (key / value lengths 0-17 and 100, so runs, the exact step's record merged
    into the run, fields shorter than a dword, 16-byte chunks straddling
    records) at odd alignments, in blocks that fit the 8 KiB ring and in
    streamed ones, plus a shape change mid-block (kv.go:88-111 materialized)."""
    rng = np.random.default_rng(31 + grammar)
    blocks = []
    for k, v in [(0, 0), (0, 1), (1, 0), (3, 5), (16, 100), (17, 3), (2, 17), (5, 1)]:
        # a fixed shape: key length k, value length v
        kb, vb = bytes(range(7, 7 + k)), bytes((i * 37) & 255 for i in range(v))
        if grammar == 0:
            rec = struct.pack("<I", v) + vb
        elif grammar == 1:
            rec = struct.pack("<I", k) + kb + struct.pack("<I", v) + vb
        else:
            rec = struct.pack("<I", k) + kb + struct.pack("<q", v * 1000 - 7)
        for reps in (1, 2, 63, 64, 65, 130, 700):
            blocks.append(rec * reps)
        blocks.append(rec * 40 + rand_records(rng, grammar, 3, kmax=9, vmax=30) + rec * 90)
    run(ctx, grammar, blocks, arena=True, align_pad=11, seed=5)
    run(ctx, grammar, blocks, arena=True, align_pad=11, seed=6, placement="offset")


@pytest.mark.parametrize("grammar", [0, 1, 2])
def test_hinted_arena_linear_ring(ctx, grammar):
    """ARENA with a bound that fits the 8 KiB ring (lsm_decode_blocks_hinted's
    linear-ring kernel): outputs equal lsm_decode_blocks' and the oracle's --
    for a batch within the bound, and for one where some blocks break it (the
    marked blocks go through the streamed fallback launch), corrupted blocks,
    odd alignments and equal-shape runs included."""
    rng = np.random.default_rng(90 + grammar)
    blocks = []
    for i in range(400):
        n = int(rng.choice([0, 1, 3, 20, 60]))
        b = rand_records(rng, grammar, n, kmax=24, vmax=int(rng.choice([8, 40])))
        blocks.append(corrupt(rng, b) if i % 5 == 0 else b)
    kb, vb = bytes(range(7, 23)), bytes((i * 37) & 255 for i in range(100))
    rec = {0: struct.pack("<I", 100) + vb, 1: struct.pack("<I", 16) + kb + struct.pack("<I", 100) + vb,
           2: struct.pack("<I", 16) + kb + struct.pack("<q", 12345)}[grammar]
    blocks += [rec * r for r in (1, 33, 60)]
    fit = [b for b in blocks if len(b) <= 4000]
    big = fit + [rand_records(rng, grammar, 400, kmax=30, vmax=200) for _ in range(5)] + [rec * 200]
    for batch, hint in ((fit, 4000), (big, 4000)):
        buf, d_in, d_off, d_len = dev_batch(ctx, batch, align_pad=7, rng=rng)
        outs = []
        for h in (None, hint):
            r = lsmgpu.alloc_decode_offset(ctx, grammar, len(batch), int(d_in.numel()), arena=True)
            for t in (r.desc, r.idx_value, r.key_arena, r.val_arena):
                if t is not None:
                    t.fill_(-1)
            lsmgpu.decode_into(ctx, grammar, d_in, d_off, d_len, r, max_blk_len=h)
            torch.cuda.synchronize()
            outs.append(r)
        a, b = outs
        assert torch.equal(a.status, b.status) and torch.equal(a.nrec, b.nrec)
        assert torch.equal(a.desc, b.desc)
        for x, y in ((a.idx_value, b.idx_value), (a.key_arena, b.key_arena), (a.val_arena, b.val_arena)):
            if x is not None:
                assert torch.equal(x, y)
        check_against_oracle(grammar, buf, d_off.cpu().numpy().view(np.uint64),
                             d_len.cpu().numpy().view(np.uint32), b, arena=True, arena_fill=0xFF)
    assert max(len(x) for x in big) > 8192  # the fallback ran
