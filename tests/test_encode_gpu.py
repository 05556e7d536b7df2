"""GPU parity: lsm_encode_blocks / lsm_build_sst / bloom vs the CPU restatement.

Byte-exact comparisons of encoded blocks and whole .sst images (header,
bloom filter block, V data region, IDX index region, footer), the config 3
stream at full size, round trips through the decoder, and sum256/probe.
"""
import json
import os

import numpy as np
import pytest
import torch

import lsmgpu
import pyoracle as ora
from lsmgpu import synth

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
REF = json.load(open(os.path.join(HERE, "golden", "reference_vectors.json")))
ORV = np.load(os.path.join(HERE, "golden", "oracle_vectors.npz"))


def rand_batch(rng, n, kmax=40, vmax=300, kmin=0, vmin=0):
    kl = rng.integers(kmin, kmax + 1, n)
    vl = rng.integers(vmin, vmax + 1, n)
    keys = rng.integers(0, 256, int(kl.sum()), dtype=np.uint8)
    vals = rng.integers(0, 256, int(vl.sum()), dtype=np.uint8)
    koff = np.zeros(n + 1, np.uint64)
    voff = np.zeros(n + 1, np.uint64)
    koff[1:] = np.cumsum(kl)
    voff[1:] = np.cumsum(vl)
    return keys, koff, vals, voff


def csr(items):
    off = np.zeros(len(items) + 1, np.uint64)
    off[1:] = np.cumsum([len(x) for x in items])
    data = np.frombuffer(b"".join(items), np.uint8) if items else np.zeros(0, np.uint8)
    return data, off


@pytest.mark.parametrize("grammar", [0, 1, 2])
@pytest.mark.parametrize("seed", [0, 1])
def test_encode_blocks_random(ctx, grammar, seed):
    rng = np.random.default_rng(seed * 3 + grammar)
    n = 3000
    keys, koff, vals, voff = rand_batch(rng, n, kmax=50, vmax=400)
    batch = lsmgpu.batch_to_device(ctx, keys, koff, vals, voff)
    cuts = np.sort(rng.choice(np.arange(1, n), 60, replace=False))
    rec_start = np.concatenate([[0], cuts, [n]]).astype(np.uint64)
    nblk = rec_start.size - 1
    sizes = [lsmgpu.codec.encoded_size(grammar, koff, voff, int(rec_start[b]),
                                       int(rec_start[b + 1])) for b in range(nblk)]
    # odd output offsets with gaps to exercise unaligned edges
    gaps = rng.integers(0, 7, nblk)
    out_off = np.zeros(nblk, np.uint64)
    pos = 0
    for b in range(nblk):
        pos += int(gaps[b])
        out_off[b] = pos
        pos += sizes[b]
    idx_off = rng.integers(-2**40, 2**40, n) if grammar == 2 else None
    d_out, _ = lsmgpu.encode_blocks(ctx, grammar, batch, rec_start, out_off=out_off,
                                    out_bytes=pos, idx_off=idx_off)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    expect = np.zeros(pos, np.uint8)
    for b in range(nblk):
        r0, r1 = int(rec_start[b]), int(rec_start[b + 1])
        e = ora.encode_records(grammar, keys, koff, vals, voff, r0, r1,
                               idx_off=idx_off[r0:r1] if idx_off is not None else None)
        expect[int(out_off[b]):int(out_off[b]) + e.size] = e
    assert np.array_equal(out[:pos], expect)


def test_encode_decode_roundtrip_kv(ctx):
    rng = np.random.default_rng(9)
    keys, koff, vals, voff = rand_batch(rng, 5000, kmax=30, vmax=200)
    batch = lsmgpu.batch_to_device(ctx, keys, koff, vals, voff)
    rec_start = np.arange(0, 5001, 50, dtype=np.uint64)
    d_out, out_off = lsmgpu.encode_blocks(ctx, 1, batch, rec_start)
    nblk = rec_start.size - 1
    lens = np.array([lsmgpu.codec.encoded_size(1, koff, voff, int(rec_start[b]),
                                               int(rec_start[b + 1])) for b in range(nblk)],
                    np.uint32)
    dev = ctx.torch_device
    r = lsmgpu.decode_blocks(ctx, 1, d_out, torch.tensor(out_off.view(np.int64), device=dev),
                             torch.tensor(lens.view(np.int32), device=dev), arena=True,
                             placement="offset")
    torch.cuda.synchronize()
    assert (r.status.cpu().numpy() == 0).all() and (r.nrec.cpu().numpy() == 50).all()
    ka = r.key_arena.cpu().numpy()
    va = r.val_arena.cpu().numpy()
    for b in range(nblk):
        r0, r1 = int(rec_start[b]), int(rec_start[b + 1])
        kb = keys[int(koff[r0]):int(koff[r1])]
        vb = vals[int(voff[r0]):int(voff[r1])]
        o = int(out_off[b])
        assert np.array_equal(ka[o:o + kb.size], kb)
        assert np.array_equal(va[o:o + vb.size], vb)


def test_config2_reencode_matches_blocks(ctx):
    """Config 3's second check: re-encode the 100k config-2 blocks from their
    record stream into 4 KiB slots and byte-diff against the generator."""
    nblk = 100_000
    buf, blk_off, blk_len = synth.uniform_kv_blocks(np.arange(nblk))
    keys, koff, vals, voff = synth.kv_stream(nblk * 33)
    batch = lsmgpu.batch_to_device(ctx, keys, koff, vals, voff)
    rec_start = np.arange(nblk + 1, dtype=np.uint64) * 33
    d_out, _ = lsmgpu.encode_blocks(ctx, 1, batch, rec_start, out_off=blk_off,
                                    out_bytes=buf.size)
    torch.cuda.synchronize()
    assert torch.equal(d_out[: buf.size].cpu(), torch.from_numpy(buf))
    # and a sample against the oracle encoder
    for b in (0, 1, 4242, nblk - 1):
        e = ora.encode_records(1, keys, koff, vals, voff, b * 33, b * 33 + 33)
        assert np.array_equal(buf[b * 4096:b * 4096 + e.size], e)


# ---- .sst build ----------------------------------------------------------------------

def sst_vs_oracle(ctx, keys, koff, vals, voff, starts, m, k):
    batch = lsmgpu.batch_to_device(ctx, keys, koff, vals, voff)
    sb = lsmgpu.build_sst(ctx, batch, starts, m=m, k=k)
    torch.cuda.synchronize()
    out = sb.out.cpu().numpy()
    foot = sb.footer.cpu().numpy().reshape(-1, 4)
    for f in range(len(starts) - 1):
        want, wf = ora.build_sst(keys, koff, vals, voff, int(starts[f]), int(starts[f + 1]),
                                 m=m, k=k)
        o = int(sb.file_off[f])
        assert int(sb.file_size[f]) == want.size
        got = out[o:o + want.size]
        if not np.array_equal(got, want):
            bad = np.nonzero(got != want)[0]
            raise AssertionError(f"file {f}: {bad.size} bytes differ, first at {bad[0]} "
                                 f"of {want.size}")
        assert np.array_equal(foot[f], wf)
    return sb


def test_sst_reference_fixtures(ctx):
    c = REF["sst_sample"]
    kd, ko = csr([x.encode() for x in c["keys"]])
    vd, vo = csr([x.encode() for x in c["values"]])
    sb = sst_vs_oracle(ctx, kd, ko, vd, vo, np.array([0, 2], np.uint64), 1_600_000, 16)
    assert np.array_equal(sb.out.cpu().numpy()[: ORV["sst_sample"].size], ORV["sst_sample"])
    c = REF["sst_iterator"]
    kd, ko = csr([x.encode() for x in c["keys"]])
    vd, vo = csr([x.encode() for x in c["values"]])
    sb = sst_vs_oracle(ctx, kd, ko, vd, vo, np.array([0, 5], np.uint64), c["m"], c["k"])
    assert np.array_equal(sb.out.cpu().numpy()[: ORV["sst_iter"].size], ORV["sst_iter"])


@pytest.mark.parametrize("m,k", [(1, 1), (63, 3), (64, 0), (65, 5), (1000, 4), (819_200, 2),
                                 (819_201, 3), (1_000_003, 20), (1_600_000, 16), (1_638_400, 33),
                                 (1_638_401, 7)])
def test_sst_random_params(ctx, m, k):
    rng = np.random.default_rng(m + k)
    keys, koff, vals, voff = rand_batch(rng, 1200, kmax=24, vmax=180)
    starts = lsmgpu.segment_files(ctx, koff, voff, threshold=20000)
    assert len(starts) > 3
    sst_vs_oracle(ctx, keys, koff, vals, voff, starts, m, k)


def test_sst_edge_records(ctx):
    # empty keys, empty values, long keys, single-record files, an empty file
    items_k = [b"", b"a", b"x" * 300, b"", b"key"] * 40
    items_v = [b"", b"", b"v" * 5000, b"q", b""] * 40
    kd, ko = csr(items_k)
    vd, vo = csr(items_v)
    starts = np.array([0, 0, 1, 2, 7, 100, 200], np.uint64)
    sst_vs_oracle(ctx, kd, ko, vd, vo, starts, 1_600_000, 16)


@pytest.mark.parametrize("vlen", [0, 1, 3, 8, 11, 12, 13, 100, 1021])
def test_sst_uniform_value_sizes(ctx, vlen):
    """Values of one size (the region writer's reciprocal record lookup):
    sizes whose 16-byte output segments hold several value prefixes (< 12),
    exactly one, or none; files starting at the arena's first byte and at odd
    offsets."""
    n = 3000
    keys = np.frombuffer(b"".join(b"k%015d" % i for i in range(n)), np.uint8)
    koff = np.arange(n + 1, dtype=np.uint64) * 16
    rng = np.random.default_rng(vlen)
    vals = rng.integers(0, 256, max(n * vlen, 1), dtype=np.uint8)
    voff = np.arange(n + 1, dtype=np.uint64) * vlen
    starts = np.array([0, 1, 70, 777, 1500, 2999, n], np.uint64)
    sst_vs_oracle(ctx, keys, koff, vals, voff, starts, 1_600_000, 16)


def test_sst_config3_full(ctx):
    """Config 3: 3.3 M records (16 B / 100 B) -> builder rule -> 207 full
    .sst images of 2,297,320 B + 1 partial, every image byte-identical."""
    n = 100_000 * 33
    keys, koff, vals, voff = synth.kv_stream(n)
    starts = lsmgpu.segment_files(ctx, koff, voff, lsmgpu.MAX_SSTABLE_SIZE)
    assert np.array_equal(starts, ora.segment_files(koff, voff, lsmgpu.MAX_SSTABLE_SIZE))
    sizes = np.diff(starts.astype(np.int64))
    assert len(sizes) == 208 and (sizes[:-1] == 15888).all() and sizes[-1] == n - 207 * 15888
    batch = lsmgpu.batch_to_device(ctx, keys, koff, vals, voff)
    sb = lsmgpu.build_sst(ctx, batch, starts)
    torch.cuda.synchronize()
    assert (sb.file_size[:-1] == 2_297_320).all()
    out = sb.out.cpu().numpy()
    for f in range(len(starts) - 1):
        want, _ = ora.build_sst(keys, koff, vals, voff, int(starts[f]), int(starts[f + 1]))
        o = int(sb.file_off[f])
        assert np.array_equal(out[o:o + want.size], want), f
    # decode every image back on the GPU (lsm_decode_sst: IDX region + V
    # region, positional join) straight from the build's device buffer
    r = lsmgpu.decode_sst(ctx, sb.out, sb.file_off, sb.file_size)
    torch.cuda.synchronize()
    meta = r.meta_numpy()
    assert (meta["stage"] == 0).all() and (meta["status"] == 0).all()
    assert np.array_equal(meta["ndata"].astype(np.int64), sizes)
    assert np.array_equal(meta["nidx"].astype(np.int64), sizes)
    idesc = r.idx_desc.cpu().numpy().view(np.uint8).view(lsmgpu.DESC_DTYPE).reshape(-1)
    ival = r.idx_value.cpu().numpy()
    ddesc = r.data_desc.cpu().numpy().view(np.uint8).view(lsmgpu.DESC_DTYPE).reshape(-1)
    bases = r.bases()
    for f in (0, 3, 207):  # and against the oracle's decode of the same image
        o = int(sb.file_off[f])
        rc, om, oi, oiv, od = ora.sst_decode(out[o:o + int(sb.file_size[f])])
        assert rc == 0 and om.ndata == sizes[f]
        b = int(bases[f])
        gi = idesc[b:b + om.nidx].copy()
        gi["rec_off"] -= np.uint64(o)
        assert np.array_equal(gi, oi) and np.array_equal(ival[b:b + om.nidx], oiv), f
        gd = ddesc[b:b + om.ndata].copy()
        gd["rec_off"] -= np.uint64(o)
        assert np.array_equal(gd, od), f


# ---- hash / probe ----------------------------------------------------------------

def test_sum256_device(ctx):
    items = [bytes(range(n % 256)) * (1 + n // 256) for n in range(0, 300)]
    items = [x[:n] for n, x in zip(range(300), items)]
    rng = np.random.default_rng(1)
    items += [rng.integers(0, 256, int(rng.integers(0, 100)), dtype=np.uint8).tobytes()
              for _ in range(300)]
    kd, ko = csr(items)
    batch = lsmgpu.batch_to_device(ctx, kd, ko, np.zeros(0, np.uint8),
                                   np.zeros(len(items) + 1, np.uint64))
    h = lsmgpu.sum256(ctx, batch).cpu().numpy().view(np.uint64)
    for i, it in enumerate(items):
        assert tuple(int(x) for x in h[i]) == ora.sum256(np.frombuffer(it, np.uint8)), i


def test_bloom_probe_device(ctx):
    m, k = ora.estimate_parameters(1000, 0.001)
    f = ora.Bloom(m, k)
    import struct
    for i in range(1000):
        f.add(struct.pack(">I", i))
    probes = [struct.pack(">I", i) for i in range(3000)]
    kd, ko = csr(probes)
    batch = lsmgpu.batch_to_device(ctx, kd, ko, np.zeros(0, np.uint8),
                                   np.zeros(len(probes) + 1, np.uint64))
    words = torch.from_numpy(f.words.view(np.int64)).to(ctx.torch_device)
    hit = lsmgpu.bloom_probe(ctx, words, m, k, batch).cpu().numpy()
    want = np.array([f.test(p) for p in probes], np.uint8)
    assert np.array_equal(hit, want)
    assert hit[:1000].all()
