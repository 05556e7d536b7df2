"""GPU parity of lsm_decode_sst against the oracle.

The oracle (oracle/lsm_oracle.c ora_sst_decode) restates SSTable.DecodeFrom
(sstable.go:87-128), DecodeDataBlock (:214-225) and GetKeyValuePairs
(:248-268).  Every image is decoded by both; the per-file meta (framing,
stage, status, entry counts) and every index entry / value view must be
identical.  Images come from the oracle's own builder (ora_build_sst) with
record shapes that keep or break the kernels' stride / offset hypotheses,
and from corruptions of them (truncation, footer fields, swapped or shifted
index offsets, extra or missing values, random bytes).
"""
import struct

import numpy as np
import pytest
import torch

import lsmgpu
import pyoracle as ora
from lsmgpu import synth

pytestmark = pytest.mark.gpu


def csr(items):
    data = b"".join(items)
    off = np.zeros(len(items) + 1, np.uint64)
    off[1:] = np.cumsum([len(x) for x in items])
    return np.frombuffer(data, np.uint8) if data else np.zeros(0, np.uint8), off


def build(keys, vals, m=4096, k=4):
    kb, ko = csr(keys)
    vb, vo = csr(vals)
    img, _ = ora.build_sst(kb, ko, vb, vo, 0, len(keys), m=m, k=k)
    return img


def pack(images, rng, pad=29):
    """Images at odd offsets in one buffer."""
    parts, offs, lens, pos = [], [], [], 0
    for im in images:
        gap = int(rng.integers(0, pad))
        parts.append(np.zeros(gap, np.uint8))
        pos += gap
        offs.append(pos)
        lens.append(im.size)
        parts.append(np.asarray(im, np.uint8))
        pos += im.size
    return np.concatenate(parts), np.array(offs, np.uint64), np.array(lens, np.uint64)


def check(ctx, images, seed=0):
    rng = np.random.default_rng(seed)
    buf, offs, lens = pack(images, rng)
    d_img = lsmgpu.to_device_bytes(buf, ctx.torch_device)
    r = lsmgpu.decode_sst(ctx, d_img, offs, lens)
    torch.cuda.synchronize()
    meta = r.meta_numpy()
    idesc = r.idx_desc.cpu().numpy().view(np.uint8).view(lsmgpu.DESC_DTYPE).reshape(-1)
    ival = r.idx_value.cpu().numpy()
    ddesc = r.data_desc.cpu().numpy().view(np.uint8).view(lsmgpu.DESC_DTYPE).reshape(-1)
    bases = r.bases()
    stages = []
    for f, im in enumerate(images):
        rc, om, oi, oiv, od = ora.sst_decode(im)
        g = meta[f]
        for name, _ in ora.SstMeta._fields_:
            assert int(g[name]) == int(getattr(om, name)), (f, name, int(g[name]), getattr(om, name))
        b, o = int(bases[f]), int(offs[f])
        gi = idesc[b:b + om.nidx].copy()
        gi["rec_off"] -= np.uint64(o)
        assert np.array_equal(gi, oi), f
        assert np.array_equal(ival[b:b + om.nidx], oiv), f
        gd = ddesc[b:b + om.ndata].copy()
        gd["rec_off"] -= np.uint64(o)
        assert np.array_equal(gd, od), f
        stages.append(int(g["stage"]))
    return stages


def kv_set(rng, n, klen=None, vmax=200, vmin=0):
    keys = [(b"k%015d" % i) if klen is None else rng.integers(97, 123, klen, dtype=np.uint8).tobytes()
            for i in range(n)]
    vals = [rng.integers(0, 256, int(rng.integers(vmin, vmax + 1)), dtype=np.uint8).tobytes()
            for _ in range(n)]
    return keys, vals


def test_well_formed_tables(ctx):
    rng = np.random.default_rng(1)
    images = []
    for n in (0, 1, 2, 3, 64, 65, 500, 3000):
        images.append(build(*kv_set(rng, n)))
    # key lengths that vary (the index stride hypothesis fails -> exact chase)
    keys = [rng.integers(97, 123, int(rng.integers(0, 40)), dtype=np.uint8).tobytes() for _ in range(700)]
    images.append(build(keys, kv_set(rng, 700)[1]))
    # uniform values (both hypotheses hold everywhere) and values larger than the ring
    images.append(build([b"k%015d" % i for i in range(2000)], [b"v" * 100] * 2000))
    images.append(build(*kv_set(rng, 40, vmin=5000, vmax=20000)))
    # empty values and empty keys
    images.append(build([b""] * 10, [b""] * 10))
    stages = check(ctx, images)
    # the empty table is the reference's quirk: DataHandle.Size == 0 means
    # "read to EOF" (data.go:51-54), so the footer is chased as values
    assert stages == [5] + [0] * (len(images) - 1)


def corrupt_footer(im, field, value):
    im = im.copy()
    n = im.size
    im[n - 32 + 8 * field:n - 24 + 8 * field] = np.frombuffer(struct.pack("<q", value), np.uint8)
    return im


def footer(im):
    return struct.unpack("<4q", im[-32:].tobytes())


def test_footer_and_framing_errors(ctx):
    rng = np.random.default_rng(2)
    base = build(*kv_set(rng, 300))
    d_off, d_size, i_off, i_size = footer(base)
    images = [
        base[:3], base[:7], base[:40], base[:200], base[:-40],      # header / filter / index cut
        np.zeros(0, np.uint8), base[:i_off + 5],
        corrupt_footer(base, 2, -1),                                # negative index offset
        corrupt_footer(base, 3, -5),                                # negative index size
        corrupt_footer(base, 3, i_size + 1000),                     # index runs past EOF
        corrupt_footer(base, 3, i_size - 7),                        # index size cuts an entry
        corrupt_footer(base, 3, 0),                                 # empty index
        corrupt_footer(base, 0, -3),                                # negative data offset
        corrupt_footer(base, 1, 0),                                 # data size 0: to EOF
        corrupt_footer(base, 1, -9),                                # negative size: to EOF
        corrupt_footer(base, 1, d_size - 50),                       # data cut mid-value
        corrupt_footer(base, 1, d_size + 10_000_000),               # data size past EOF
        corrupt_footer(base, 0, d_off + 4 + 1),                     # data starts mid-record
        corrupt_footer(base, 0, 10 ** 12),                          # data offset past EOF
        corrupt_footer(base, 2, 10 ** 12),                          # index offset past EOF
    ]
    check(ctx, images, seed=3)


def test_index_offsets_that_lie(ctx):
    """Index offsets are only a hint for the value positions: swapped,
    shifted or garbage offsets must give the serial chase's values."""
    rng = np.random.default_rng(4)
    images = []
    for trial in range(24):
        keys, vals = kv_set(rng, int(rng.integers(1, 400)), vmax=int(rng.choice([8, 100, 3000])))
        im = build(keys, vals)
        d_off, d_size, i_off, i_size = footer(im)
        n = len(keys)
        # index entry j's offset field sits at i_off + j*28 + 4 + 16 (16-byte keys)
        j = int(rng.integers(0, n))
        at = i_off + j * 28 + 20
        kind = trial % 6
        im = im.copy()
        if kind == 0 and n > 1:  # swap two offsets
            j2 = (j + 1) % n
            at2 = i_off + j2 * 28 + 20
            a, b = im[at:at + 8].copy(), im[at2:at2 + 8].copy()
            im[at:at + 8], im[at2:at2 + 8] = b, a
        elif kind == 1:
            im[at:at + 8] = np.frombuffer(struct.pack("<q", int(rng.integers(-2**40, 2**40))), np.uint8)
        elif kind == 2:
            v = struct.unpack("<q", im[at:at + 8].tobytes())[0]
            im[at:at + 8] = np.frombuffer(struct.pack("<q", v + 1), np.uint8)
        elif kind == 3:  # a value length field in the data region
            vs = int(rng.integers(d_off, d_off + d_size - 4)) if d_size > 4 else d_off
            im[vs:vs + 4] = np.frombuffer(struct.pack("<I", int(rng.integers(0, 2**32))), np.uint8)
        elif kind == 4:  # a key length field in the index region
            im[i_off + j * 28:i_off + j * 28 + 4] = np.frombuffer(struct.pack("<I", int(rng.choice([0, 15, 17, 2**31]))), np.uint8)
        else:  # random bytes over both regions
            k = int(rng.integers(1, 20))
            pos = rng.integers(d_off, im.size - 32, k)
            im[pos] = rng.integers(0, 256, k, dtype=np.uint8)
        images.append(im)
    check(ctx, images, seed=5)


def test_count_mismatch(ctx):
    """DataBlock and IndexBlock of different lengths: stage 6 (sstable.go:254-257)."""
    rng = np.random.default_rng(6)
    keys, vals = kv_set(rng, 50)
    im = build(keys, vals)
    d_off, d_size, i_off, i_size = footer(im)
    # drop the last index entry (index size - 28)
    short_idx = corrupt_footer(im, 3, i_size - 28)
    # make the data region end before the last value
    vlast = 4 + len(vals[-1])
    short_data = corrupt_footer(im, 1, d_size - vlast)
    stages = check(ctx, [short_idx, short_data], seed=7)
    assert stages == [6, 6]


def test_config3_images(ctx):
    """The bench's encode workload: 208 GPU-built images (15,888 records of
    16 B keys / 100 B values each, default bloom), decoded in one call."""
    keys, koff, vals, voff = synth.kv_stream(3_300_000)
    batch = lsmgpu.batch_to_device(ctx, keys, koff, vals, voff)
    starts = lsmgpu.segment_files(ctx, koff, voff)
    sb = lsmgpu.build_sst(ctx, batch, starts)
    torch.cuda.synchronize()
    nf = len(starts) - 1
    assert nf == 208
    r = lsmgpu.decode_sst(ctx, sb.out, sb.file_off, sb.file_size)
    torch.cuda.synchronize()
    meta = r.meta_numpy()
    counts = np.diff(starts.astype(np.int64))
    assert (meta["stage"] == 0).all()
    assert np.array_equal(meta["nidx"], counts) and np.array_equal(meta["ndata"], counts)
    # every value view points at its record's bytes; every key at its key
    idesc = r.idx_desc.view(-1, 4)
    ddesc = r.data_desc.view(-1, 4)
    bases = torch.from_numpy(r.bases().astype(np.int64)).to(ctx.torch_device)
    cnt = torch.from_numpy(counts).to(ctx.torch_device)
    rec = torch.repeat_interleave(torch.arange(nf, device=ctx.torch_device), cnt)
    first = torch.repeat_interleave(torch.cumsum(cnt, 0) - cnt, cnt)
    slot = bases[rec] + torch.arange(int(cnt.sum()), device=ctx.torch_device) - first
    koff_d = (idesc[slot, 0].long() & 0xFFFFFFFF) + 4
    voff_d = (ddesc[slot, 0].long() & 0xFFFFFFFF) + 4
    assert bool((idesc[slot, 2] == 16).all()) and bool((ddesc[slot, 3] == 100).all())
    kb = sb.out[koff_d[:, None] + torch.arange(16, device=ctx.torch_device)[None, :]]
    vb = sb.out[voff_d[:, None] + torch.arange(100, device=ctx.torch_device)[None, :]]
    assert torch.equal(kb.reshape(-1).cpu(), torch.from_numpy(keys))
    assert torch.equal(vb.reshape(-1).cpu(), torch.from_numpy(vals))
    # oracle on a sample of files
    out = sb.out.cpu().numpy()
    for f in (0, 1, 103, 207):
        o, n = int(sb.file_off[f]), int(sb.file_size[f])
        rc, om, *_ = ora.sst_decode(out[o:o + n])
        for name, _ in ora.SstMeta._fields_:
            assert int(meta[f][name]) == int(getattr(om, name)), (f, name)


@pytest.mark.parametrize("shape", ["rare_key_break", "wide_values", "tiny_records", "mid_corrupt"])
def test_fuzz_large_tables(ctx, shape):
    """Tables large enough to be split over many workgroups, with the
    stride / offset hypotheses broken rarely (so a break can land on a
    workgroup boundary) or a byte corrupted somewhere in the middle."""
    rng = np.random.default_rng(sum(map(ord, shape)))
    images = []
    for _ in range(4):
        n = int(rng.integers(5_000, 16_000))
        if shape == "rare_key_break":
            keys = [b"k%015d" % i if rng.random() > 0.001 else b"k%016d" % i for i in range(n)]
            vals = [rng.integers(0, 256, 100, dtype=np.uint8).tobytes() for _ in range(n)]
        elif shape == "wide_values":
            keys, vals = kv_set(rng, n, vmax=600)
        elif shape == "tiny_records":
            keys = [rng.integers(97, 123, int(rng.integers(0, 4)), dtype=np.uint8).tobytes() for _ in range(n)]
            vals = [rng.integers(0, 256, int(rng.integers(0, 5)), dtype=np.uint8).tobytes() for _ in range(n)]
        else:
            keys, vals = kv_set(rng, n, vmax=150)
        im = build(keys, vals)
        if shape == "mid_corrupt":
            d_off, d_size, i_off, i_size = footer(im)
            im = im.copy()
            at = int(rng.integers(d_off, i_off + i_size))
            im[at] ^= np.uint8(1 << int(rng.integers(0, 8)))
        images.append(im)
    check(ctx, images, seed=11)
