"""GPU parity: the builder rule on the device (lsm_segment_files) and the
builder path over one sorted stream (lsm_build_sst_stream) vs the CPU
restatement.

The rule restates Builder.Add / ShouldFlush (builder.go:34-42, EstimateSize
kv.go:118-121) as CompactAndMergeKVs drives it (merge.go:106-128): the file
starts must equal ora.segment_files exactly, for streams of one record size
(config 3: one prediction round), of mixed and skewed sizes (the window
rounds), thresholds that cut every record, and the empty stream.  The stream
build must write, file for file, the oracle's .sst images.
"""
import numpy as np
import pytest
import torch

import lsmgpu
import pyoracle as ora
from lsmgpu import synth

pytestmark = pytest.mark.gpu

MiB2 = lsmgpu.MAX_SSTABLE_SIZE


def stream(rng, n, kmin, kmax, vmin, vmax, skew=False):
    kl = rng.integers(kmin, kmax + 1, n)
    if skew:  # config 5's value skew: 8 B .. 4 KiB, mostly small
        vl = np.minimum((8 * np.exp(rng.exponential(1.6, n))).astype(np.int64), 4096)
    else:
        vl = rng.integers(vmin, vmax + 1, n)
    keys = rng.integers(0, 256, max(int(kl.sum()), 1), dtype=np.uint8)
    vals = rng.integers(0, 256, max(int(vl.sum()), 1), dtype=np.uint8)
    koff = np.zeros(n + 1, np.uint64)
    voff = np.zeros(n + 1, np.uint64)
    koff[1:] = np.cumsum(kl)
    voff[1:] = np.cumsum(vl)
    return keys, koff, vals, voff


def check_rule(ctx, keys, koff, vals, voff, threshold):
    batch = lsmgpu.batch_to_device(ctx, keys, koff, vals, voff)
    got, counts = lsmgpu.segment_files_device(ctx, batch, threshold)
    want = ora.segment_files(koff, voff, threshold)
    assert int(counts[3]) == 0
    assert np.array_equal(got, want), (threshold, len(got), len(want))
    sizes = np.diff(want.astype(np.int64))
    assert int(counts[1]) == (int(sizes.max()) if sizes.size else 0)
    return want


@pytest.mark.parametrize("threshold", [0, 1, 17, 100, 5000, 20000, 262144, MiB2])
@pytest.mark.parametrize("shape", ["uniform", "mixed", "skewed"])
def test_segment_files_device(ctx, threshold, shape):
    rng = np.random.default_rng(threshold % 1009 + len(shape))
    n = 40_000
    if shape == "uniform":
        keys, koff, vals, voff = stream(rng, n, 16, 16, 100, 100)
    elif shape == "mixed":
        keys, koff, vals, voff = stream(rng, n, 0, 40, 0, 300)
    else:
        keys, koff, vals, voff = stream(rng, n, 4, 24, 0, 0, skew=True)
    check_rule(ctx, keys, koff, vals, voff, threshold)


@pytest.mark.parametrize("n", [0, 1, 2, 129])
def test_segment_files_small_streams(ctx, n):
    rng = np.random.default_rng(n)
    keys, koff, vals, voff = stream(rng, n, 0, 20, 0, 50)
    for t in (0, 1, 40, 400, MiB2):
        check_rule(ctx, keys, koff, vals, voff, t)


def test_segment_files_config3_full(ctx):
    """Config 3's stream: 207 files of 15,888 records and a partial one."""
    n = 100_000 * 33
    keys, koff, vals, voff = synth.kv_stream(n)
    want = check_rule(ctx, keys, koff, vals, voff, MiB2)
    assert len(want) == 209


def test_segment_files_drifting_sizes(ctx):
    """Record sizes that drift along the stream (values growing from 10 to
    900 B): every prediction from the mean so far misses, so the window
    rounds carry the whole chain."""
    n = 60_000
    vl = np.linspace(10, 900, n).astype(np.int64)
    koff = np.arange(n + 1, dtype=np.uint64) * 16
    voff = np.zeros(n + 1, np.uint64)
    voff[1:] = np.cumsum(vl)
    keys = np.zeros(16 * n, np.uint8)
    vals = np.zeros(int(voff[-1]), np.uint8)
    for t in (5000, 65536, MiB2):
        check_rule(ctx, keys, koff, vals, voff, t)


def test_segment_files_overflow(ctx):
    """A bound below the files the stream needs: nfile = 0, overflow = 1."""
    rng = np.random.default_rng(3)
    keys, koff, vals, voff = stream(rng, 5000, 8, 8, 50, 50)
    batch = lsmgpu.batch_to_device(ctx, keys, koff, vals, voff)
    need = len(ora.segment_files(koff, voff, 4096)) - 1
    _, c = lsmgpu.segment_files_device(ctx, batch, 4096, nfile_max=need - 1)
    assert int(c[0]) == 0 and int(c[3]) == 1
    fs, c = lsmgpu.segment_files_device(ctx, batch, 4096, nfile_max=need)
    assert int(c[0]) == need and int(c[3]) == 0
    assert np.array_equal(fs, ora.segment_files(koff, voff, 4096))


def images_vs_oracle(ctx, keys, koff, vals, voff, threshold, m, k, sample=None):
    batch = lsmgpu.batch_to_device(ctx, keys, koff, vals, voff)
    ss = lsmgpu.build_sst_stream(ctx, batch, threshold, m=m, k=k)
    sb = ss.result()
    starts = ora.segment_files(koff, voff, threshold)
    assert np.array_equal(sb.file_start, starts)
    out = sb.out.cpu().numpy()
    foot = sb.footer.cpu().numpy().reshape(-1, 4)
    nf = len(starts) - 1
    # 16-byte aligned offsets, packed in file order (lsm_sst_layout's layout)
    pad = (sb.file_size.astype(np.int64) + 15) // 16 * 16
    assert np.array_equal(sb.file_off.astype(np.int64), np.concatenate([[0], np.cumsum(pad)[:-1]])[:nf])
    for f in (range(nf) if sample is None else sample):
        want, wf = ora.build_sst(keys, koff, vals, voff, int(starts[f]), int(starts[f + 1]), m=m, k=k)
        o = int(sb.file_off[f])
        assert int(sb.file_size[f]) == want.size, f
        got = out[o:o + want.size]
        if not np.array_equal(got, want):
            bad = np.nonzero(got != want)[0]
            raise AssertionError(f"file {f}: {bad.size} bytes differ, first at {bad[0]} of {want.size}")
        assert np.array_equal(foot[f], wf), f
    return sb


@pytest.mark.parametrize("m,k", [(1_600_000, 16), (1_000_003, 20), (1000, 4), (1_638_401, 7)])
def test_build_sst_stream_random(ctx, m, k):
    """Mixed record sizes, many files; go-lsm's filter shape (every launch
    sized on the bound) and other shapes (the counts read back)."""
    rng = np.random.default_rng(m + k)
    keys, koff, vals, voff = stream(rng, 3000, 0, 24, 0, 180)
    images_vs_oracle(ctx, keys, koff, vals, voff, 20000, m, k)


def test_build_sst_stream_edges(ctx):
    """A threshold below every record (one file per record), never flush
    (one file), and a record larger than the threshold mid-stream."""
    items_k = [b"", b"a", b"x" * 300, b"", b"key"] * 40
    items_v = [b"", b"", b"v" * 5000, b"q", b""] * 40
    koff = np.zeros(len(items_k) + 1, np.uint64)
    koff[1:] = np.cumsum([len(x) for x in items_k])
    voff = np.zeros(len(items_v) + 1, np.uint64)
    voff[1:] = np.cumsum([len(x) for x in items_v])
    keys = np.frombuffer(b"".join(items_k), np.uint8)
    vals = np.frombuffer(b"".join(items_v), np.uint8)
    for t in (1, 0, 4000):
        images_vs_oracle(ctx, keys, koff, vals, voff, t, 1_600_000, 16)


def test_build_sst_stream_config3(ctx):
    """Config 3 through the one-call stream build: the 208 images equal, byte
    for byte, lsm_build_sst's (every one of which test_sst_config3_full checks
    against the oracle), three sampled against the oracle here, and every
    image decodes back (lsm_decode_sst)."""
    n = 100_000 * 33
    keys, koff, vals, voff = synth.kv_stream(n)
    sb = images_vs_oracle(ctx, keys, koff, vals, voff, MiB2, 1_600_000, 16, sample=(0, 101, 207))
    assert sb.nfile == 208 and (sb.file_size[:-1] == 2_297_320).all()
    batch = lsmgpu.batch_to_device(ctx, keys, koff, vals, voff)
    ref = lsmgpu.build_sst(ctx, batch, sb.file_start)
    torch.cuda.synchronize()
    assert np.array_equal(ref.file_off, sb.file_off)
    # image by image (the alignment gaps between images are never written)
    for f in range(sb.nfile):
        o, z = int(sb.file_off[f]), int(sb.file_size[f])
        assert torch.equal(ref.out[o:o + z], sb.out[o:o + z]), f"image {f} differs"
    r = lsmgpu.decode_sst(ctx, sb.out, sb.file_off, sb.file_size)
    torch.cuda.synchronize()
    meta = r.meta_numpy()
    sizes = np.diff(sb.file_start.astype(np.int64))
    assert (meta["stage"] == 0).all() and np.array_equal(meta["nidx"].astype(np.int64), sizes)


def test_build_sst_stream_many_files(ctx):
    """More files than the plan kernel keeps in LDS (4,096): the layout reads
    the later file starts from global memory."""
    rng = np.random.default_rng(11)
    keys, koff, vals, voff = stream(rng, 5000, 1, 12, 0, 30)
    images_vs_oracle(ctx, keys, koff, vals, voff, 1, 1000, 4,
                     sample=(0, 1, 4095, 4096, 4097, 4999))
