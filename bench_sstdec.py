"""Whole-.sst decode bench (BASELINE config 1 at one
image): `python bench.py --config sstdec` decodes the config-3 image set
(208 .sst images per GPU, built on the GPU by lsm_build_sst) with
lsm_decode_sst -- SSTable.DecodeFrom + DecodeDataBlock + GetKeyValuePairs in
one call; `--config sstdec1` decodes one 2,297,320-byte image (config 1).
Secondary bench lines; the headline is block decode (bench.py).
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "go-lsm_amd"))

import lsmgpu  # noqa: E402
from lsmgpu import synth  # noqa: E402

GIB = float(1 << 30)


def bench_sst_decode(args, world, rank, local):
    from bench import barrier, max_over_ranks, sum_over_ranks, timed_region, kernel_times, HBM_PEAK_GBS
    ctx = lsmgpu.Context(local)
    one = args.config == "sstdec1"
    n = 15_888 if one else (args.blocks or 100_000) * 33
    keys, koff, vals, voff = synth.kv_stream(n, first=rank * n)
    batch = lsmgpu.batch_to_device(ctx, keys, koff, vals, voff)
    starts = lsmgpu.segment_files(ctx, koff, voff, lsmgpu.MAX_SSTABLE_SIZE)
    sb = lsmgpu.build_sst(ctx, batch, starts)
    torch.cuda.synchronize()
    del batch
    nf = len(starts) - 1
    r = lsmgpu.alloc_sst_decode(ctx, sb.file_off, sb.file_size, int(sb.out.numel()))
    stream = torch.cuda.current_stream()
    for _ in range(args.warmup):
        lsmgpu.decode_sst_into(ctx, sb.out, r, stream=stream)
    torch.cuda.synchronize()
    meta = r.meta_numpy()
    assert (meta["stage"] == 0).all() and int(meta["nidx"].sum()) == n, "decode failed"

    def step():
        lsmgpu.decode_sst_into(ctx, sb.out, r, stream=stream)

    elapsed = timed_region(world, step, args.steps)
    times, kern_ms = kernel_times(step, stream, args.steps)
    parsed = float(meta["data_size"].astype(np.float64).sum() +
                   meta["idx_size"].astype(np.float64).sum())
    parsed_all = sum_over_ranks(world, parsed)
    # algorithmic bytes: both regions read; per record a key view (16 B), its
    # i64 offset (8 B) and a value view (16 B) written; 112 B meta per file
    alg = parsed + 40.0 * n + 112.0 * nf
    achieved = alg / (kern_ms * 1e-3) / 1e9
    from bench import traffic_from_profile
    traffic, tsrc = traffic_from_profile(f"{args.config}:{nf}")
    out = {
        "metric": "GiB/s of .sst data+index region bytes decoded to KV records",
        "value": round(parsed_all * args.steps / elapsed / GIB, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seed 0x5EED, keys k%015d, splitmix64 values); images built on the GPU",
        "config": {"workload": f"decode {nf} whole .sst image(s) per GPU ({n} records, "
                               f"16 B keys / 100 B values, 2 MiB flush)",
                   "files_per_gpu": nf, "records_per_gpu": n,
                   "parsed_bytes_per_gpu": int(parsed),
                   "parallelism": f"dp{world} (files per rank, no collective)",
                   "scaling_note": "weak, per-rank copy: every rank decodes its own image set"},
        "roofline": {"bound": "hbm", "kernel": "lsm_decode_sst (4 launches)",
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "traffic_source": tsrc,
                     "alg_bytes_per_launch": int(alg), "kernel_ms": round(kern_ms, 5)},
    }
    return out, (sb.out.cpu().numpy(), sb.file_off, sb.file_size, meta)


def cpu_baseline_sst_decode(args, data):
    """The oracle's SSTable decode (ora_sst_decode: framing, both chases,
    join counts; oracle/lsm_oracle.c) on the same images: 1 thread, and the
    CPU share's threads over whole images."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as ora
    from bench import host_cpu, timed_threads
    img, file_off, file_size, meta = data
    cpu = host_cpu()
    nf = len(file_off)
    parsed = (meta["data_size"] + meta["idx_size"]).astype(np.float64)

    def one(f):
        o, n = int(file_off[f]), int(file_size[f])
        ora.sst_decode(img[o:o + n])

    t1, done = 0.0, 0
    while (t1 < args.cpu_seconds / 3 or done == 0) and done < 10_000:
        t0 = time.perf_counter()
        one(done % nf)
        t1 += time.perf_counter() - t0
        done += 1
    v1 = float(sum(parsed[f % nf] for f in range(done))) / t1 / GIB
    passes, tn = timed_threads(one, list(range(nf)), cpu["threads"], args.cpu_seconds)
    vn = float(parsed.sum()) * passes / tn / GIB
    out = {"value": round(vn, 4), "unit": "GiB/s", "cores": cpu["threads"], "kind": "port",
           "sample": f"all {nf} images x {passes} passes on {cpu['threads']} threads in "
                     f"{tn:.1f} s; 1 thread: {done} image decodes in {t1:.1f} s",
           "value_1t": round(v1, 4), "host": cpu}
    if args.config == "sstdec1":
        out["file_backed"] = file_backed_baseline(args, img, file_off, file_size, parsed)
    return out


def file_backed_baseline(args, img, file_off, file_size, parsed):
    """config 1 from a real file the way the reference
    reads it -- SSTable.DecodeFrom(path) + GetDataBlockFromFile(path) over an
    unbuffered *os.File, one read(2) per length field, key and value
    (sstable.go:87-127,214-268; ora_sst_decode_file).  The file sits in the
    page cache (written just before), as a freshly flushed table does.
    1 thread: the reference decodes one file per goroutine."""
    import tempfile
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as ora
    o, n = int(file_off[0]), int(file_size[0])
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "000001.sst")
        with open(path, "wb") as f:
            f.write(img[o:o + n].tobytes())
        want = ora.sst_decode(img[o:o + n])[1].nidx
        t, reps = 0.0, 0
        while t < args.cpu_seconds / 3 or reps == 0:
            t0 = time.perf_counter()
            got = ora.sst_decode_file(path)
            t += time.perf_counter() - t0
            reps += 1
            assert got == want, (got, want)
    return {"value": round(float(parsed[0]) * reps / t / GIB, 5), "unit": "GiB/s", "cores": 1,
            "kind": "port", "ms_per_file": round(t * 1e3 / reps, 3),
            "sample": f"one {n}-byte .sst file, {want} pairs, {reps} decodes in {t:.1f} s "
                      "(one read(2) per field, page cache)"}


def bench_may_contain(args, world, rank, local):
    """batched SSTable.MayContain -- 1M probe keys (half
    held by the files, half not) against the 208 config-3 images."""
    from bench import barrier, max_over_ranks, sum_over_ranks, timed_region, kernel_times
    ctx = lsmgpu.Context(local)
    n = (args.blocks or 100_000) * 33
    keys, koff, vals, voff = synth.kv_stream(n, first=rank * n)
    batch = lsmgpu.batch_to_device(ctx, keys, koff, vals, voff)
    starts = lsmgpu.segment_files(ctx, koff, voff, lsmgpu.MAX_SSTABLE_SIZE)
    sb = lsmgpu.build_sst(ctx, batch, starts)
    r = lsmgpu.decode_sst(ctx, sb.out, sb.file_off, sb.file_size)
    torch.cuda.synchronize()
    del batch
    nf = len(starts) - 1
    nprobe = 1 << 20
    rng = np.random.default_rng(synth.SEED + rank)
    held = rng.integers(rank * n, rank * n + n, nprobe // 2)
    absent = rng.integers(10 ** 12, 10 ** 13, nprobe - nprobe // 2)  # outside every range
    ids = rng.permutation(np.concatenate([held, absent]))
    pk = synth.keys_for(ids).reshape(-1)
    pko = np.arange(nprobe + 1, dtype=np.uint64) * np.uint64(synth.KEY_LEN)
    probes = lsmgpu.batch_to_device(ctx, pk, pko, np.zeros(1, np.uint8),
                                    np.zeros(nprobe + 1, np.uint64))
    hit = torch.zeros((nprobe, nf), dtype=torch.uint8, device=ctx.torch_device)
    ws = lsmgpu.may_contain_workspace(ctx, nf, nprobe)
    stream = torch.cuda.current_stream()
    for _ in range(args.warmup):
        lsmgpu.may_contain_into(ctx, sb.out, r, probes, hit, ws=ws, stream=stream)
    torch.cuda.synchronize()

    def step():
        lsmgpu.may_contain_into(ctx, sb.out, r, probes, hit, ws=ws, stream=stream)

    elapsed = timed_region(world, step, args.steps)
    times, kern_ms = kernel_times(step, stream, args.steps)
    # checked after the timed region: host work between warmup and timing
    # left the GPU idle long enough to add ~20 ms of wake-up to the first step
    rows = hit.sum(dim=1).cpu().numpy()
    is_held = ids < 10 ** 12
    assert (rows[is_held] >= 1).all(), "false negative"
    total = sum_over_ranks(world, float(nprobe))
    fbits = r.meta_numpy()["filter_nbits"].astype(np.float64)
    alg = float(nprobe) * nf + pk.size + 8.0 * (nprobe + 1) + float((8 * np.ceil(fbits / 64)).sum())
    from bench import traffic_from_profile
    traffic, tsrc = traffic_from_profile(f"probe:{nf}:{nprobe}")
    out = {
        "metric": "M keys/s probed by SSTable.MayContain against every file",
        "value": round(total * args.steps / elapsed / 1e6, 2),
        "unit": "M keys/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 5),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic: the 208 config-3 images; probes half held, half outside every range",
        "config": {"workload": f"{nprobe} keys x {nf} .sst files per GPU (range check + bloom "
                               f"m=1.6M k=16)", "files_per_gpu": nf, "probes_per_gpu": nprobe,
                   "false_positive_rate_absent": float(rows[~is_held].astype(bool).mean()),
                   "parallelism": f"dp{world} (probe batches per rank, no collective)",
                   "scaling_note": "weak, per-rank copy: every rank probes its own level copy"},
        # algorithmic bytes per launch: the hit matrix written once, the probe
        # keys and offsets read once, every file's stored filter words read once
        "roofline": {"bound": "hbm", "kernel": "lsm_may_contain (all launches)",
                     "kernel_ms": round(kern_ms, 5), "achieved": round(alg / (kern_ms * 1e-3) / 1e9, 1),
                     "peak": 8000.0, "unit": "GB/s", "frac": round(alg / (kern_ms * 1e-3) / 1e9 / 8000.0, 4),
                     "traffic": traffic, "traffic_source": tsrc, "alg_bytes_per_launch": int(alg)},
    }
    return out, (sb.out.cpu().numpy(), sb.file_off, r.meta_numpy(), pk, nprobe)


def cpu_baseline_may_contain(args, data):
    """The oracle's batched SSTable.MayContain (ora_may_contain_batch: per
    (key, file) the range check in Go string order, then Filter.Test hashing
    the key as bloom.go does per file) over the same images and probes: 1
    thread, and the CPU share's threads over probe chunks."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as ora
    from bench import host_cpu, timed_threads
    img, file_off, meta, pk, nprobe = data
    cpu = host_cpu()
    nf = len(file_off)
    # lsm_sst_meta and the oracle's ora_sst_meta share one layout
    metas = (ora.SstMeta * nf).from_buffer_copy(np.ascontiguousarray(meta).tobytes())
    pko = np.arange(nprobe + 1, dtype=np.uint64) * np.uint64(16)
    chunk = 4096

    def one(c):
        ora.may_contain_batch(img, file_off, metas, pk, pko, c, min(nprobe, c + chunk))

    t1, done = 0.0, 0
    while (t1 < args.cpu_seconds / 3 or done == 0) and done < nprobe:
        t0 = time.perf_counter()
        one(done)
        t1 += time.perf_counter() - t0
        done += chunk
    sample = list(range(0, nprobe, chunk))
    passes, tn = timed_threads(one, sample, cpu["threads"], args.cpu_seconds)
    return {"value": round(nprobe * passes / tn / 1e6, 4), "unit": "M keys/s",
            "cores": cpu["threads"], "kind": "port",
            "sample": f"all {nprobe} probes x {nf} files x {passes} passes on {cpu['threads']} "
                      f"threads in {tn:.1f} s; 1 thread: {min(done, nprobe)} probes in {t1:.1f} s",
            "value_1t": round(min(done, nprobe) / t1 / 1e6, 4), "host": cpu}


def bench_level_search(args, world, rank, local):
    """SURVEY.md §8(f) f3 in the reference's own shape: batched
    Manager.searchFromLevelWithSparseIndex (manager.go:178-207) up to
    MayContain -- per probe the one candidate table of the level (sort.Search
    on MinKey, index--) and its MayContain; 1M probes (half held, half above
    every range) against the 208 config-3 images as one level."""
    from bench import sum_over_ranks, timed_region, kernel_times, traffic_from_profile
    ctx = lsmgpu.Context(local)
    n = (args.blocks or 100_000) * 33
    keys, koff, vals, voff = synth.kv_stream(n, first=rank * n)
    batch = lsmgpu.batch_to_device(ctx, keys, koff, vals, voff)
    starts = lsmgpu.segment_files(ctx, koff, voff, lsmgpu.MAX_SSTABLE_SIZE)
    sb = lsmgpu.build_sst(ctx, batch, starts)
    r = lsmgpu.decode_sst(ctx, sb.out, sb.file_off, sb.file_size)
    torch.cuda.synchronize()
    del batch
    nf = len(starts) - 1
    nprobe = 1 << 20
    rng = np.random.default_rng(synth.SEED + rank)
    held = rng.integers(rank * n, rank * n + n, nprobe // 2)
    absent = rng.integers(10 ** 12, 10 ** 13, nprobe - nprobe // 2)  # above every range
    ids = rng.permutation(np.concatenate([held, absent]))
    pk = synth.keys_for(ids).reshape(-1)
    pko = np.arange(nprobe + 1, dtype=np.uint64) * np.uint64(synth.KEY_LEN)
    probes = lsmgpu.batch_to_device(ctx, pk, pko, np.zeros(1, np.uint8),
                                    np.zeros(nprobe + 1, np.uint64))
    dev = ctx.torch_device
    table = torch.empty(nprobe, dtype=torch.int32, device=dev)
    may = torch.empty(nprobe, dtype=torch.uint8, device=dev)
    ws = lsmgpu.level_may_contain_workspace(ctx, nf, nprobe)
    stream = torch.cuda.current_stream()
    # the level's sparse index, built when the level changes (Manager keeps
    # sparseIndexes per level, manager.go:183-187), not per search batch
    index = lsmgpu.level_index(ctx, sb.out, r, stream=stream)
    # --config get: the whole batched Get of one level (searchFromTable,
    # manager.go:209-223): past the may bit, Iterator.Seek over the table's
    # decoded index and the value read by its offset (lsm_level_get)
    get = args.config == "get"
    result = torch.empty(nprobe, dtype=torch.int32, device=dev)
    value = torch.empty((nprobe, 4), dtype=torch.int32, device=dev)
    # the level's Seek tree (Go's bisection laid down as 16-byte key prefixes
    # in 128-byte blocks of three levels), built with the level like the
    # sparse index; --get-tree off walks the index itself (A/B)
    gtree = None
    if get and getattr(args, "get_tree", "on") == "on":
        t0 = time.perf_counter()
        gtree = lsmgpu.level_get_tree(ctx, sb.out, r, stream=stream)
        torch.cuda.synchronize()
        tree_build_ms = (time.perf_counter() - t0) * 1e3

    def step():
        if get:  # the level's search and Get in one call (lsm_level_search_get)
            lsmgpu.level_search_get_into(ctx, sb.out, r, probes, index, table, may, result, value,
                                         tree=gtree, ws=ws, stream=stream)
        else:
            lsmgpu.level_may_contain_into(ctx, sb.out, r, probes, table, may, ws=ws, stream=stream,
                                          index=index)

    for _ in range(args.warmup):
        step()
    elapsed = timed_region(world, step, args.steps)
    times, kern_ms = kernel_times(step, stream, args.steps)
    # the timed output: a held key's candidate is the table holding it, and
    # it may be there; a key above every range has the last table and no hit
    t_h, m_h = table.cpu().numpy(), may.cpu().numpy()
    is_held = ids < 10 ** 12
    rec = ids[is_held] - rank * n
    want_t = np.searchsorted(starts[1:].astype(np.int64), rec, side="right")
    assert np.array_equal(t_h[is_held], want_t), "candidate table"
    assert (m_h[is_held] == 1).all(), "false negative"
    assert (t_h[~is_held] == nf - 1).all() and (m_h[~is_held] == 0).all(), "absent keys"
    if get:
        # every held key found, its view the value's own bytes in its image;
        # every absent key absent
        res, val = result.cpu().numpy(), value.cpu().numpy().view(lsmgpu.DESC_DTYPE).reshape(-1)
        assert (res[is_held] == lsmgpu.GET_FOUND).all(), "held key not found"
        assert (res[~is_held] == lsmgpu.GET_ABSENT).all(), "absent key found"
        assert (val["val_len"][is_held] == synth.VAL_LEN).all() and (val["key_len"] == 0).all()
        fo = sb.file_off.astype(np.int64)
        st = starts.astype(np.int64)
        # header (two 16-byte keys) | filter block (32 + 8 words) | data region
        data_off = 8 + 2 * synth.KEY_LEN + 32 + 8 * ((lsmgpu.DEFAULT_BLOOM_M + 63) // 64)
        want_off = fo[want_t] + data_off + (rec - st[want_t]) * (4 + synth.VAL_LEN)
        assert np.array_equal(val["rec_off"][is_held].astype(np.int64), want_off), "value view"
    total = sum_over_ranks(world, float(nprobe))
    fbits = r.meta_numpy()["filter_nbits"].astype(np.float64)
    # algorithmic bytes per launch: 5 B out per probe (table + may), the probe
    # keys and offsets read once, every stored filter word read once; with
    # the Get also 20 B out per probe (result + value view) and, per probe
    # that passes MayContain, its index entry (4 + key + 8 B) and the value's
    # length prefix (4 B) read once
    alg = 5.0 * nprobe + pk.size + 8.0 * (nprobe + 1) + float((8 * np.ceil(fbits / 64)).sum())
    if get:
        npass = float(m_h.sum())
        alg += 20.0 * nprobe + npass * (4 + synth.KEY_LEN + 8 + 4)
    traffic, tsrc = traffic_from_profile(f"{'get' if get else 'level'}:{nf}:{nprobe}")
    out = {
        "metric": ("M keys/s looked up in one level (candidate table + MayContain + Seek + value)"
                   if get else "M keys/s searched in one level (candidate table + SSTable.MayContain)"),
        "value": round(total * args.steps / elapsed / 1e6, 2),
        "unit": "M keys/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 5),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic: the 208 config-3 images as one level; probes half held, half above "
                "every range",
        "verified": "every held probe: candidate = its table, may = 1; every absent probe: "
                    "the last table, may = 0" + ("; every held probe found with its value's view, "
                                                 "every absent probe absent" if get else ""),
        "config": {"workload": f"{nprobe} keys x one level of {nf} .sst files per GPU "
                               "(searchFromLevelWithSparseIndex -> MayContain" +
                               (" -> Iterator.Seek -> GetValueByOffset" if get else "") +
                               ", bloom m=1.6M k=16)",
                   "files_per_gpu": nf, "probes_per_gpu": nprobe,
                   "parallelism": f"dp{world} (probe batches per rank, no collective)",
                   "scaling_note": "weak, per-rank copy: every rank probes its own level copy"},
        **({"seek_tree": ({"bytes": int(gtree.data.numel()), "max_nidx": gtree.max_nidx,
                          "build_ms_once": round(tree_build_ms, 3),
                          "note": "built with the level (lsm_level_get_tree_build), outside the step, "
                                  "like the sparse index"} if gtree is not None else
                         "off: Seek bisects the decoded index")} if get else {}),
        "roofline": {"bound": "hbm", "kernel": ("lsm_level_search_get: lv_classify_kernel -> lv_test_kernel "
                                                "(MayContain) -> level_get_kernel (Seek through the Seek "
                                                "tree + value); sparse index and tree built once, "
                                                "outside the step" if get else
                                                "lsm_level_may_contain_indexed (all launches; the level's "
                                                "sparse index built once, outside the step)"),
                     "kernel_ms": round(kern_ms, 5),
                     "kernel_ms_median": round(float(np.median(times)), 5),
                     "achieved": round(alg / (kern_ms * 1e-3) / 1e9, 1),
                     "peak": 8000.0, "unit": "GB/s",
                     "frac": round(alg / (kern_ms * 1e-3) / 1e9 / 8000.0, 4),
                     "traffic": traffic, "traffic_source": tsrc, "alg_bytes_per_launch": int(alg)},
    }
    return out, (sb.out.cpu().numpy(), sb.file_off, r.meta_numpy(), pk, nprobe, sb.file_size, get)


def cpu_baseline_level_search(args, data):
    """The oracle's level search (ora_level_may_contain: Go's sort.Search over
    the MinKeys, then MayContain of the one candidate) over the same images
    and probes: 1 thread, and the CPU share's threads over probe chunks."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as ora
    from bench import host_cpu, timed_threads
    img, file_off, meta, pk, nprobe, file_size, get = data
    cpu = host_cpu()
    nf = len(file_off)
    metas = (ora.SstMeta * nf).from_buffer_copy(np.ascontiguousarray(meta).tobytes())
    pko = np.arange(nprobe + 1, dtype=np.uint64) * np.uint64(16)
    chunk = 16384
    gidx = None
    if get:  # the tables' index blocks, decoded once (SSTable.DecodeFrom at Recover)
        dec = [ora.sst_decode(img[int(file_off[f]):int(file_off[f]) + int(file_size[f])])
               for f in range(nf)]
        gidx = ora.level_get_index([d[2] for d in dec], [d[3] for d in dec])

    def one(c):
        c1 = min(nprobe, c + chunk)
        t, m = ora.level_may_contain(img, file_off, metas, pk, pko, c, c1)
        if get:
            ora.level_get(img, file_off, file_size, metas, None, None, pk, pko, c, c1, t, m,
                          index=gidx)

    t1, done = 0.0, 0
    while (t1 < args.cpu_seconds / 3 or done == 0) and done < nprobe:
        t0 = time.perf_counter()
        one(done)
        t1 += time.perf_counter() - t0
        done += chunk
    sample = list(range(0, nprobe, chunk))
    passes, tn = timed_threads(one, sample, cpu["threads"], args.cpu_seconds)
    return {"value": round(nprobe * passes / tn / 1e6, 4), "unit": "M keys/s",
            "cores": cpu["threads"], "kind": "port",
            "sample": f"all {nprobe} probes x {passes} passes on {cpu['threads']} threads in "
                      f"{tn:.1f} s; 1 thread: {min(done, nprobe)} probes in {t1:.1f} s",
            "value_1t": round(min(done, nprobe) / t1 / 1e6, 4), "host": cpu}


def level0_tables(rank, ntab=3, per=15_888, space=40_000):
    """go-lsm's level 0: ntab memtable flushes (2 MiB each, memtable.go:26;
    a third table triggers the level-0 compaction, manager.go:389-395), newest
    first (manager.go:284-287).  Table t holds `per` distinct random ids of one
    key space of `space` ids, so the tables overlap and share keys (the newer
    version wins); values differ per table.  -> list of (sorted ids, values)."""
    rng = np.random.default_rng(synth.SEED + 77 + rank)
    out = []
    for t in range(ntab):
        ids = np.sort(rng.choice(space, per, replace=False)).astype(np.int64)
        vals = synth.value_bytes(ids + (t + 1) * 10 ** 9, synth.VAL_LEN)
        out.append((ids, vals))
    return out


def bench_level0_get(args, world, rank, local):
    """SURVEY.md §8(f) f3 at level 0: batched Manager.searchFromLevel0
    (manager.go:160-176) -- per probe every level-0 table in order, newest
    first: MayContain, Seek, the value; the first value wins -- 1M probes
    (half held by some table, a quarter absent inside the tables' ranges, a
    quarter above them) against the 3 overlapping 2 MiB tables of a full
    level 0."""
    from bench import sum_over_ranks, timed_region, kernel_times, traffic_from_profile
    ctx = lsmgpu.Context(local)
    dev = ctx.torch_device
    space = 40_000
    tabs = level0_tables(rank, space=space)
    nf = len(tabs)
    # the tables' images, built on the device one after the other into one buffer
    imgs, offs, lens = [], [], []
    pos = 0
    for ids, vals in tabs:
        n = ids.size
        keys = synth.keys_for(ids).reshape(-1)
        batch = lsmgpu.batch_to_device(ctx, keys, np.arange(n + 1, dtype=np.uint64) * np.uint64(16),
                                       vals.reshape(-1).copy(),
                                       np.arange(n + 1, dtype=np.uint64) * np.uint64(synth.VAL_LEN))
        sb = lsmgpu.build_sst(ctx, batch, np.array([0, n], np.uint64))
        torch.cuda.synchronize()
        size = int(sb.file_size[0])
        imgs.append(sb.out[:size])
        offs.append(pos)
        lens.append(size)
        pos += (size + 15) // 16 * 16
    d_img = torch.zeros(pos + 64, dtype=torch.uint8, device=dev)
    for im, o in zip(imgs, offs):
        d_img[o:o + im.numel()] = im
    del imgs
    offs = np.array(offs, np.uint64)
    lens = np.array(lens, np.uint64)
    r = lsmgpu.decode_sst(ctx, d_img, offs, lens)
    tree = lsmgpu.level_get_tree(ctx, d_img, r)
    torch.cuda.synchronize()
    nprobe = 1 << 20
    rng = np.random.default_rng(synth.SEED + 5 + rank)
    union = np.unique(np.concatenate([t[0] for t in tabs]))
    missing = np.setdiff1d(np.arange(space), union)
    held = rng.choice(union, nprobe // 2)
    inside = rng.choice(missing, nprobe // 4)
    above = rng.integers(10 ** 12, 10 ** 13, nprobe - nprobe // 2 - nprobe // 4)
    ids = rng.permutation(np.concatenate([held, inside, above]))
    pk = synth.keys_for(ids).reshape(-1)
    pko = np.arange(nprobe + 1, dtype=np.uint64) * np.uint64(synth.KEY_LEN)
    probes = lsmgpu.batch_to_device(ctx, pk, pko, np.zeros(1, np.uint8), np.zeros(nprobe + 1, np.uint64))
    table = torch.empty(nprobe, dtype=torch.int32, device=dev)
    result = torch.empty(nprobe, dtype=torch.int32, device=dev)
    value = torch.empty((nprobe, 4), dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream()

    def step():
        lsmgpu.level0_get_into(ctx, d_img, r, probes, table, result, value, tree=tree, stream=stream)

    for _ in range(args.warmup):
        step()
    elapsed = timed_region(world, step, args.steps)
    times, kern_ms = kernel_times(step, stream, args.steps)
    # the timed output against the tables' own contents: a held key is
    # answered by the newest table holding it, with that version's value view
    # in that table's data region; every other key absent
    t_h, res = table.cpu().numpy(), result.cpu().numpy()
    val = value.cpu().numpy().view(lsmgpu.DESC_DTYPE).reshape(-1)
    want_t = np.full(nprobe, -1, np.int64)
    want_off = np.zeros(nprobe, np.int64)
    data_off = 8 + 2 * synth.KEY_LEN + 32 + 8 * ((lsmgpu.DEFAULT_BLOOM_M + 63) // 64)
    for t in range(nf - 1, -1, -1):  # older first, newer overwrite
        tid = tabs[t][0]
        j = np.searchsorted(tid, ids)
        inn = (j < tid.size) & (tid[np.minimum(j, tid.size - 1)] == ids)
        want_t[inn] = t
        want_off[inn] = int(offs[t]) + data_off + j[inn] * (4 + synth.VAL_LEN)
    found = want_t >= 0
    assert np.array_equal(t_h.astype(np.int64), want_t), "answering table"
    assert (res[found] == lsmgpu.GET_FOUND).all() and (res[~found] == lsmgpu.GET_ABSENT).all()
    assert np.array_equal(val["rec_off"][found].astype(np.int64), want_off[found]), "value view"
    assert (val["val_len"][found] == synth.VAL_LEN).all()
    total = sum_over_ranks(world, float(nprobe))
    fbits = r.meta_numpy()["filter_nbits"].astype(np.float64)
    # algorithmic bytes per launch: the probe keys and offsets read once, 24 B
    # out per probe (table, result, value view), every stored filter word read
    # once, and per table a probe is sought in (held keys: the tables up to the
    # answering one that hold it or pass its filter; counted here as the
    # answering table alone, a lower bound) its index entry (4 + key + 8 B)
    # and the value's length prefix (4 B) read once
    alg = pk.size + 8.0 * (nprobe + 1) + 24.0 * nprobe + float((8 * np.ceil(fbits / 64)).sum()) + \
        float(found.sum()) * (4 + synth.KEY_LEN + 8 + 4)
    traffic, tsrc = traffic_from_profile(f"get0:{nf}:{nprobe}")
    out = {
        "metric": "M keys/s looked up in level 0 (every table in order: MayContain + Seek + value)",
        "value": round(total * args.steps / elapsed / 1e6, 2),
        "unit": "M keys/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 5),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": f"synthetic: level 0 of {nf} overlapping 2 MiB tables (15,888 random keys each of one "
                f"{space}-key space, newest first); probes half held, a quarter absent inside the "
                "ranges, a quarter above them",
        "verified": "every probe: the answering table = the newest holding the key, its value's view; "
                    "every other probe absent",
        "config": {"workload": f"{nprobe} keys x level 0 of {nf} .sst files per GPU "
                               "(searchFromLevel0 -> searchFromTable per table: MayContain -> "
                               "Iterator.Seek -> GetValueByOffset, bloom m=1.6M k=16)",
                   "files_per_gpu": nf, "probes_per_gpu": nprobe,
                   "found": int(found.sum()),
                   "parallelism": f"dp{world} (probe batches per rank, no collective)",
                   "scaling_note": "weak, per-rank copy: every rank probes its own level copy"},
        "seek_tree": {"bytes": int(tree.data.numel()), "max_nidx": tree.max_nidx,
                      "note": "built with the level (lsm_level_get_tree_build), outside the step"},
        "roofline": {"bound": "hbm", "kernel": "lsm_level0_get (level0_get_kernel)",
                     "kernel_ms": round(kern_ms, 5),
                     "kernel_ms_median": round(float(np.median(times)), 5),
                     "achieved": round(alg / (kern_ms * 1e-3) / 1e9, 1),
                     "peak": 8000.0, "unit": "GB/s",
                     "frac": round(alg / (kern_ms * 1e-3) / 1e9 / 8000.0, 4),
                     "traffic": traffic, "traffic_source": tsrc, "alg_bytes_per_launch": int(alg)},
    }
    return out, (d_img.cpu().numpy(), offs, lens, pk, nprobe)


def cpu_baseline_level0_get(args, data):
    """The oracle's searchFromLevel0 (ora_level0_get: per probe every table in
    order, MayContain then Seek and the value) over the same images and probes:
    1 thread, and the CPU share's threads over probe chunks."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as ora
    from bench import host_cpu, timed_threads
    img, offs, lens, pk, nprobe = data
    cpu = host_cpu()
    nf = len(offs)
    dec = [ora.sst_decode(img[int(offs[f]):int(offs[f]) + int(lens[f])]) for f in range(nf)]
    metas = [d[1] for d in dec]
    gidx = ora.level_get_index([d[2] for d in dec], [d[3] for d in dec])
    pko = np.arange(nprobe + 1, dtype=np.uint64) * np.uint64(16)
    chunk = 16384

    def one(c):
        ora.level0_get(img, offs, lens, metas, None, None, pk, pko, c, min(nprobe, c + chunk), index=gidx)

    t1, done = 0.0, 0
    while (t1 < args.cpu_seconds / 3 or done == 0) and done < nprobe:
        t0 = time.perf_counter()
        one(done)
        t1 += time.perf_counter() - t0
        done += chunk
    sample = list(range(0, nprobe, chunk))
    passes, tn = timed_threads(one, sample, cpu["threads"], args.cpu_seconds)
    return {"value": round(nprobe * passes / tn / 1e6, 4), "unit": "M keys/s",
            "cores": cpu["threads"], "kind": "port",
            "sample": f"all {nprobe} probes x {passes} passes on {cpu['threads']} threads in "
                      f"{tn:.1f} s; 1 thread: {min(done, nprobe)} probes in {t1:.1f} s",
            "value_1t": round(min(done, nprobe) / t1 / 1e6, 4), "host": cpu}
