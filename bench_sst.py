"""BASELINE config 3: batch-encode a sorted KV stream through the builder rule
into .sst images with the bloom build fused (lsm_build_sst).  Secondary
bench line (`python bench.py --config sst`); the headline is decode.

Per GPU: 3.3 M records (16 B keys / 100 B values) -> 2 MiB flush rule ->
207 full .sst images (15,888 records, 2,297,320 B each) + 1 partial.
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


def sst_deal(args, world, rank):
    """Config 3 over N GPUs: the global stream -- 3.3M
    records by default -- is cut into files by the builder rule
    (builder.go:34-59) and whole files are dealt round-robin, file f -> rank
    f mod N (each file's filter is private: no reduction, no collective; the
    callers, manager.go:74-95 / :349-362, build each table on its own).
    -> (this rank's CSR batch of its files' records, its local file starts,
    its global file ids, the global file count, the builder-rule ms)."""
    n = (args.blocks or 100_000) * 33
    keys, koff, vals, voff = synth.kv_stream(n)
    tb0 = time.perf_counter()
    lib = lsmgpu._lib.load()
    gs = np.zeros(n + 2, dtype=np.uint64)
    nf = int(lib.lsm_segment_files_host(koff.ctypes.data, voff.ctypes.data, n,
                                        lsmgpu.MAX_SSTABLE_SIZE, gs.ctypes.data))
    gs = gs[:nf + 1].astype(np.int64)
    rule_ms = (time.perf_counter() - tb0) * 1e3
    mine = np.arange(rank, nf, world, dtype=np.int64)
    if world == 1:
        return (keys, koff, vals, voff), gs.astype(np.uint64), mine, nf, rule_ms
    lk, lv, lko, lvo, starts = [], [], [np.zeros(1, np.int64)], [np.zeros(1, np.int64)], [0]
    kb = vb = 0
    for f in mine:
        s, e = int(gs[f]), int(gs[f + 1])
        k0, k1, v0, v1 = int(koff[s]), int(koff[e]), int(voff[s]), int(voff[e])
        lk.append(keys[k0:k1])
        lv.append(vals[v0:v1])
        lko.append(koff[s + 1:e + 1].astype(np.int64) - k0 + kb)
        lvo.append(voff[s + 1:e + 1].astype(np.int64) - v0 + vb)
        kb += k1 - k0
        vb += v1 - v0
        starts.append(starts[-1] + (e - s))
    batch = (np.concatenate(lk), np.concatenate(lko).astype(np.uint64),
             np.concatenate(lv), np.concatenate(lvo).astype(np.uint64))
    return batch, np.array(starts, np.uint64), mine, nf, rule_ms


def bench_sst(args, world, rank, local):
    from bench import (barrier, max_over_ranks, sum_over_ranks, timed_region, kernel_times,
                       HBM_PEAK_GBS, aggregate_roofline)
    ctx = lsmgpu.Context(local)
    (keys, koff, vals, voff), starts, mine, nf_all, rule_ms = sst_deal(args, world, rank)
    n = len(koff) - 1
    batch = lsmgpu.batch_to_device(ctx, keys, koff, vals, voff)
    # One step = the whole builder path over this rank's stream as one call
    # (lsm_build_sst_stream): the builder rule on the device (builder.go:34-42
    # as merge.go:106-128 drives it), the image layout, then the images with
    # the fused bloom -- sized on host-known bounds, nothing read back.
    ss = lsmgpu.prepare_sst_stream(ctx, batch, lsmgpu.MAX_SSTABLE_SIZE)
    stream = torch.cuda.current_stream()
    for _ in range(args.warmup):
        lsmgpu.build_sst_stream_into(ctx, batch, ss, stream=stream)
    torch.cuda.synchronize()

    def step():
        lsmgpu.build_sst_stream_into(ctx, batch, ss, stream=stream)

    elapsed = timed_region(world, step, args.steps)
    times, kern_ms = kernel_times(step, stream, args.steps)
    sb = ss.result()
    # the device rule cut this rank's stream into exactly the files dealt to it
    if not np.array_equal(sb.file_start, starts):
        raise SystemExit("bench_sst: the device builder rule disagrees with the host rule")
    img = float(sb.file_size.astype(np.float64).sum())
    img_all = sum_over_ranks(world, img)
    nf = len(starts) - 1
    files_all = sum_over_ranks(world, float(nf))
    assert int(files_all) == nf_all, "every file built exactly once"
    # algorithmic bytes: keys + values + CSR offsets read once, images written
    alg = float(keys.size + vals.size + 16 * (n + 1)) + img
    achieved = alg / (kern_ms * 1e-3) / 1e9
    from bench import traffic_from_profile
    traffic, tsrc = traffic_from_profile(f"sst:{nf}")
    out = {
        "metric": "GiB/s of .sst image bytes encoded (builder rule + fused bloom)",
        "value": round(img_all * args.steps / elapsed / GIB, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 5),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seed 0x5EED, keys k%015d, splitmix64 values)",
        "config": {"workload": f"encode one {(args.blocks or 100_000) * 33}-record stream "
                               f"(16 B / 100 B) into {nf_all} .sst (2 MiB flush, bloom m=1.6M "
                               f"k=16), whole files dealt round-robin over {world} GPU(s)",
                   "files_total": nf_all, "files_rank0": nf, "image_bytes_rank0": int(img),
                   "step": "lsm_build_sst_stream: the builder rule (device), the layout and the "
                           "images in one call, no host round trip",
                   "deal_rule_ms": round(rule_ms, 3),
                   "deal": "the host rule cuts the global stream to deal whole files over the "
                           "ranks (outside the timed region); each rank's device rule re-derives "
                           "its files inside the step",
                   "parallelism": f"dp{world} (file f -> rank f mod {world}, no collective)"},
        "roofline": {"bound": "hbm", "kernel": "lsm_build_sst_stream: sst_stream_plan_kernel (rule + layout) -> "
                                               "sst_regions_kernel (regions + key hash) -> bloom_or_kernel "
                                               "(filter bits + framing)",
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "traffic_source": tsrc,
                     "alg_bytes_per_launch": int(alg), "kernel_ms": round(kern_ms, 5),
                     "kernel_ms_median": round(float(np.median(times)), 5),
                     "kernel_ms_min": round(float(times.min()), 5)},
    }
    if world > 1:
        out["roofline"]["aggregate"] = aggregate_roofline(world, alg, kern_ms)
    if not args.no_verify:
        verify_sst(ctx, batch, sb, keys, koff)
    out["config"]["verified"] = False if args.no_verify else ("device file starts equal the host rule's; "
                                 "every image parsed by lsm_decode_sst, V/IDX regions equal to the "
                                 "input, every 16th key present in its file's filter")
    return out, (keys, koff, vals, voff, starts, sb.file_size)


def verify_sst(ctx, batch, sb, keys, koff):
    """Check the timed output on the device, through the product's own f1
    and f3 paths (their parity is tested against the oracle): every image
    parses (SSTable.DecodeFrom stage ok, index and data counts equal the file's
    records), its V region holds [u32 vlen][value] of exactly the input's
    values, its IDX region [u32 klen][key][i64 offset] the input's keys and
    their records' offsets, and every 16th key tests present in its own file's
    filter (a bloom filter has no false negatives).  Fails the line on any
    difference."""
    nf = len(sb.file_start) - 1
    r = lsmgpu.decode_sst(ctx, sb.out, sb.file_off, sb.file_size)
    meta = r.meta_numpy()
    cnt = np.diff(sb.file_start.astype(np.int64))
    bad = np.nonzero((meta["stage"] != 0) | (meta["status"] != 0) |
                     (meta["ndata"] != cnt) | (meta["nidx"] != cnt))[0]
    if bad.size:
        raise SystemExit(f"bench_sst: {bad.size} images fail to decode (first {int(bad[0])}: "
                         f"stage {int(meta['stage'][bad[0]])})")
    kl, vl = int(koff[1] - koff[0]), int(batch.voff_host[1] - batch.voff_host[0])
    img = sb.out
    dev = img.device
    le = lambda x: torch.tensor(list(int(x).to_bytes(4, "little")), dtype=torch.uint8, device=dev)
    for f in range(nf):
        s, e = int(sb.file_start[f]), int(sb.file_start[f + 1])
        n, base = e - s, int(sb.file_off[f])
        d0, i0 = base + int(meta["data_off"][f]), base + int(meta["idx_off"][f])
        V = img[d0:d0 + n * (4 + vl)].view(n, 4 + vl)
        I = img[i0:i0 + n * (12 + kl)].view(n, 12 + kl)
        off = int(meta["data_off"][f]) + (4 + vl) * torch.arange(n, dtype=torch.int64, device=dev)
        ok = (bool((V[:, :4] == le(vl)).all()) and
              torch.equal(V[:, 4:], batch.vals[s * vl:e * vl].view(n, vl)) and
              bool((I[:, :4] == le(kl)).all()) and
              torch.equal(I[:, 4:4 + kl], batch.keys[s * kl:e * kl].view(n, kl)) and
              torch.equal(I[:, 4 + kl:].contiguous().view(torch.int64).view(-1), off))
        if not ok:
            raise SystemExit(f"bench_sst: image {f} differs from the input")
    sample = np.arange(0, len(koff) - 1, 16)
    ks = keys.reshape(-1, kl)[sample].reshape(-1)
    probe = lsmgpu.batch_to_device(ctx, ks, np.arange(sample.size + 1, dtype=np.uint64) * kl,
                                   np.zeros(16, np.uint8), np.zeros(sample.size + 1, np.uint64))
    hit = lsmgpu.may_contain(ctx, img, r, probe)
    fidx = torch.from_numpy(np.searchsorted(sb.file_start[1:].astype(np.int64), sample,
                                            side="right")).to(dev)
    own = hit[torch.arange(sample.size, device=dev), fidx]
    if not bool((own == 1).all()):
        raise SystemExit(f"bench_sst: {int((own != 1).sum())} sampled keys missing from their filter")


def cpu_baseline_sst(args, data):
    """The C restatement of Builder.Add/Build + SSTable.EncodeTo + Filter.Add
    (oracle/lsm_oracle.c ora_build_sst) on the host's cores: 1 thread, and
    the CPU share's threads over whole files (files are independent)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as ora
    from bench import host_cpu, timed_threads
    keys, koff, vals, voff, starts, file_size = data
    nf = len(starts) - 1
    cpu = host_cpu()

    def one(f):
        ora.build_sst(keys, koff, vals, voff, int(starts[f]), int(starts[f + 1]))

    t1, done = 0.0, 0
    while (t1 < args.cpu_seconds / 3 or done == 0) and done < nf:
        t0 = time.perf_counter()
        one(done)
        t1 += time.perf_counter() - t0
        done += 1
    v1 = float(np.sum(file_size[:done], dtype=np.float64)) / t1 / GIB
    passes, tn = timed_threads(one, list(range(nf)), cpu["threads"], args.cpu_seconds)
    vn = float(np.sum(file_size, dtype=np.float64)) * passes / tn / GIB
    return {"value": round(vn, 4), "unit": "GiB/s", "cores": cpu["threads"], "kind": "port",
            "sample": f"all {nf} .sst images x {passes} passes on {cpu['threads']} threads "
                      f"in {tn:.1f} s; 1 thread: {done} images in {t1:.1f} s",
            "value_1t": round(v1, 4), "host": cpu}
