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


def bench_sst(args, world, rank, local):
    from bench import barrier, max_over_ranks, sum_over_ranks, HBM_PEAK_GBS
    ctx = lsmgpu.Context(local)
    n = (args.blocks or 100_000) * 33
    keys, koff, vals, voff = synth.kv_stream(n, first=rank * n)
    batch = lsmgpu.batch_to_device(ctx, keys, koff, vals, voff)
    starts = lsmgpu.segment_files(ctx, koff, voff, lsmgpu.MAX_SSTABLE_SIZE)
    sb = lsmgpu.prepare_sst(ctx, batch, starts)
    stream = torch.cuda.current_stream()
    for _ in range(args.warmup):
        lsmgpu.build_sst_into(ctx, batch, sb, stream=stream)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s, e in ev:
        s.record(stream)
        lsmgpu.build_sst_into(ctx, batch, sb, stream=stream)
        e.record(stream)
    torch.cuda.synchronize()
    barrier(world)
    elapsed = max_over_ranks(world, time.perf_counter() - t0)
    kern_ms = float(np.mean([s.elapsed_time(e) for s, e in ev]))
    img = float(sb.file_size.astype(np.float64).sum())
    img_all = sum_over_ranks(world, img)
    nf = len(starts) - 1
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
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seed 0x5EED, keys k%015d, splitmix64 values)",
        "config": {"workload": f"encode {n} records (16 B / 100 B) per GPU into {nf} .sst "
                               f"(2 MiB flush, bloom m=1.6M k=16)",
                   "files_per_gpu": nf, "image_bytes_per_gpu": int(img),
                   "parallelism": f"dp{world} (record ranges per rank, no collective)"},
        "roofline": {"bound": "hbm", "kernel": "lsm_build_sst (bloom + regions + meta)",
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "traffic_source": tsrc,
                     "alg_bytes_per_launch": int(alg), "kernel_ms": round(kern_ms, 5)},
    }
    return out, (keys, koff, vals, voff, starts)


def cpu_baseline_sst(args, data):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as ora
    keys, koff, vals, voff, starts = data
    t, done, img = 0.0, 0, 0
    f = 0
    while t < args.cpu_seconds and f < len(starts) - 1:
        t0 = time.perf_counter()
        out, _ = ora.build_sst(keys, koff, vals, voff, int(starts[f]), int(starts[f + 1]))
        t += time.perf_counter() - t0
        img += out.size
        done += 1
        f += 1
    return {"value": round(img / t / GIB, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"{done} of {len(starts) - 1} .sst images built by the C restatement "
                      f"in {t:.1f} s (1 thread)"}
