#!/usr/bin/env python3
"""Benchmark of the gfx950 go-lsm block codec (BASELINE.json metric).

Default workload (N=1): BASELINE config 2 -- batch-decode 100,000 synthetic
4 KiB KV blocks (33 records of 16 B keys / 100 B values, 4,092 parsed bytes
per 4,096-byte slot), device resident, descriptor output.  One step = one
lsm_decode_blocks launch over the whole batch.

N>1 (torchrun, one process per GPU): the global batch is N x 100,000 blocks
dealt round-robin (block i -> rank i mod N); no data-path collective, the
ranks only meet at the barriers around the timed region (weak scaling).

value = sum of parsed block bytes over all ranks / max-over-ranks wall time.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "go-lsm_amd"))

import lsmgpu  # noqa: E402
from lsmgpu import synth  # noqa: E402

METRIC = "GiB/s of device-resident .sst data-block bytes decoded to KV records"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, MI355X_MICROARCH.md
GIB = float(1 << 30)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="decode4k",
                    choices=["decode4k", "decode64k", "mixed", "sst", "sstdec", "sstdec1", "wal",
                             "probe", "compact"])
    ap.add_argument("--blocks", type=int, default=None, help="blocks per GPU")
    ap.add_argument("--arena", action="store_true", help="materialize keys/values too")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--e2e", action="store_true",
                    help="host-resident blocks: pinned H2D -> decode -> compact -> D2H "
                         "(the PCIe-inclusive rate recorded in DESIGN.md; not the headline)")
    ap.add_argument("--chunk", type=int, default=8192, help="blocks per e2e pipeline chunk")
    return ap.parse_args()


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and os.environ.get("LSM_BENCH_REHEARSE"):
        # rehearsal of the N-rank path on a one-GPU box: every rank on cuda:0,
        # gloo for the barrier and the two scalar reductions (never a result)
        import torch.distributed as dist
        local = 0
        torch.cuda.set_device(0)
        dist.init_process_group("gloo")
    elif world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)
    return world, rank, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def _reduce(world, x, op):
    if world == 1:
        return x
    import torch.distributed as dist
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=op)
    return float(t.item())


def max_over_ranks(world, x):
    import torch.distributed as dist
    return _reduce(world, x, dist.ReduceOp.MAX if world > 1 else None)


def sum_over_ranks(world, x):
    import torch.distributed as dist
    return _reduce(world, x, dist.ReduceOp.SUM if world > 1 else None)


def shard_block_ids(rank, world, per):
    """Round-robin deal of the global batch: block i -> rank i mod N."""
    return rank + world * np.arange(per, dtype=np.int64)


def traffic_from_profile(workload_key):
    """HBM bytes per launch from the committed PMC summary (rocprofv3 --pmc,
    FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM + WRITE_SIZE), if any."""
    d = os.path.join(ROOT, "profiles")
    if not os.path.isdir(d):
        return None, None
    best = None
    for name in sorted(os.listdir(d)):
        if name.endswith(".json") and "pmc" in name:
            try:
                j = json.load(open(os.path.join(d, name)))
            except Exception:
                continue
            if j.get("workload_key") == workload_key and "hbm_bytes_per_launch" in j:
                best = (float(j["hbm_bytes_per_launch"]), "profiles/" + name)
    return best if best else (None, None)


def make_workload(args, world, rank):
    if args.config in ("decode4k", "decode64k"):
        per = args.blocks or (100_000 if args.config == "decode4k" else 6_400)
        ids = shard_block_ids(rank, world, per)
        if args.config == "decode4k":
            buf, off, ln = synth.uniform_kv_blocks(ids)
            desc = "decode %d x 4 KiB KV blocks per GPU (33 x 16 B key / 100 B value)" % per
        else:
            # 64 KiB slots: 528 records x 124 B = 65,472 parsed bytes
            buf, off, ln = synth.uniform_kv_blocks(ids, recs=528, slot=65536)
            desc = "decode %d x 64 KiB KV blocks per GPU (528 x 16 B key / 100 B value)" % per
        return buf, off, ln, desc
    if args.config == "mixed":
        total = (args.blocks or 1 << 30)
        buf, off, ln, _ = synth.mixed_kv_blocks(total, seed=synth.SEED + rank)
        return buf, off, ln, "decode mixed 4/16/64 KiB KV blocks, values log-uniform 8 B-4 KiB"
    if args.config == "wal":
        # §8(f) f4: wal.Recover of memtable-sized logs shaped by go-lsm's
        # benchmark; 16 distinct logs generated, dealt 4x (generation is slow)
        nlog = args.blocks or 64
        b16, o16, l16, _ = synth.wal_logs(min(16, nlog), seed=synth.SEED + rank)
        reps = (nlog + 15) // 16
        span = b16.size
        buf = np.tile(b16, reps)
        off = np.concatenate([o16 + np.uint64(r * span) for r in range(reps)])[:nlog]
        ln = np.tile(l16, reps)[:nlog]
        return buf, off, ln, (f"replay {nlog} write-ahead logs per GPU (2 MiB memtables, "
                              "benchmark.go-shaped records)")
    raise ValueError(args.config)


def bench_decode(args, world, rank, local):
    ctx = lsmgpu.Context(local)
    dev = ctx.torch_device
    buf, blk_off, blk_len, wdesc = make_workload(args, world, rank)
    nblk = blk_off.size
    d_in = lsmgpu.to_device_bytes(buf, dev)
    d_off = torch.tensor(blk_off.view(np.int64), device=dev)
    d_len = torch.tensor(blk_len.view(np.int32), device=dev)
    r = lsmgpu.alloc_decode_offset(ctx, lsmgpu.GRAMMAR_KV, nblk, int(d_in.numel()),
                                   arena=args.arena)
    stream = torch.cuda.current_stream()

    wal_max = int(blk_len.max()) if args.config == "wal" else 0
    wal_ws = lsmgpu.wal_workspace(ctx, nblk, wal_max) if args.config == "wal" else None

    def step():
        if args.config == "wal":
            lsmgpu.wal_replay_into(ctx, d_in, d_off, d_len, wal_max, r, wal_ws, stream=stream)
        else:
            lsmgpu.decode_into(ctx, lsmgpu.GRAMMAR_KV, d_in, d_off, d_len, r, stream=stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # correctness gate on the warmed-up output: every block decoded cleanly
    assert int((r.status[:nblk] != 0).sum()) == 0, "decode reported errors"
    nrec_total = int(r.nrec[:nblk].sum().item())

    starts = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        starts[i].record(stream)
        step()
        ends[i].record(stream)
    torch.cuda.synchronize()
    barrier(world)
    t1 = time.perf_counter()
    elapsed = max_over_ranks(world, t1 - t0)
    kern_ms = float(np.mean([s.elapsed_time(e) for s, e in zip(starts, ends)]))

    parsed = float(blk_len.astype(np.float64).sum())
    parsed_all = sum_over_ranks(world, parsed)
    value = parsed_all * args.steps / elapsed / GIB

    # algorithmic bytes of one launch: block bytes +
    # per-block metadata (blk_off 8 + blk_len 4) read; 16 B per record
    # descriptor + nrec/status (8 B per block) written; arenas add the key and
    # value bytes written.
    alg = parsed + 12.0 * nblk + 16.0 * nrec_total + 8.0 * nblk
    if args.arena:
        alg += float(nrec_total) * (16 + 100) if args.config != "mixed" else parsed
    achieved = alg / (kern_ms * 1e-3) / 1e9
    wkey = f"{args.config}:{nblk}:{'arena' if args.arena else 'desc'}"
    traffic, tsrc = traffic_from_profile(wkey)
    out = {
        "metric": METRIC,
        "value": round(value, 2),
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
        "config": {
            "workload": wdesc,
            "grammar": "KV (kv/kv.go:46-115)",
            "output": "ARENA (descriptors + packed keys/values)" if args.arena else
                      "DESC (16 B record descriptors)",
            "blocks_per_gpu": int(nblk),
            "records_per_gpu": nrec_total,
            "parsed_bytes_per_gpu": int(parsed),
            "parallelism": f"dp{world} (blocks round-robin, no collective)",
        },
        "roofline": {
            "bound": "hbm",
            "kernel": ("lsm_wal_replay (seg + stitch + compact launches)" if args.config == "wal"
                       else "decode_v2_kernel<KV,8>"),
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_source": tsrc,
            "alg_bytes_per_launch": int(alg),
            "kernel_ms": round(kern_ms, 5),
        },
    }
    return out, (buf, blk_off, blk_len)


def bench_e2e(args, world, rank, local):
    """decode4k with the blocks in pinned host memory (the page cache stand-in)
    and the decoded records returned to pinned host memory, chunked so the
    H2D copy, the decode + compaction and the D2H copy of consecutive chunks
    overlap on three streams (two device slots)."""
    ctx = lsmgpu.Context(local)
    dev = ctx.torch_device
    per = args.blocks or 100_000
    buf, blk_off, blk_len = synth.uniform_kv_blocks(shard_block_ids(rank, world, per))
    slot_bytes = 4096
    h_in = torch.from_numpy(buf[: per * slot_bytes]).pin_memory()
    h_len = torch.from_numpy(blk_len.view(np.int32).copy()).pin_memory()
    C = min(args.chunk, per)
    nch = (per + C - 1) // C
    g = lsmgpu.GRAMMAR_KV
    d_off = torch.arange(C, dtype=torch.int64, device=dev) * slot_bytes
    cap = C * (slot_bytes // 8)
    slots = []
    for _ in range(2):
        d_in = torch.zeros(C * slot_bytes + 64, dtype=torch.uint8, device=dev)
        r = lsmgpu.alloc_decode_offset(ctx, g, C, C * slot_bytes)
        slots.append(dict(d_in=d_in, d_len=torch.empty(C, dtype=torch.int32, device=dev), r=r,
                          dense=lsmgpu.alloc_dense(ctx, g, C, cap)))
    h_desc = torch.empty((per * 33 + 64, 4), dtype=torch.int32).pin_memory()
    h_meta = torch.zeros((nch, 2, C), dtype=torch.int32).pin_memory()
    h_cnt = torch.zeros(nch, dtype=torch.int64).pin_memory()
    s_h2d, s_comp, s_d2h = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    ev_h2d = [torch.cuda.Event() for _ in range(2)]
    ev_comp = [torch.cuda.Event() for _ in range(2)]
    ev_free = [torch.cuda.Event() for _ in range(2)]

    def run_once():
        pos = 0
        for c in range(nch + 1):
            if c < nch:
                sl = slots[c % 2]
                n = min(C, per - c * C)
                s_h2d.wait_event(ev_free[c % 2])
                with torch.cuda.stream(s_h2d):
                    sl["d_in"][: n * slot_bytes].copy_(
                        h_in[c * C * slot_bytes:(c * C + n) * slot_bytes], non_blocking=True)
                    sl["d_len"][:n].copy_(h_len[c * C:c * C + n], non_blocking=True)
                    ev_h2d[c % 2].record(s_h2d)
                s_comp.wait_event(ev_h2d[c % 2])
                lsmgpu.decode_into(ctx, g, sl["d_in"], d_off[:n], sl["d_len"][:n], sl["r"],
                                   stream=s_comp)
                lsmgpu.compact_into(ctx, g, d_off[:n], sl["r"], sl["dense"], stream=s_comp)
                with torch.cuda.stream(s_comp):
                    h_cnt[c:c + 1].copy_(sl["dense"].base[n:n + 1], non_blocking=True)
                    ev_comp[c % 2].record(s_comp)
            if c >= 1:
                p = c - 1
                sl = slots[p % 2]
                n = min(C, per - p * C)
                ev_comp[p % 2].synchronize()
                k = int(h_cnt[p])
                s_d2h.wait_event(ev_comp[p % 2])
                with torch.cuda.stream(s_d2h):
                    h_desc[pos:pos + k].copy_(sl["dense"].desc[:k], non_blocking=True)
                    h_meta[p, 0, :n].copy_(sl["r"].nrec[:n], non_blocking=True)
                    h_meta[p, 1, :n].copy_(sl["r"].status[:n], non_blocking=True)
                    ev_free[p % 2].record(s_d2h)
                pos += k
        s_d2h.synchronize()
        return pos

    for _ in range(max(1, args.warmup // 10)):
        nrec = run_once()
    assert nrec == per * 33 and int(h_meta[:, 1].abs().sum()) == 0
    torch.cuda.synchronize()
    barrier(world)
    t0 = time.perf_counter()
    steps = max(1, args.steps // 20)
    for _ in range(steps):
        run_once()
    torch.cuda.synchronize()
    barrier(world)
    elapsed = max_over_ranks(world, time.perf_counter() - t0)
    parsed = float(blk_len.astype(np.float64).sum())
    value = sum_over_ranks(world, parsed) * steps / elapsed / GIB
    h2d_bytes, d2h_bytes = per * slot_bytes, nrec * 16 + per * 8
    return {
        "metric": "GiB/s end-to-end: pinned host blocks -> H2D -> decode -> compact -> D2H records",
        "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": steps,
        "ms_per_step": round(elapsed * 1e3 / steps, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": f"decode {per} x 4 KiB KV blocks per GPU from host memory",
                   "chunk_blocks": C, "h2d_bytes": h2d_bytes, "d2h_bytes": d2h_bytes,
                   "pcie_GBps_h2d_equiv": round(h2d_bytes * steps / elapsed / 1e9, 2)},
    }


def cpu_baseline(args, data):
    """The oracle's Go-pattern decode (fresh heap buffer per key and value,
    append-grown slices; oracle/lsm_oracle.c) timed on this host's cores."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as ora

    buf, blk_off, blk_len = data
    threads = min(16, os.cpu_count() or 1)
    parsed = float(blk_len.astype(np.float64).sum())

    def timed(th, nb, budget):
        reps, t, recs = 0, 0.0, 0
        while t < budget or reps == 0:
            t0 = time.perf_counter()
            recs = ora.bench_decode_golike(ora.GRAMMAR_KV, buf, blk_off[:nb], blk_len[:nb], th)
            t += time.perf_counter() - t0
            reps += 1
        return reps, t, recs

    reps, t, recs = timed(threads, blk_off.size, args.cpu_seconds)
    v = parsed * reps / t / GIB
    nb1 = max(1, blk_off.size // 10)
    reps1, t1, _ = timed(1, nb1, args.cpu_seconds / 3)
    p1 = float(blk_len[:nb1].astype(np.float64).sum())
    return {
        "value": round(v, 3),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "sample": f"full workload ({blk_off.size} blocks, {recs} records) x {reps} passes "
                  f"in {t:.1f} s on {threads} threads; 1-thread: {nb1} blocks x {reps1} passes",
        "value_1t": round(p1 * reps1 / t1 / GIB, 3),
    }


def main():
    args = parse()
    world, rank, local = dist_setup(args)
    if args.e2e:
        out = bench_e2e(args, world, rank, local)
        if rank == 0:
            print(json.dumps(out), flush=True)
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return
    if args.config == "sst":
        from bench_sst import bench_sst  # encode path (config 3)
        out, data = bench_sst(args, world, rank, local)
    elif args.config in ("sstdec", "sstdec1"):
        from bench_sstdec import bench_sst_decode  # whole-.sst decode (§8(f) f1; config 1)
        out, data = bench_sst_decode(args, world, rank, local)
    elif args.config == "probe":
        from bench_sstdec import bench_may_contain  # batched MayContain (§8(f) f3)
        out, data = bench_may_contain(args, world, rank, local)
    elif args.config == "compact":
        from bench_compact import bench_compact  # L0 -> L1 compaction (§8(f) f1 + f2)
        out, data = bench_compact(args, world, rank, local)
    else:
        out, data = bench_decode(args, world, rank, local)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if args.config == "sst":
            from bench_sst import cpu_baseline_sst
            out["cpu_baseline"] = cpu_baseline_sst(args, data)
        elif args.config in ("sstdec", "sstdec1"):
            from bench_sstdec import cpu_baseline_sst_decode
            out["cpu_baseline"] = cpu_baseline_sst_decode(args, data)
        elif args.config == "probe":
            from bench_sstdec import cpu_baseline_may_contain
            out["cpu_baseline"] = cpu_baseline_may_contain(args, data)
        elif args.config == "compact":
            from bench_compact import cpu_baseline_compact
            out["cpu_baseline"] = cpu_baseline_compact(args, data)
        else:
            out["cpu_baseline"] = cpu_baseline(args, data)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
