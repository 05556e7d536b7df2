#!/usr/bin/env python3
"""Benchmark of the gfx950 go-lsm block codec (BASELINE.json metric).

Default workload (N=1): BASELINE config 2 -- batch-decode 100,000 synthetic
4 KiB KV blocks (33 records of 16 B keys / 100 B values, 4,092 parsed bytes
per 4,096-byte slot), device resident, descriptor output.  One step = one
lsm_decode_blocks launch over the whole batch.

N>1 (one process per GPU): BASELINE config 4 -- a fixed global batch of
1,000,000 blocks dealt round-robin (block i -> rank i mod N; strong scaling,
`--global-blocks` sets the batch, `--blocks` switches to a per-GPU batch and
weak scaling).  No data-path collective: the ranks only meet at the barriers
around the timed region and in two scalar reductions.  Launched by the driver
under torch.distributed.run; a plain `python bench.py --gpus N` starts that
launcher itself as a child process before anything touches the GPU.

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

# lsmgpu (the HIP library) is imported by main() only after the launcher
# decision: a parent that spawns the rank processes never loads it.
lsmgpu = None
synth = None

CONFIG4_GLOBAL_BLOCKS = 1_000_000  # BASELINE.json configs[3]

METRIC = "GiB/s of device-resident .sst data-block bytes decoded to KV records"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, MI355X_MICROARCH.md
GIB = float(1 << 30)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="decode4k",
                    choices=["decode4k", "decode64k", "mixed", "sst", "sstdec", "sstdec1", "wal",
                             "probe", "level", "get", "get0", "compact"])
    ap.add_argument("--blocks", type=int, default=None, help="blocks per GPU (weak scaling)")
    ap.add_argument("--global-blocks", type=int, default=None,
                    help="fixed global batch dealt round-robin over the ranks (strong "
                         "scaling); default %d for decode4k at N>1 (config 4)"
                         % CONFIG4_GLOBAL_BLOCKS)
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher and deal only (gloo, no device work): prints the deal")
    ap.add_argument("--arena", action="store_true", help="materialize keys/values too")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--placement", default="offset", choices=["offset", "plan"],
                    help="decode output placement: offset-addressed (no plan) or dense "
                         "(lsm_plan_* inside every step)")
    ap.add_argument("--no-cold", action="store_true",
                    help="skip the cold-input pass (input rotated over copies the MALL cannot hold)")
    ap.add_argument("--no-verify", action="store_true",
                    help="skip the post-timing output check (diagnostic library variants only)")
    ap.add_argument("--e2e", action="store_true",
                    help="host-resident blocks: pinned H2D -> decode -> compact -> D2H "
                         "(the PCIe-inclusive rate recorded in DESIGN.md; not the headline)")
    ap.add_argument("--chunk", type=int, default=8192, help="blocks per e2e pipeline chunk")
    ap.add_argument("--get-tree", default="on", choices=["on", "off"],
                    help="--config get: Seek through the level's Seek tree "
                         "(lsm_level_get_tree_build, built once with the level), or by "
                         "bisecting the decoded index itself")
    ap.add_argument("--tie", default="input", choices=["input", "goheap"],
                    help="--config compact: equal keys in input order (LSM_TIE_INPUT) or in "
                         "container/heap's pop order, the reference's exact output (LSM_TIE_GOHEAP)")
    return ap.parse_args(argv)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args, argv):
    """`python bench.py --gpus N` without a launcher around it: start N rank
    processes under torch.distributed.run as a CHILD (this process has not
    touched the GPU and never does), pass rank 0's JSON line through, and
    return the child's exit code."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)
    return subprocess.call(cmd)


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: "
                         "launch one process per GPU (torch.distributed.run) or omit WORLD_SIZE")
    if args.dry_run:
        if world > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo")
        return world, rank, local
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


def gather_over_ranks(world, x):
    """[x of rank 0, x of rank 1, ...] (a scalar per rank; world 1: [x])."""
    if world == 1:
        return [x]
    import torch.distributed as dist
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    parts = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return [float(p.item()) for p in parts]


def aggregate_roofline(world, alg, kern_ms):
    """N > 1: the job's roofline -- the algorithmic bytes of every rank's
    launch over the slowest rank's kernel time, against N x the peak -- and
    the per-rank kernel times it comes from."""
    algs = gather_over_ranks(world, float(alg))
    kms = gather_over_ranks(world, float(kern_ms))
    ach = sum(algs) / (max(kms) * 1e-3) / 1e9
    return {"achieved": round(ach, 1), "peak": HBM_PEAK_GBS * world, "unit": "GB/s",
            "frac": round(ach / (HBM_PEAK_GBS * world), 4),
            "alg_bytes_per_launch": int(sum(algs)), "kernel_ms_max": round(max(kms), 5),
            "kernel_ms_per_rank": [round(x, 5) for x in kms],
            "def": "sum of the ranks' algorithmic bytes / max-over-ranks kernel time / (N x peak)"}


def shard_block_ids(rank, world, per):
    """Round-robin deal of a global batch of N x per blocks: block i -> rank i mod N."""
    return rank + world * np.arange(per, dtype=np.int64)


def deal_global(rank, world, total):
    """Round-robin deal of a fixed global batch of `total` blocks (config 4):
    rank r gets blocks r, r+N, r+2N, ... < total."""
    return np.arange(rank, total, world, dtype=np.int64)


def block_ids_for(args, world, rank):
    """This rank's global block ids and the scaling mode of the line."""
    per_default = 100_000 if args.config == "decode4k" else 6_400
    total = args.global_blocks
    if total is None and args.blocks is None and world > 1 and args.config == "decode4k":
        total = CONFIG4_GLOBAL_BLOCKS
    if total is not None:
        return deal_global(rank, world, total), "strong", total
    per = args.blocks or per_default
    return shard_block_ids(rank, world, per), "weak", per * world


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


UNIFORM = {"decode4k": dict(recs=33, slot=4096), "decode64k": dict(recs=528, slot=65536)}


def make_workload(args, world, rank):
    if args.config in ("decode4k", "decode64k"):
        ids, scaling, total = block_ids_for(args, world, rank)
        shape = UNIFORM[args.config]
        # 4 KiB: 33 x 124 B = 4,092 parsed bytes; 64 KiB: 528 x 124 B = 65,472
        buf, off, ln = synth.uniform_kv_blocks(ids, **shape)
        kib = shape["slot"] // 1024
        if scaling == "strong":
            desc = (f"decode {total} x {kib} KiB KV blocks ({shape['recs']} x 16 B key / 100 B "
                    f"value) dealt round-robin over {world} GPU(s)")
        else:
            desc = (f"decode {ids.size} x {kib} KiB KV blocks per GPU ({shape['recs']} x 16 B "
                    "key / 100 B value)")
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
    if args.placement == "plan":
        # dense outputs: the plan (exclusive scans of blk_len) is part of
        # every step, as for a batch whose layout is new each time
        plan = lsmgpu.plan(ctx, lsmgpu.GRAMMAR_KV, d_len, arena=args.arena)
        r = lsmgpu.alloc_decode(ctx, lsmgpu.GRAMMAR_KV, nblk, plan, arena=args.arena)
    else:
        plan = None
        r = lsmgpu.alloc_decode_offset(ctx, lsmgpu.GRAMMAR_KV, nblk, int(d_in.numel()),
                                       arena=args.arena)
    args._d_in = d_in
    stream = torch.cuda.current_stream()

    wal_max = int(blk_len.max()) if args.config == "wal" else 0
    wal_ws = lsmgpu.wal_workspace(ctx, nblk, wal_max) if args.config == "wal" else None
    # a batch of mixed block sizes goes through lsm_decode_blocks_scheduled
    # (largest first, the bucketing inside every timed call)
    sched = lsmgpu.schedule_workspace(ctx, nblk) if args.config == "mixed" else None
    # uniform batches: the block size the workload is built with, as a caller
    # that configures its block size passes it (lsm_decode_blocks_hinted)
    hint = UNIFORM[args.config]["slot"] if args.config in UNIFORM else None

    def step():
        if args.config == "wal":
            lsmgpu.wal_replay_into(ctx, d_in, d_off, d_len, wal_max, r, wal_ws, stream=stream)
        else:
            if plan is not None:
                lsmgpu.replan(ctx, lsmgpu.GRAMMAR_KV, d_len, plan, stream=stream)
            lsmgpu.decode_into(ctx, lsmgpu.GRAMMAR_KV, d_in, d_off, d_len, r, stream=stream,
                               schedule=sched, max_blk_len=hint)

    for _ in range(args.warmup):
        step()
    # no host read-back between the warm-up and t0 (only the contract's own
    # synchronize): the GPU idles for microseconds, not for the milliseconds
    # of two extra host round trips (profiles/r04_ktrace_driver.txt); the
    # output is checked after the timed region
    elapsed = timed_region(world, step, args.steps)
    # correctness gate on the timed output: every block decoded cleanly
    assert int((r.status[:nblk] != 0).sum()) == 0, "decode reported errors"
    nrec_total = int(r.nrec[:nblk].sum().item())
    # kernel time from HIP events, in passes of their own: an event pair
    # around every launch puts a ~10 us marker gap between launches
    # (profiles/r03_ktrace_events.txt), so the wall-timed loop has none
    times, kern_ms = kernel_times(step, stream, args.steps)
    # the timed output is checked after the timed region: the line fails on a
    # single wrong descriptor (kv/kv.go:77-115 record chain, closed form)
    verify_decode(args, r, d_off, d_len, nblk)

    parsed = float(blk_len.astype(np.float64).sum())
    cold = (cold_input_pass(args, ctx, buf, d_off, d_len, nblk, hint, stream, parsed)
            if args.config in UNIFORM and not args.no_cold and args.placement == "offset" else None)
    parsed_all = sum_over_ranks(world, parsed)
    value = parsed_all * args.steps / elapsed / GIB
    scaling = block_ids_for(args, world, rank)[1] if args.config in UNIFORM else "weak"

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
    if args.config == "mixed":
        # the FETCH_SIZE x 2 correction is not calibrated for this access
        # pattern (it read below the algorithmic bytes): no figure
        traffic, tsrc = None, "not calibrated for the scheduled mixed-size pattern (DESIGN.md §7)"
    if cold is not None:
        cold["frac"] = round(alg / (cold["kernel_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 5),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seed 0x5EED, keys k%015d, splitmix64 values)",
        "verified": "every record descriptor, nrec and status of the timed output (closed form)",
        "config": {
            "workload": wdesc,
            "grammar": "KV (kv/kv.go:46-115)",
            "output": "ARENA (descriptors + packed keys/values)" if args.arena else
                      "DESC (16 B record descriptors)",
            "blocks_per_gpu": int(nblk),
            "records_per_gpu": nrec_total,
            "parsed_bytes_per_gpu": int(parsed),
            "parallelism": (f"dp{world} (logs per rank, no collective)" if args.config == "wal" else
                            f"dp{world} (blocks round-robin, no collective)"),
            **({"scaling_note": "weak, per-rank copy: every rank replays its own log set"}
               if args.config == "wal" else {}),
        },
        "roofline": {
            "bound": "hbm",
            "kernel": decode_kernel_label(args),
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_source": tsrc,
            "alg_bytes_per_launch": int(alg),
            "kernel_ms": round(kern_ms, 5),
            "kernel_ms_source": KERNEL_MS_SOURCE,
            "kernel_ms_median": round(float(np.median(times)), 5),
            "kernel_ms_min": round(float(times.min()), 5),
        },
    }
    if cold is not None:
        out["cold_input"] = cold
    if world > 1:
        out["roofline"]["aggregate"] = aggregate_roofline(world, alg, kern_ms)
    return out, (buf, blk_off, blk_len)


def cold_input_pass(args, ctx, buf, d_off, d_len, nblk, hint, stream, parsed, copies=None):
    """The same decode with input the Infinity Cache (MALL, 256 MB) cannot
    hold: K launches rotating over `copies` distinct copies of the batch, each
    with its own outputs (8 x 409.6 MB for config 2), so every launch reads
    blocks no launch has read for copies - 1 launches.  The steady-state line
    above re-decodes one batch, part of which stays resident in the MALL
    between launches (tools/mall_probe.py: 78.5 us resident vs 86.1 us with
    10 rotating copies).  Event-timed over the whole pass; every copy's
    output is checked."""
    dev = ctx.torch_device
    if copies is None:  # >= 3.2 GB of input in rotation (2 copies of a GB-scale batch)
        batch = nblk * UNIFORM[args.config]["slot"]
        copies = int(min(8, max(2, -(-3_200_000_000 // batch))))
    ins = [args._d_in] + [lsmgpu.to_device_bytes(buf, dev) for _ in range(copies - 1)]
    outs = [lsmgpu.alloc_decode_offset(ctx, lsmgpu.GRAMMAR_KV, nblk, int(ins[0].numel()),
                                       arena=args.arena) for _ in range(copies)]
    k = max(args.steps, 2 * copies)

    def run():
        for i in range(k):
            lsmgpu.decode_into(ctx, lsmgpu.GRAMMAR_KV, ins[i % copies], d_off, d_len,
                               outs[i % copies], stream=stream, max_blk_len=hint)

    run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(stream)
    run()
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / k
    for r in outs:
        assert int((r.status[:nblk] != 0).sum()) == 0, "cold pass: decode reported errors"
        assert int(r.nrec[:nblk].sum()) == UNIFORM[args.config]["recs"] * nblk, "cold pass: nrec"
    del ins, outs
    torch.cuda.empty_cache()
    return {"copies": copies, "input_bytes": int(copies * nblk * UNIFORM[args.config]["slot"]),
            "launches": k, "kernel_ms": round(ms, 5),
            "value": round(parsed / (ms * 1e-3) / GIB, 2), "unit": "GiB/s"}


def decode_kernel_label(args):
    """The kernel (instantiation) a decode line times, from config and output
    mode together."""
    if args.config == "wal":
        return "lsm_wal_replay (seg + stitch + compact launches)"
    arena = ",ARENA" if args.arena else ""
    if args.config == "mixed":
        return ("lsm_decode_blocks_scheduled (size-class bucketing + "
                f"decode_v2_kernel<KV,2{arena}>, all launches)")
    if args.config == "decode64k":
        return f"decode_v2_kernel<KV,16{arena}> (lsm_decode_blocks_hinted)"
    return f"decode_v2_kernel<KV,8{arena}>"


KERNEL_MS_SOURCE = ("HIP events around K back-to-back launches on the launch stream "
                    "(a pass of its own); median / min from per-launch event pairs")


def timed_region(world, step, steps):
    """The driver contract's timed region: barrier + synchronize, exactly
    `steps` steps, synchronize; t1 is read before the trailing barrier (rank
    skew would otherwise be charged to every rank), the max over ranks is the
    elapsed time.  Nothing else is enqueued inside it."""
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier(world)
    return max_over_ranks(world, t1 - t0)


def kernel_times(step, stream, steps):
    """Average launch duration from one event pair around `steps` back-to-back
    launches (no marker between them, as in the timed region), and per-launch
    event pairs in a second pass for the median and minimum.
    -> (per-launch ms array, mean ms)."""
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(stream)
    for _ in range(steps):
        step()
    e1.record(stream)
    torch.cuda.synchronize()
    mean = e0.elapsed_time(e1) / steps
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(steps)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(steps)]
    for i in range(steps):
        starts[i].record(stream)
        step()
        ends[i].record(stream)
    torch.cuda.synchronize()
    return np.array([s.elapsed_time(e) for s, e in zip(starts, ends)]), mean


def verify_decode(args, r, d_off, d_len, nblk):
    """Check the decode output the timed region produced, on the device.

    For every block: status 0, records chained back to back from blk_off
    (record j+1 starts where record j ends: 8 + klen + vlen bytes later,
    kv/kv.go:77-115), the chain ending exactly at blk_off + blk_len.  For the
    uniform configs also the closed form: nrec, klen = 16, vlen = 100, record j
    at blk_off + 124 j.  WAL replay output is dense per log (checked the same
    way through its own nrec)."""
    if args.config == "wal":
        return
    dev = r.nrec.device
    nrec = r.nrec[:nblk].to(torch.int64)
    assert int((r.status[:nblk] != 0).sum()) == 0, "decode reported errors"
    off = d_off.to(torch.int64)
    ln = d_len.to(torch.int64) & 0xFFFFFFFF
    # each block's first record slot: the dense plan's rec_base (--placement
    # plan), else offset addressing
    base = (r.rec_base[:nblk].to(torch.int64) if r.rec_base is not None
            else off // lsmgpu.codec.MIN_RECORD[lsmgpu.GRAMMAR_KV])
    abase = (r.arena_base[:nblk].to(torch.int64) if r.arena_base is not None else off)
    chunk = 1 << 16
    for b0 in range(0, nblk, chunk):
        b1 = min(nblk, b0 + chunk)
        n = nrec[b0:b1]
        tot = int(n.sum())
        blk = torch.repeat_interleave(torch.arange(b0, b1, device=dev), n)
        first = torch.cumsum(n, 0) - n
        j = torch.arange(tot, device=dev) - torch.repeat_interleave(first, n)
        slot = base[blk] + j
        d = r.desc[slot].to(torch.int64)
        rec_off = (d[:, 0] & 0xFFFFFFFF) | (d[:, 1] << 32)
        klen, vlen = d[:, 2] & 0xFFFFFFFF, d[:, 3] & 0xFFFFFFFF
        end = rec_off + 8 + klen + vlen
        # chain: first record at blk_off, each next one at the previous end
        starts_ok = torch.where(j == 0, rec_off == off[blk],
                                rec_off == torch.roll(end, 1))
        assert bool(starts_ok.all()), "decode: record chain broken"
        last = torch.cumsum(n, 0) - 1
        nz = n > 0
        assert bool((end[last[nz]] == (off[b0:b1] + ln[b0:b1])[nz]).all()), \
            "decode: chain does not end at blk_off + blk_len"
        assert bool((ln[b0:b1][~nz] == 0).all()), "decode: empty output for a non-empty block"
        if args.config in UNIFORM:
            recs = UNIFORM[args.config]["recs"]
            assert bool((n == recs).all()), "decode: nrec"
            if getattr(args, "arena", False) and r.key_arena is not None:
                # ARENA: block b's keys / values packed at its arena base
                # (blk_off[b], or the plan's arena_base), equal to the record
                # fields of the input (kv.go:88-111 make + ReadFull)
                slot = UNIFORM[args.config]["slot"]
                ka = abase[b0:b1].unsqueeze(1) + torch.arange(recs * 16, device=dev)
                rows = r.key_arena[ka]
                recs_in = args._d_in[: nblk * slot].view(nblk, slot)[b0:b1, : recs * 124]
                recs_in = recs_in.reshape(b1 - b0, recs, 124)
                assert torch.equal(rows.reshape(b1 - b0, recs, 16),
                                   recs_in[:, :, 4:20]), "arena: keys"
                va = abase[b0:b1].unsqueeze(1) + torch.arange(recs * 100, device=dev)
                vrows = r.val_arena[va]
                assert torch.equal(vrows.reshape(b1 - b0, recs, 100),
                                   recs_in[:, :, 24:124]), "arena: values"
            assert bool(((klen == 16) & (vlen == 100)).all()), "decode: record lengths"
            assert bool((rec_off == off[blk] + 124 * j).all()), "decode: record offsets"



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
    t1 = time.perf_counter()
    barrier(world)
    elapsed = max_over_ranks(world, t1 - t0)
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


def host_cpu():
    """The host cores a CPU baseline may use, and what they are.

    On the GPU box `nproc` / os.cpu_count() report the whole machine while the
    job's CPU share is OMP_NUM_THREADS (16 per GPU); the baselines use that
    share (capped by the affinity mask) and record all three numbers."""
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    share = int(os.environ.get("OMP_NUM_THREADS") or 0) or affinity
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"threads": max(1, min(share, affinity)), "nproc": os.cpu_count(),
            "affinity": affinity, "model": model}


def timed_threads(fn, items, threads, budget):
    """Run fn(item) over items on `threads` host threads (ctypes releases the
    GIL, so the C restatement runs in parallel), repeating whole passes until
    `budget` seconds have passed.  -> (passes, seconds)."""
    from concurrent.futures import ThreadPoolExecutor
    passes, t = 0, 0.0
    with ThreadPoolExecutor(max_workers=threads) as ex:
        while t < budget or passes == 0:
            t0 = time.perf_counter()
            list(ex.map(fn, items))
            t += time.perf_counter() - t0
            passes += 1
    return passes, t


def cpu_baseline(args, data):
    """The oracle's Go-pattern decode (fresh heap buffer per key and value,
    append-grown slices; oracle/lsm_oracle.c) timed on this host's cores."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as ora

    buf, blk_off, blk_len = data
    cpu = host_cpu()
    threads = cpu["threads"]
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
        "host": cpu,
    }


def dry_run(args, world, rank):
    """--dry-run: the launcher and the deal without device work (CPU, gloo).
    Rank 0 prints the deal: blocks per rank and checksums of the dealt ids."""
    recs = 0
    if args.config in UNIFORM:
        ids, scaling, total = block_ids_for(args, world, rank)
    elif args.config == "sst":
        # config 3's deal: whole .sst files of one stream, file f -> rank f mod N
        from bench_sst import sst_deal
        batch, starts, ids, total, _ = sst_deal(args, world, rank)
        scaling, recs = "strong", int(starts[-1])
    else:
        ids, scaling, total = np.arange(rank, rank + 1, dtype=np.int64), "weak", world
    assert bool((ids % world == rank).all())
    recs_all = gather_over_ranks(world, float(recs))
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([ids.size, int(ids.sum()), int((ids.astype(np.float64) ** 2).sum())],
                         dtype=torch.float64)
        parts = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(parts, t)
        rows = [p.tolist() for p in parts]
    else:
        rows = [[ids.size, int(ids.sum()), float((ids.astype(np.float64) ** 2).sum())]]
    return {"dry_run": True, "n_gpus": world, "config": args.config, "scaling": scaling,
            "global_blocks": total, "blocks_per_rank": [int(r[0]) for r in rows],
            "id_sum": int(sum(r[1] for r in rows)), "id_sumsq": float(sum(r[2] for r in rows)),
            "records_per_rank": [int(x) for x in recs_all], "pid": os.getpid()}


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args, argv))
    world, rank, local = dist_setup(args)
    if args.dry_run:
        out = dry_run(args, world, rank)
        if rank == 0:
            print(json.dumps(out), flush=True)
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return
    global lsmgpu, synth
    import lsmgpu as _lsmgpu
    lsmgpu, synth = _lsmgpu, _lsmgpu.synth
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
    elif args.config in ("level", "get"):
        # level search, reference shape (§8(f) f3); get: + Seek + value
        from bench_sstdec import bench_level_search
        out, data = bench_level_search(args, world, rank, local)
    elif args.config == "get0":
        # level 0's Get (§8(f) f3): every table in order (searchFromLevel0)
        from bench_sstdec import bench_level0_get
        out, data = bench_level0_get(args, world, rank, local)
    elif args.config == "compact":
        from bench_compact import bench_compact  # L0 -> L1 compaction (§8(f) f1 + f2)
        out, data = bench_compact(args, world, rank, local)
    else:
        out, data = bench_decode(args, world, rank, local)
    # the CPU baseline on rank 0, after every rank's timed region (at N > 1
    # over rank 0's shard: the same sample shape as at N = 1)
    if rank == 0 and not args.no_cpu_baseline:
        if args.config == "sst":
            from bench_sst import cpu_baseline_sst
            out["cpu_baseline"] = cpu_baseline_sst(args, data)
        elif args.config in ("sstdec", "sstdec1"):
            from bench_sstdec import cpu_baseline_sst_decode
            out["cpu_baseline"] = cpu_baseline_sst_decode(args, data)
        elif args.config == "probe":
            from bench_sstdec import cpu_baseline_may_contain
            out["cpu_baseline"] = cpu_baseline_may_contain(args, data)
        elif args.config in ("level", "get"):
            from bench_sstdec import cpu_baseline_level_search
            out["cpu_baseline"] = cpu_baseline_level_search(args, data)
        elif args.config == "get0":
            from bench_sstdec import cpu_baseline_level0_get
            out["cpu_baseline"] = cpu_baseline_level0_get(args, data)
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
