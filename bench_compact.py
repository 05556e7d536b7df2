"""Compaction bench (SURVEY.md §8(f) rows f1 + f2 + a9): `python bench.py
--config compact` runs go-lsm's level-0 -> level-1 compaction on the GPU
(compactLevel, compaction.go:75-133): decode every input .sst
(GetDataBlockFromFile, sstable.go:227-246) -> the positional join in file
order (loadLevelData, compaction.go:173-193) -> CompactAndMergeKVs
(merge.go:42-94) -> the new .sst images (Builder + EncodeTo).

Inputs per GPU (built on the GPU before timing): level 1 = the 208 config-3
files (3.3M sorted unique records, 16 B keys / 100 B values); level 0 = 8
memtable-sized files of updates (sorted, unique per file, newest first, one
in 16 a tombstone) spread over the whole key range, so every level-1 file
overlaps and is rewritten.  Secondary bench line; the headline is block decode.
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
L0_FILES = 8
L0_RECS = 15_888  # records of a 2 MiB memtable flush (README's 2.2 MB file)


def level0_ids(n1, first, rank, nfiles=L0_FILES, per=L0_RECS):
    """The key ids of the L0 flushes, newest file first."""
    rng = np.random.default_rng(synth.SEED + 77 + rank)
    return [np.unique(rng.integers(first, first + n1, per)) for _ in range(nfiles)]


def level0_runs(n1, first, rank, nfiles=L0_FILES, per=L0_RECS):
    """L0 flushes: sorted unique update keys inside level 1's key range;
    newest file first (go-lsm lists level-0 files newest first)."""
    runs = []
    for f, ids in enumerate(level0_ids(n1, first, rank, nfiles, per)):
        keys = synth.keys_for(ids).reshape(-1)
        vals = synth.value_bytes(ids + (f + 1) * 10 ** 9, synth.VAL_LEN).reshape(len(ids), -1)
        vlen = np.full(len(ids), synth.VAL_LEN, np.int64)
        tomb = (ids * 7 + f) % 16 == 0
        vbytes = [lsmgpu.TOMBSTONE if t else v.tobytes() for v, t in zip(vals, tomb)]
        vlen = np.array([len(v) for v in vbytes], np.int64)
        koff = np.arange(len(ids) + 1, dtype=np.uint64) * np.uint64(synth.KEY_LEN)
        voff = np.concatenate([[0], np.cumsum(vlen)]).astype(np.uint64)
        runs.append((keys, koff, np.frombuffer(b"".join(vbytes), np.uint8), voff))
    return runs


def build_images(ctx, runs):
    """Each run -> its .sst images (2 MiB flush), concatenated in run order."""
    parts, offs, sizes, base = [], [], [], 0
    for keys, koff, vals, voff in runs:
        batch = lsmgpu.batch_to_device(ctx, keys, koff, vals, voff)
        starts = lsmgpu.segment_files(ctx, koff, voff, lsmgpu.MAX_SSTABLE_SIZE)
        sb = lsmgpu.build_sst(ctx, batch, starts)
        parts.append(sb.out)
        offs.append(sb.file_off.astype(np.uint64) + np.uint64(base))
        sizes.append(sb.file_size.astype(np.uint64))
        base += int(sb.out.numel())
    torch.cuda.synchronize()
    return torch.cat(parts), np.concatenate(offs), np.concatenate(sizes)


def bench_compact(args, world, rank, local):
    from bench import barrier, max_over_ranks, sum_over_ranks, timed_region
    ctx = lsmgpu.Context(local)
    n1 = (args.blocks or 100_000) * 33
    first = rank * n1
    l1 = synth.kv_stream(n1, first=first)
    img, file_off, file_size = build_images(ctx, level0_runs(n1, first, rank) + [l1])
    nf_in = len(file_off)
    r = lsmgpu.alloc_sst_decode(ctx, file_off, file_size, int(img.numel()))
    lsmgpu.decode_sst_into(ctx, img, r)
    torch.cuda.synchronize()
    meta = r.meta_numpy()
    assert (meta["stage"] == 0).all(), "input decode failed"
    kd, vd, prefix = lsmgpu.sst_pairs(ctx, r)
    n = int(kd.shape[0])
    key_bytes = int(meta["idx_size"].astype(np.int64).sum())   # bounds the selected keys
    val_bytes = int(meta["data_size"].astype(np.int64).sum())  # and values
    mg = lsmgpu.alloc_merge(ctx, n)
    # LSM_TIE_INPUT: equal keys in input order (merge.go:41's contract, all on
    # the device); LSM_TIE_GOHEAP: container/heap's own pop order, the
    # reference's exact output (the heap's history replayed on one host thread)
    tie = lsmgpu.TIE_GOHEAP if getattr(args, "tie", "input") == "goheap" else lsmgpu.TIE_INPUT
    stream = torch.cuda.current_stream()
    ev_names = ("decode", "join", "merge", "gather", "build")
    keep = {}  # the gather's and the build's buffers, allocated by the first step
    # the merge's counts stay on the device (lsm_merge_kvs_async): the gather
    # runs on the device count while the host reads it (pinned, one event)
    d_counts = torch.zeros(3, dtype=torch.int64, device=ctx.torch_device)
    h_counts = torch.zeros(3, dtype=torch.int64, pin_memory=True)
    counted = torch.cuda.Event()

    def step(evs=None, tie=tie):
        def mark(i):
            if evs is not None:
                evs[i].record(stream)
        mark(0)
        lsmgpu.decode_sst_into(ctx, img, r, stream=stream)
        mark(1)
        lsmgpu.sst_pairs_into(ctx, r, kd, vd, prefix, stream=stream)
        mark(2)
        lsmgpu.merge_kvs_into(ctx, img, kd, vd, mg, level=1, stream=stream, d_counts=d_counts, tie=tie)
        h_counts.copy_(d_counts, non_blocking=True)
        counted.record(stream)
        mark(3)
        # keys packed; values read in place by the build (no second copy)
        batch = lsmgpu.gather_kvs(ctx, img, kd, vd, mg.out, n, key_bytes, None,
                                  stream=stream, reuse=keep.get("batch"), d_nout=d_counts)
        counted.synchronize()  # while the gather runs
        mg.nout, mg.nfiles, mg.max_recs = (int(x) for x in h_counts.tolist())
        batch.n = mg.nout
        mark(4)
        sb = lsmgpu.prepare_sst_device(ctx, batch, mg.file_start, mg.nfiles, mg.max_recs,
                                       val_bytes=val_bytes, stream=stream, reuse=keep.get("sb"))
        keep["batch"], keep["sb"] = batch, sb
        lsmgpu.build_sst_views_into(ctx, batch, sb, img, kd, vd, mg.out, stream=stream)
        mark(5)
        return sb, batch

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    steps = max(1, min(args.steps, 20))
    elapsed = timed_region(world, step, steps)
    # stage times from events in a pass of their own (markers between the
    # stages would add their gaps to the wall-timed region)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(6)] for _ in range(steps)]
    for s in range(steps):
        sb, batch = step(evs[s])
    torch.cuda.synchronize()
    stage_ms = {nm: float(np.mean([e[i].elapsed_time(e[i + 1]) for e in evs]))
                for i, nm in enumerate(ev_names)}
    goheap = None
    if tie == lsmgpu.TIE_GOHEAP:
        # what the exact tie order costs: the host replay alone on this
        # input's key ranks (the L0 and L1 key ids are their dense ranks),
        # and the merge stage against the input-order merge of the same run
        ids = np.concatenate(level0_ids(n1, first, rank) + [np.arange(first, first + n1)])
        ranks = (ids - first).astype(np.uint32)
        assert ranks.size == n
        rep, push, pop = [], [], []
        for _ in range(3):
            t0 = time.perf_counter()
            _, pu, po = lsmgpu.goheap_pop_order(ctx, ranks, phases=True)
            rep.append(time.perf_counter() - t0)
            push.append(pu)
            pop.append(po)
        evi = [[torch.cuda.Event(enable_timing=True) for _ in range(6)] for _ in range(3)]
        for s_ in range(3):
            step(evi[s_], tie=lsmgpu.TIE_INPUT)
        torch.cuda.synchronize()
        merge_in = float(np.mean([e[2].elapsed_time(e[3]) for e in evi]))
        goheap = {"replay_host_ms": round(min(rep) * 1e3, 2),
                  "replay_host_ms_mean": round(float(np.mean(rep)) * 1e3, 2),
                  "push_ms": round(float(np.median(push)), 2),
                  "pop_ms": round(float(np.median(pop)), 2),
                  "replays_in_timed_steps": int(ctx.lib.lsm_goheap_replays(ctx.handle)),
                  "merge_stage_ms": round(stage_ms["merge"], 3),
                  "merge_stage_input_order_ms": round(merge_in, 4),
                  "chain_ms": round(elapsed * 1e3 / steps, 3),
                  "note": "merge stage = device sort + equal-key flags + read-back of the sorted "
                          "order + host ranks and container/heap replay (one thread) + the order "
                          "back + the device group / flush / emit passes"}
    in_bytes = float(file_size.astype(np.float64).sum())
    total = sum_over_ranks(world, in_bytes)
    # the build stage (lsm_sst_layout + lsm_build_sst_views) moves the most
    # bytes: per written pair the packed key and its koff / voff (16 B), the
    # index (4 B) and value descriptor (16 B), the value bytes read, and every
    # image byte written
    key_b = float(batch.koff[mg.nout].item())
    val_b = float(batch.voff[mg.nout].item())
    build_alg = key_b + val_b + 36.0 * mg.nout + float(sb.file_size.astype(np.float64).sum())
    from bench import HBM_PEAK_GBS
    b_ach = build_alg / (stage_ms["build"] * 1e-3) / 1e9
    chain_alg = in_bytes + float(sb.file_size.astype(np.float64).sum())
    # HBM bytes of every kernel of one compaction (PMC, scripts/gpu_evidence.sh)
    from bench import traffic_from_profile
    traffic, tsrc = traffic_from_profile(f"compact:{nf_in}")
    out = {
        "metric": "GiB/s of input .sst bytes compacted (decode + merge + rebuild)",
        "value": round(total * steps / elapsed / GIB, 3),
        "unit": "GiB/s",
        "n_gpus": world, "steps": steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / steps, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic: level 1 = config-3 images, level 0 = 8 update flushes (1/16 tombstones)",
        "config": {"workload": f"compact {nf_in} .sst ({L0_FILES} L0 + {nf_in - L0_FILES} L1) -> "
                               f"{mg.nfiles} files per GPU ({n} pairs in, {mg.nout} out)",
                   "files_in": nf_in, "files_out": mg.nfiles, "pairs_in": n, "pairs_out": mg.nout,
                   "input_bytes_per_gpu": int(in_bytes),
                   "stage_ms": {k: round(v, 4) for k, v in stage_ms.items()},
                   "tie": ("goheap: container/heap's pop order for equal keys (the reference's "
                           "exact output)" if goheap else
                           "input: equal keys in input order (merge.go:41's contract)"),
                   "parallelism": f"dp{world} (one compaction per rank, no collective)",
                   "scaling_note": "weak, per-rank copy: every rank compacts its own copy-shaped input"},
        # the whole chain: an ideal compaction reads every input image byte
        # once and writes every output image byte once; everything between
        # (descriptors, the permutation, packed keys) is this implementation's
        # own traffic and counts against it
        "roofline": {"bound": "hbm",
                     "kernel": "whole compaction per step (decode + join + merge + gather + "
                               "build), wall time of the timed region",
                     "achieved": round(chain_alg / (elapsed / steps) / 1e9, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(chain_alg / (elapsed / steps) / 1e9 / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "traffic_source": tsrc,
                     "alg_bytes_per_launch": int(chain_alg),
                     "alg_bytes_def": "input image bytes read once + output image bytes written once",
                     "kernel_ms": round(elapsed * 1e3 / steps, 5),
                     "build_stage": {"kernel": "lsm_sst_layout + lsm_build_sst_views (events)",
                                     "alg_bytes": int(build_alg), "ms": round(stage_ms["build"], 5),
                                     "achieved": round(b_ach, 1),
                                     "frac": round(b_ach / HBM_PEAK_GBS, 4)}},
    }
    if goheap:
        out["goheap"] = goheap
    return out, (img.cpu().numpy(), file_off, file_size)


def cpu_baseline_compact(args, data):
    """The C restatement on a bounded sample: decode the 8 level-0 files and
    the first level-1 files (ora_sst_decode), merge (ora_merge_kvs, input-order
    ties) and build the output images (ora_build_sst), 1 thread."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as ora
    img, file_off, file_size = data
    nl1 = 6
    files = list(range(L0_FILES)) + list(range(L0_FILES, L0_FILES + nl1))
    t0 = time.perf_counter()
    kpos, klen, vpos, vlen, bufs, base = [], [], [], [], [], 0
    for f in files:
        o, n = int(file_off[f]), int(file_size[f])
        im = img[o:o + n]
        rc, meta, idesc, _, ddesc = ora.sst_decode(im)
        assert rc == 0
        kpos.append(idesc["rec_off"].astype(np.uint64) + np.uint64(4 + base))
        klen.append(idesc["key_len"].astype(np.uint32))
        vpos.append(ddesc["rec_off"].astype(np.uint64) + np.uint64(4 + base))
        vlen.append(ddesc["val_len"].astype(np.uint32))
        bufs.append(im)
        base += n
    buf = np.concatenate(bufs)
    kpos, klen = np.concatenate(kpos), np.concatenate(klen)
    vpos, vlen = np.concatenate(vpos), np.concatenate(vlen)
    goheap = getattr(args, "tie", "input") == "goheap"
    out, starts = ora.merge_kvs(buf, kpos, klen, vpos, vlen, 1, lsmgpu.MAX_SSTABLE_SIZE,
                                ora.TIE_GOHEAP if goheap else ora.TIE_INPUT)
    keys = np.concatenate([buf[int(kpos[i]):int(kpos[i]) + int(klen[i])] for i in out])
    vals = np.concatenate([buf[int(vpos[i]):int(vpos[i]) + int(vlen[i])] for i in out])
    koff = np.concatenate([[0], np.cumsum(klen[out].astype(np.uint64))]).astype(np.uint64)
    voff = np.concatenate([[0], np.cumsum(vlen[out].astype(np.uint64))]).astype(np.uint64)
    for f in range(len(starts) - 1):
        ora.build_sst(keys, koff, vals, voff, int(starts[f]), int(starts[f + 1]))
    t = time.perf_counter() - t0
    in_bytes = float(sum(int(file_size[f]) for f in files))
    return {"value": round(in_bytes / t / GIB, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"{len(files)} input files ({int(in_bytes)} B, {len(kpos)} pairs) -> "
                      f"{len(starts) - 1} files by the C restatement in {t:.1f} s (1 thread, "
                      f"Python-driven gathers; {'container/heap' if goheap else 'input-order'} ties)"}
