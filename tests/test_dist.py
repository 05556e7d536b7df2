"""CPU multi-process test of bench.py's N>1 host logic with gloo (world 2):
round-robin block dealing covers the global batch exactly once, the ranks
share nothing on the data path, and the barrier + max/sum reductions give the
whole-job numbers.  Decoding here uses the oracle (test infrastructure)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, per, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "go-lsm_amd"), os.path.join(ROOT, "oracle")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    import pyoracle as ora
    from lsmgpu import synth
    ids = bench.shard_block_ids(rank, world, per)
    buf, off, ln = synth.uniform_kv_blocks(ids)
    recs = ora.bench_decode_golike(ora.GRAMMAR_KV, buf, off, ln, 1)
    bench.barrier(world)
    tot_recs = bench.sum_over_ranks(world, float(recs))
    tot_bytes = bench.sum_over_ranks(world, float(ln.astype(np.float64).sum()))
    mx = bench.max_over_ranks(world, float(rank + 1))
    q.put((rank, ids.tolist(), recs, tot_recs, tot_bytes, mx))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_round_robin_shards_and_reductions(world):
    per = 50
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, per, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    ids = sorted(i for r in res for i in r[1])
    assert ids == list(range(world * per))          # every block exactly once
    for rank, rids, recs, tot_recs, tot_bytes, mx in res:
        assert all(i % world == rank for i in rids)  # block i -> rank i mod N
        assert recs == per * 33
        assert tot_recs == world * per * 33
        assert tot_bytes == world * per * 4092
        assert mx == world


def _bench_dry(*extra):
    """Run `python bench.py --dry-run ...` as the driver would (no WORLD_SIZE in
    the environment) and return rank 0's JSON line and the parent's pid."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.Popen([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", *extra],
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env, cwd=ROOT)
    out, err = p.communicate(timeout=240)
    assert p.returncode == 0, err.decode()[-2000:]
    lines = [ln for ln in out.decode().splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.decode()
    return json.loads(lines[0]), p.pid


def test_launcher_gpus2_deals_config4_exactly():
    """`bench.py --gpus 2` launches two rank processes itself (config 4: the
    fixed 1,000,000-block batch dealt round-robin, block i -> rank i mod 2)."""
    G = 1_000_000
    j, parent = _bench_dry("--gpus", "2")
    assert j["n_gpus"] == 2 and j["scaling"] == "strong" and j["global_blocks"] == G
    assert j["blocks_per_rank"] == [G // 2, G // 2]
    assert j["id_sum"] == G * (G - 1) // 2                       # every block once
    assert j["id_sumsq"] == float((G - 1) * G * (2 * G - 1) // 6)
    assert j["pid"] != parent                                     # rank 0 is a child


def test_launcher_uneven_deal_and_weak_mode():
    j, _ = _bench_dry("--gpus", "3", "--global-blocks", "10")
    assert j["blocks_per_rank"] == [4, 3, 3] and j["id_sum"] == 45 and j["id_sumsq"] == 285.0
    j, _ = _bench_dry("--gpus", "2", "--blocks", "50")
    assert j["scaling"] == "weak" and j["blocks_per_rank"] == [50, 50] and j["id_sum"] == 99 * 50
    j, _ = _bench_dry()
    assert j["n_gpus"] == 1 and j["global_blocks"] == 100_000    # N=1: config 2


def test_world_mismatch_is_refused():
    import subprocess
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run"],
                       capture_output=True, env=env, cwd=ROOT, timeout=120)
    assert p.returncode != 0 and b"WORLD_SIZE=2" in p.stderr


def test_launcher_gpus2_deals_sst_files_exactly():
    """`bench.py --config sst --gpus N`: config 3's stream is cut into .sst
    files by the builder rule and whole files are dealt round-robin (file f ->
    rank f mod N): every file exactly once, every record in
    exactly one rank's batch."""
    # 2,000 blocks x 33 records = 66,000 records of 132 B EstimateSize -> 5 files
    j, _ = _bench_dry("--config", "sst", "--gpus", "2", "--blocks", "2000")
    nf = j["global_blocks"]
    assert nf == 5 and j["scaling"] == "strong"
    assert j["blocks_per_rank"] == [3, 2]
    assert j["id_sum"] == nf * (nf - 1) // 2 and j["id_sumsq"] == float(sum(f * f for f in range(nf)))
    assert sum(j["records_per_rank"]) == 66_000
    last = 66_000 - 4 * 15888                                       # file 4: the partial one
    assert j["records_per_rank"] == [2 * 15888 + last, 2 * 15888]   # files 0, 2, 4 | 1, 3
    j, _ = _bench_dry("--config", "sst", "--gpus", "3", "--blocks", "2000")
    assert j["blocks_per_rank"] == [2, 2, 1] and sum(j["records_per_rank"]) == 66_000


def test_sst_deal_rule_rederives_each_ranks_files():
    """At N > 1 each rank's step runs the builder rule on the device over its
    own concatenation of dealt files (bench_sst.py).  That re-derives exactly
    the dealt files: every dealt file but the global last is full, the rule
    restarts at each file start, and the partial last file ends its rank's
    stream.  Checked here with the oracle's rule (ora_segment_files, the
    restatement of builder.go:34-42 the device rule is tested against)."""
    import argparse
    sys.path[:0] = [ROOT, os.path.join(ROOT, "go-lsm_amd"), os.path.join(ROOT, "oracle")]
    import bench_sst
    import lsmgpu
    import pyoracle as ora
    args = argparse.Namespace(blocks=2000)
    for world in (2, 3):
        seen = 0
        for rank in range(world):
            (keys, koff, vals, voff), starts, mine, nf, _ = bench_sst.sst_deal(args, world, rank)
            again = ora.segment_files(koff, voff, lsmgpu.MAX_SSTABLE_SIZE)
            assert np.array_equal(again.astype(np.int64), starts.astype(np.int64)), (world, rank)
            assert len(starts) - 1 == len(mine)
            seen += len(mine)
        assert seen == nf
