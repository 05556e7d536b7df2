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
