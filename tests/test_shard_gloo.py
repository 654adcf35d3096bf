"""The N>1 path on CPU: key-owner sharding over a world-size-2 gloo group.

Each rank ingests its half of a C2-shaped stream, the halves are exchanged by
key owner with ``siddhi_amd.shard.exchange`` (the function bench.py uses over RCCL), and each
rank runs the state machine on the keys it owns — here the CPU oracle stands in for the
per-rank engine.  Rank 0 checks that the union of the ranks' matches equals the single-process
run per key: same tuples (global event sequence numbers), same order.
"""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, keys, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from diff_util import per_key, program_for, small_stream
        from oracle.oracle import OracleEngine
        from siddhi_amd import shard
        g = small_stream(2, n, keys)
        lo, hi = rank * n // world, (rank + 1) * n // world
        cols = {"ts": torch.from_numpy(g["ts"][lo:hi].copy()), "key": torch.from_numpy(g["key"][lo:hi].copy()),
                "price": torch.from_numpy(g["price"][lo:hi].copy()),
                "gseq": torch.arange(lo, hi, dtype=torch.int64)}
        got = {k: v.numpy() for k, v in shard.exchange(cols, "key", world, dist).items()}
        assert (shard.owner_of(got["key"], world) == rank).all()
        cq = program_for(2)
        eng = OracleEngine(cq.program_json(), 0)
        m = len(got["ts"])
        eng.push(got["ts"], shard.local_key(got["key"], world).astype(np.int32), np.zeros(m, np.int32),
                 [got["price"]], [None])
        mb = eng.fetch()
        # local sequence numbers -> global ones; local key ids -> global keys
        mb["refs"] = got["gseq"][mb["refs"]]
        mb["pos"] = got["gseq"][mb["pos"]]
        mb["key"] = (mb["key"].astype(np.int64) * world + rank).astype(np.int32)
        res = per_key(mb)
        allres = [None] * world
        dist.all_gather_object(allres, res)
        if rank == 0:
            merged = {}
            for r in allres:
                assert not (set(r) & set(merged)), "a key was owned by two ranks"
                merged.update(r)
            q.put(merged)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_matches_equal_single_process(world):
    import torch.multiprocessing as mp
    sys.path[:0] = [os.path.join(ROOT, "tests")]
    from diff_util import compare, per_key, program_for, run, small_stream
    from oracle.oracle import OracleEngine
    n, keys = 30_000, 64
    cq = program_for(2)
    ref = per_key(run(OracleEngine(cq.program_json(), 0), cq, small_stream(2, n, keys)))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, keys, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        got = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert sum(len(v) for v in ref.values()) > 1000
    msg = compare(ref, got)
    assert msg is None, msg
