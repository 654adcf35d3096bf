"""The N>1 device exchange on the GPU.

``shp_shard_partition_soa`` must be a stable split by key owner into SoA columns, and
``siddhi_amd.shard.DeviceExchange`` (bench.py's exchange: one all-to-all per column) must hand
each rank exactly the events of the keys it owns, in global arrival order.  The two-rank case
runs both ranks on cuda:0 with gloo collectives (the rehearsal mode of ``bench.py
--same-device``); each rank runs the HIP engine on what it received and rank 0 checks the union
of the ranks' matches against the single-process oracle run, per key, bit-exact.
"""
import ctypes
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

from diff_util import compare, per_key, program_for, run, small_stream  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("G,with_stream", [(2, False), (8, False), (3, True)])
def test_shard_partition_soa_is_stable(G, with_stream):
    import torch
    from siddhi_amd import native
    L = native.lib()
    n = 400_003
    g = small_stream(4, n, 1000)
    dev = torch.device("cuda", 0)
    ts = torch.from_numpy(g["ts"]).to(dev)
    key = torch.from_numpy(g["key"]).to(dev)
    price = torch.from_numpy(g["price"]).to(dev)
    stream = torch.from_numpy(g["stream"]).to(dev) if with_stream else None
    o_ts, o_key = torch.full((n,), -7, dtype=torch.int64, device=dev), torch.empty(n, dtype=torch.int32, device=dev)
    o_p = torch.empty(n, dtype=torch.float32, device=dev)
    o_s = torch.empty(n, dtype=torch.int32, device=dev) if with_stream else None
    ws = torch.empty(int(L.shp_shard_workspace_bytes(n, G)), dtype=torch.uint8, device=dev)
    counts = (ctypes.c_int64 * G)()
    assert L.shp_shard_partition_soa(n, ts.data_ptr(), key.data_ptr(), price.data_ptr(),
                                     stream.data_ptr() if with_stream else None, G, o_ts.data_ptr(),
                                     o_key.data_ptr(), o_p.data_ptr(), o_s.data_ptr() if with_stream else None,
                                     counts, ws.data_ptr(), None) == 0
    torch.cuda.synchronize()
    dst = g["key"] % G
    order = np.argsort(dst, kind="stable")
    assert list(counts) == [int((dst == r).sum()) for r in range(G)]
    assert (o_ts.cpu().numpy() == g["ts"][order]).all()
    assert (o_key.cpu().numpy() == (g["key"] // G)[order]).all()
    assert (o_p.cpu().numpy().view(np.uint32) == g["price"][order].view(np.uint32)).all()
    if with_stream:
        assert (o_s.cpu().numpy() == g["stream"][order]).all()
    # a missing output column for a present input column is an argument error, not a fault
    assert L.shp_shard_partition_soa(n, ts.data_ptr(), key.data_ptr(), price.data_ptr(), None, G, o_ts.data_ptr(),
                                     o_key.data_ptr(), None, None, counts, ws.data_ptr(), None) == -1


def _worker(rank, world, port, n, keys, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from siddhi_amd import shard
        from siddhi_amd.native import HipEngine
        g = small_stream(2, n, keys)
        dev = torch.device("cuda", 0)
        xch = shard.DeviceExchange(n, world, dist, dev, False, cpu_collectives=True)
        cq = program_for(2)
        kl = -(-keys // world)
        eng = HipEngine(cq.program_json(), 0, max_keys=kl, max_batch=n, max_matches=n)
        # two batches per rank: the ranks' slices of each batch are consecutive pieces of the stream
        half = n // 2
        out = []
        for b in range(2):
            lo_b = b * half
            hi_b = n if b == 1 else half
            lo = lo_b + rank * (hi_b - lo_b) // world
            hi = lo_b + (rank + 1) * (hi_b - lo_b) // world
            cols = [torch.from_numpy(g[c][lo:hi].copy()).to(dev) for c in ("ts", "key", "price")]
            ts, key, price, stream = xch(*cols)
            assert stream is None
            # global sequence numbers of the received events: by source rank, then arrival
            gseq = []
            for src in range(world):
                s_lo = lo_b + src * (hi_b - lo_b) // world
                s_hi = lo_b + (src + 1) * (hi_b - lo_b) // world
                idx = np.arange(s_lo, s_hi)
                gseq.append(idx[g["key"][s_lo:s_hi] % world == rank])
            gseq = np.concatenate(gseq)
            t, k, p = ts.cpu().numpy(), key.cpu().numpy(), price.cpu().numpy()
            assert (t == g["ts"][gseq]).all() and (k == g["key"][gseq] // world).all()
            eng.push(t, k, np.zeros(len(t), np.int32), [p], [None])
            mb = eng.fetch()
            out.append((mb, gseq))
        # local sequence numbers (running over the pushes) -> global ones
        allseq = np.concatenate([s for _, s in out])
        res = {}
        for mb, _ in out:
            mb["refs"] = allseq[mb["refs"]]
            mb["pos"] = allseq[mb["pos"]]
            mb["key"] = (mb["key"].astype(np.int64) * world + rank).astype(np.int32)
            for kk, v in per_key(mb).items():
                res.setdefault(kk, []).extend(v)
        eng.close()
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


def test_device_exchange_two_ranks_match_single_process():
    import torch.multiprocessing as mp
    from oracle.oracle import OracleEngine
    from test_shard_gloo import _free_port
    n, keys = 200_000, 600  # 300 keys per rank: the sweep path
    cq = program_for(2)
    ref = per_key(run(OracleEngine(cq.program_json(), 0), cq, small_stream(2, n, keys)))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n, keys, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        got = q.get(timeout=100)
    finally:
        for p in procs:
            p.join(timeout=30)
    assert all(p.exitcode == 0 for p in procs)
    assert sum(len(v) for v in ref.values()) > 10_000
    msg = compare(ref, got)
    assert msg is None, msg
