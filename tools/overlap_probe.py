#!/usr/bin/env python3
"""Does the N>1 exchange split overlap the engine on one GPU?  Times, for C2 at the per-rank key
count of an N=8 job (1250 keys, 100M events): the engine push alone, the exchange split alone
(G=8), and both at once (push on a worker thread, as bench.py does).  Prints one JSON line."""
import ctypes
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from siddhi_amd import native, synth
    from siddhi_amd.query.compiler import compile_app
    L = native.lib()
    N, K, G = 100_000_000, 1250, 8
    _, qs, _ = compile_app(synth.QUERIES[2])
    cq = qs[0]
    eng = native.HipEngine(cq.program_json(), 0, max_keys=K, max_batch=N, max_matches=N,
                           match_layout=native.LAYOUT_PAIRS)
    dev = torch.device("cuda", 0)

    def gen(b):
        ts = torch.empty(N, dtype=torch.int64, device=dev)
        key = torch.empty(N, dtype=torch.int32, device=dev)
        price = torch.empty(N, dtype=torch.float32, device=dev)
        assert L.shp_synth_fill(2, b * N, N, K, 1, 0, ts.data_ptr(), key.data_ptr(), price.data_ptr(),
                                None, None, None) == 0
        return ts, key, price

    bs = [gen(b) for b in range(8)]
    x = gen(9)
    torch.cuda.synchronize()
    ws = torch.empty(int(L.shp_shard_workspace_bytes(N, G)), dtype=torch.uint8, device=dev)
    o = [torch.empty(N, dtype=d, device=dev) for d in (torch.int64, torch.int32, torch.float32)]
    counts = (ctypes.c_int64 * G)()
    cur = torch.cuda.current_stream().cuda_stream

    def push(b):
        ts, key, price = bs[b]
        colp = (ctypes.c_void_p * 1)(price.data_ptr())
        bt = native.ShpBatch(N, ts.data_ptr(), key.data_ptr(), None, ctypes.cast(colp, ctypes.c_void_p), None)
        mt = native.ShpMatches()
        assert L.shp_push_batch_device(eng.h, ctypes.byref(bt), ctypes.byref(mt)) == 0

    def split():
        assert L.shp_shard_partition_soa(N, x[0].data_ptr(), x[1].data_ptr(), x[2].data_ptr(), None, G,
                                         o[0].data_ptr(), o[1].data_ptr(), o[2].data_ptr(), None, counts,
                                         ws.data_ptr(), cur) == 0

    def tm(fn):
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) * 1e3

    push(0)
    split()
    res = {"push_ms": [], "split_ms": [], "both_ms": []}
    for b in range(1, 7, 2):
        res["push_ms"].append(tm(lambda: push(b)))
        res["split_ms"].append(tm(split))

        def both():
            th = threading.Thread(target=push, args=(b + 1,))
            th.start()
            split()
            th.join()
        res["both_ms"].append(tm(both))
    print(json.dumps({k: min(v) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
