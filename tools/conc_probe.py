"""Concurrency probe (diagnostic): do two C2 engines pushing at once on one MI355X (two host threads,
each engine on its own streams) finish more events per second than one engine pushing alone?  An
upper bound for overlapping one push's owner partition with the previous push's solve."""
import ctypes
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from siddhi_amd import native, synth  # noqa: E402
from siddhi_amd.query.compiler import compile_app  # noqa: E402

N, K, REPS = 100_000_000, 10_000, 6
L = native.lib()
cq = compile_app(synth.QUERIES[2])[1][0]
spec = synth.StreamSpec(2, N, K, 1, False)


def gen(start):
    ts = torch.empty(N, dtype=torch.int64, device="cuda")
    key = torch.empty(N, dtype=torch.int32, device="cuda")
    price = torch.empty(N, dtype=torch.float32, device="cuda")
    assert L.shp_synth_fill(2, start, N, K, 1, 0, ts.data_ptr(), key.data_ptr(), price.data_ptr(), None, None, None) == 0
    return ts, key, price


def mk():
    return native.HipEngine(cq.program_json(), 0, max_keys=K, max_batch=N, max_matches=N,
                            match_layout=native.LAYOUT_PAIRS32)


def push(e, b):
    ts, key, price = b
    colp = (ctypes.c_void_p * 1)(price.data_ptr())
    bb = native.ShpBatch(N, ts.data_ptr(), key.data_ptr(), None, ctypes.cast(colp, ctypes.c_void_p), None)
    mt = native.ShpMatches()
    rc = L.shp_push_batch_device(e.h, ctypes.byref(bb), ctypes.byref(mt))
    assert rc == 0, L.shp_last_error(e.h)


ea, eb = mk(), mk()
ba = [gen(i * N) for i in range(REPS + 1)]
bb = [gen((100 + i) * N) for i in range(REPS + 1)]
torch.cuda.synchronize()
push(ea, ba[0])
push(eb, bb[0])
t0 = time.perf_counter()
for i in range(1, REPS + 1):
    push(ea, ba[i])
t1 = time.perf_counter()
one = (t1 - t0) / REPS
ea2, eb2 = mk(), mk()
push(ea2, ba[0])
push(eb2, bb[0])


def worker(e, bs):
    for i in range(1, REPS + 1):
        push(e, bs[i])


th = [threading.Thread(target=worker, args=(ea2, ba)), threading.Thread(target=worker, args=(eb2, bb))]
t0 = time.perf_counter()
for t in th:
    t.start()
for t in th:
    t.join()
t1 = time.perf_counter()
two = (t1 - t0) / REPS
print(f"one engine: {one * 1e3:.3f} ms per 100M push ({N / one / 1e9:.1f} G/s); two engines at once: "
      f"{two * 1e3:.3f} ms per pair of pushes ({2 * N / two / 1e9:.1f} G/s), {2 * one / two:.2f}x")
