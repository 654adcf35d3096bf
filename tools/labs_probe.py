#!/usr/bin/env python3
"""Diagnostics for the logical-absent path (C4): kernel times and (stamps build) k_labs_w's
per-phase wave cycles and counts per key.

Usage: SIDDHI_HIP_DIAG_LIB=siddhi_amd/libsiddhi_hip_stamps.so python tools/labs_probe.py [--events N] [--keys K]
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=100_000_000)
    ap.add_argument("--keys", type=int, default=1_000)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--disorder", type=float, default=0.0, help="as bench.py --disorder")
    a = ap.parse_args()
    import torch
    from siddhi_amd import native, synth
    from siddhi_amd.query.compiler import compile_app
    _, qs, _ = compile_app(synth.QUERIES[4])
    cq = qs[0]
    N, K = a.events, a.keys
    eng = native.HipEngine(cq.program_json(), 0, max_keys=K, max_batch=N, max_matches=N, profile_kernels=True,
                           force_general=4)
    L = native.lib()
    stamps = hasattr(L, "shp_debug_la_stamps")
    for rep in range(a.reps):
        ts = torch.empty(N, dtype=torch.int64, device="cuda")
        key = torch.empty(N, dtype=torch.int32, device="cuda")
        price = torch.empty(N, dtype=torch.float32, device="cuda")
        stream = torch.empty(N, dtype=torch.int32, device="cuda")
        assert L.shp_synth_fill(4, rep * N, N, K, 3, 1, ts.data_ptr(), key.data_ptr(), price.data_ptr(), None,
                                stream.data_ptr(), None) == 0
        if a.disorder > 0:  # (bench.py's disorder: events moved back by up to 8 s)
            gg = torch.Generator(device="cuda").manual_seed(1000 + rep * N)
            back = torch.rand(N, device="cuda", generator=gg) < a.disorder
            ts -= back.to(torch.int64) * torch.randint(0, 8000, (N,), device="cuda", generator=gg)
        torch.cuda.synchronize()
        ncol = max(1, len(cq.columns))  # one pointer per program column (S1, S2, S3 price): all the price column
        colp = (ctypes.c_void_p * ncol)(*([price.data_ptr()] * ncol))
        b = native.ShpBatch(N, ts.data_ptr(), key.data_ptr(), stream.data_ptr(), ctypes.cast(colp, ctypes.c_void_p),
                            None)
        mt = native.ShpMatches()
        rc = L.shp_push_batch_device(eng.h, ctypes.byref(b), ctypes.byref(mt))
        assert rc == 0, L.shp_last_error(eng.h)
        ks = {k: eng.kernel_ms(k) for k in ("labs_count", "labs_mscan", "labs_split", "labs", "labs_segcheck",
                                            "labs_out", "clock_scan")}
        print(f"rep {rep}: m={mt.m} segmiss={eng.stat('labs_segmiss')} " +
              " ".join(f"{k}={v:.3f}ms" for k, v in ks.items()), flush=True)
        if stamps:
            S = 16
            buf = (ctypes.c_ulonglong * (K * 4 * S))()  # (k_labs_w segments: up to 4 slots per key)
            L.shp_debug_la_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
            nk = L.shp_debug_la_stamps(eng.h, buf, K * 4 * S)
            st = np.frombuffer(buf, dtype=np.uint64, count=nk * S).reshape(nk, S).astype(np.float64)
            phases = [(0, "load+filters"), (1, "partial"), (2, "doomed E_D"), (3, "leave search"), (8, "Z kills"),
                      (9, "firings"), (4, "settle"), (5, "queue"), (13, "exact blocks"), (15, "exact firings")]
            tot = sum(st[:, x].sum() for x, _ in phases)
            blocks = st[:, 7].sum() / 64
            for x, name in phases:
                print(f"    {name:<14} {100 * st[:, x].sum() / tot:5.1f}%  cycles/block {st[:, x].sum() / blocks:8.0f}")
            print(f"    waiting pairs/block {st[:, 6].sum() / blocks:.1f}  kill rounds/block {st[:, 10].sum() / blocks:.2f}"
                  f"  Z/block {st[:, 11].sum() / blocks:.1f}  events/key {st[:, 7].mean():.0f}"
                  f"  cycles/block {tot / blocks:.0f}")
            print(f"    exact variant: {int(st[:, 14].sum())} of {nk} slots; events by the exact rule "
                  f"{st[:, 12].sum() / st[:, 7].sum():.3f} of all, {(st[:, 13].sum() + st[:, 15].sum()) / max(1, st[:, 12].sum()):.0f} cycles each "
                  f"({st[:, 15].sum() / max(1, st[:, 12].sum()):.0f} in the timer firings)")

if __name__ == "__main__":
    main()
