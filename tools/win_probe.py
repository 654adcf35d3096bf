#!/usr/bin/env python3
"""Diagnostics for k_sw_win (sweep_win.h): kernel times and (stamps build) cycles per phase summed
over the units, reset before each push.

Usage: SIDDHI_HIP_DIAG_LIB=siddhi_amd/libsiddhi_hip_stamps.so python tools/win_probe.py [--events N] [--keys K]
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
    ap.add_argument("--keys", type=int, default=10_000)
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch
    from siddhi_amd import native, synth
    from siddhi_amd.query.compiler import compile_app
    _, qs, _ = compile_app(synth.QUERIES[a.config])
    cq = qs[0]
    N, K = a.events, a.keys
    eng = native.HipEngine(cq.program_json(), 0, max_keys=K, max_batch=N, max_matches=N, profile_kernels=True,
                           match_layout=native.LAYOUT_PAIRS32)
    L = native.lib()
    stamps = hasattr(L, "shp_debug_sw_stamps")
    names = ["ticket", "owner+init", "halo", "segment", "lookback", "flush", "total", "halo recs"]
    prev = np.zeros(16)
    wn = ["load+masks", "own probe", "carried probe", "emit own", "carried emit+compact", "carried entries"]
    for rep in range(a.reps):
        ts = torch.empty(N, dtype=torch.int64, device="cuda")
        key = torch.empty(N, dtype=torch.int32, device="cuda")
        price = torch.empty(N, dtype=torch.float32, device="cuda")
        assert L.shp_synth_fill(a.config, rep * N, N, K, 1, 0, ts.data_ptr(), key.data_ptr(), price.data_ptr(),
                                None, None, None) == 0
        torch.cuda.synchronize()
        colp = (ctypes.c_void_p * 1)(price.data_ptr())
        b = native.ShpBatch(N, ts.data_ptr(), key.data_ptr(), None, ctypes.cast(colp, ctypes.c_void_p), None)
        mt = native.ShpMatches()
        rc = L.shp_push_batch_device(eng.h, ctypes.byref(b), ctypes.byref(mt))
        assert rc == 0, L.shp_last_error(eng.h)
        ks = {k: eng.kernel_ms(k) for k in ("sw_count", "sw_scatter", "sw_win", "sw_win_tail", "sw_lean", "sw_solve")}
        print(f"rep {rep}: m={mt.m} " + " ".join(f"{k}={v:.3f}ms" for k, v in ks.items()), flush=True)
        if stamps:
            buf = (ctypes.c_ulonglong * 64)()
            L.shp_debug_sw_stamps(eng.h, buf, 64)
            cur = np.frombuffer(buf, dtype=np.uint64, count=16).astype(np.float64)
            d, prev = cur - prev, cur
            units = (N + 1023) // 1024
            print(f"  per unit ({units} units): " + " ".join(f"{names[k]}={d[k] / units:.0f}" for k in range(8)))
            print("  share of total: " + " ".join(f"{names[k]}={100 * d[k] / max(1, d[6]):.1f}%" for k in range(6)))
            wins = units * 16
            print("  segment windows, wave-cycles per window: " + " ".join(f"{wn[k]}={d[8 + k] / wins:.0f}" for k in range(6)))


if __name__ == "__main__":
    main()
