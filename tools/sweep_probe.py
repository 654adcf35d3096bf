#!/usr/bin/env python3
"""Diagnostics for the sweep path: kernel times and (stamps build) per-phase cycles of k_sw_solve.

Usage: SIDDHI_HIP_DIAG_LIB=siddhi_amd/libsiddhi_hip_stamps.so python tools/sweep_probe.py [--events N] [--keys K]
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
    ap.add_argument("--agg", action="store_true", help="SHP_LAYOUT_AGG (the query must have an aggregate)")
    a = ap.parse_args()
    import torch
    from siddhi_amd import native, synth
    from siddhi_amd.query.compiler import compile_app
    _, qs, _ = compile_app(synth.QUERIES[a.config])
    cq = qs[0]
    N, K = a.events, a.keys
    eng = native.HipEngine(cq.program_json(), 0, max_keys=K, max_batch=N, max_matches=N, profile_kernels=True,
                           match_layout=native.LAYOUT_AGG if a.agg else native.LAYOUT_PAIRS)
    L = native.lib()
    stamps = hasattr(L, "shp_debug_sw_stamps")
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
        ks = {k: eng.kernel_ms(k) for k in ("sw_count", "sw_scan", "sw_scatter", "sw_lean", "sw_solve")}
        print(f"rep {rep}: m={mt.m} " + " ".join(f"{k}={v:.3f}ms" for k, v in ks.items()), flush=True)
        if stamps and ks["sw_lean"] > 0:  # k_sw_lean: wave cycles per phase, summed over the waves
            buf = (ctypes.c_ulonglong * (1 << 20))()
            nown = L.shp_debug_sw_stamps(eng.h, buf, 1 << 20)
            st = np.frombuffer(buf, dtype=np.uint64, count=nown * 8).reshape(nown, 8).astype(np.float64)
            names = ["rank+A", "emit(prev)", "scan+B", "place+C", "probe", "scanpass+carry", "-", "-"]
            tot = st.sum()
            for k in range(6):
                print(f"    {names[k]:<16} {100 * st[:, k].sum() / tot:.1f}%  (mean wave-cycles/owner {st[:, k].mean():.3e})")
        elif stamps:
            buf = (ctypes.c_ulonglong * (1 << 20))()
            nown = L.shp_debug_sw_stamps(eng.h, buf, 1 << 20)
            st = np.frombuffer(buf, dtype=np.uint64, count=nown * 8).reshape(nown, 8).astype(np.float64)
            tot = st.sum(1)
            raw = np.frombuffer(buf, dtype=np.uint64, count=nown * 8).reshape(nown, 8)
            steps = (raw[:, 7] >> np.uint64(24)).astype(np.float64)
            cands = (raw[:, 7] & np.uint64(0xffffff)).astype(np.float64)
            chunks = (raw[:, 6] >> np.uint64(40)).astype(np.float64)
            ncs = (raw[:, 6] & np.uint64(0xffffffffff)).astype(np.float64)
            print(f"  worklist items/round={steps.sum() / max(1, cands.sum()):.2f} rounds/owner={cands.mean():.0f} "
                  f"chunks/owner={chunks.mean():.1f} mean carried/chunk={ncs.sum() / max(1, chunks.sum()):.1f}")
            st[:, 6:] = 0
            tot = st.sum(1)
            names = ["rank+place", "probe", "offsets+carry", "emit", "-", "-", "-", "-"]
            print(f"  owners={nown} cycles/owner mean={tot.mean():.3e} max={tot.max():.3e}")
            for k in range(6):
                print(f"    {names[k]:<18} mean={st[:, k].mean():.3e} ({100 * st[:, k].sum() / tot.sum():.1f}%)")


if __name__ == "__main__":
    main()
