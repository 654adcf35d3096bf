#!/usr/bin/env python3
"""The group split (k_gs_count / k_gs_scatter) at an N=8 job's per-rank shape, on one GPU: an
in-process group of 8 ranks on cuda:0, each rank's slice 100M / 8 events of the C2 stream, so one
stage() splits 100M events (run it under rocprofv3 --kernel-trace --stats for the kernel times).
Prints the stage() wall time per push."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from siddhi_amd import native, synth
    from siddhi_amd.query.compiler import compile_app
    L = native.lib()
    G, K, N = 8, 10_000, 100_000_000 // 8
    cq = compile_app(synth.QUERIES[2])[1][0]
    grp = native.HipGroup(cq.program_json(), 0, max_keys=K, max_batch=N * 3 // 2, max_matches=N * 2,
                          devices=[0] * G, match_layout=native.LAYOUT_PAIRS32)
    spec = synth.CONFIGS[2]
    sl = []
    for r in range(G):
        ts = torch.empty(N, dtype=torch.int64, device="cuda")
        key = torch.empty(N, dtype=torch.int32, device="cuda")
        price = torch.empty(N, dtype=torch.float32, device="cuda")
        assert L.shp_synth_fill(2, r * N, N, K, 1, int(spec.dense), ts.data_ptr(), key.data_ptr(), price.data_ptr(),
                                None, None, None) == 0
        sl.append((ts, key, None, [price]))
    torch.cuda.synchronize()
    for it in range(6):
        t0 = time.perf_counter()
        keep = grp.stage_device(sl)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        grp.run()
        torch.cuda.synchronize()
        print(f"push {it}: stage {1e3 * (t1 - t0):.3f} ms (8 splits of {N} events + copies)", flush=True)
        del keep


if __name__ == "__main__":
    main()
