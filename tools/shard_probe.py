#!/usr/bin/env python3
"""Time the N>1 exchange kernels on one GPU (no collective): the packed split + unpack against
the SoA split that replaced them, 100M C2 events over G ranks.  Prints one JSON line."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from siddhi_amd import native
    L = native.lib()
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    res = {"events": n}
    dev = torch.device("cuda", 0)
    ts = torch.empty(n, dtype=torch.int64, device=dev)
    key = torch.empty(n, dtype=torch.int32, device=dev)
    price = torch.empty(n, dtype=torch.float32, device=dev)
    assert L.shp_synth_fill(2, 0, n, 10_000, 1, 0, ts.data_ptr(), key.data_ptr(), price.data_ptr(),
                            None, None, None) == 0
    cur = torch.cuda.current_stream().cuda_stream
    for G in (2, 8):
        ws = torch.empty(int(L.shp_shard_workspace_bytes(n, G)), dtype=torch.uint8, device=dev)
        counts = (ctypes.c_int64 * G)()
        packed = torch.empty((n, 2), dtype=torch.int64, device=dev)
        o = [torch.empty(n, dtype=d, device=dev) for d in (torch.int64, torch.int32, torch.float32)]

        def timed(fn, reps=5):
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ms = []
            for _ in range(reps):
                e0.record()
                fn()
                e1.record()
                torch.cuda.synchronize()
                ms.append(e0.elapsed_time(e1))
            return min(ms)

        def part_packed():
            assert L.shp_shard_partition(n, ts.data_ptr(), key.data_ptr(), price.data_ptr(), None, G,
                                         packed.data_ptr(), counts, ws.data_ptr(), cur) == 0

        def unpack():
            assert L.shp_shard_unpack(n, packed.data_ptr(), o[0].data_ptr(), o[1].data_ptr(), o[2].data_ptr(),
                                      None, cur) == 0

        def part_soa():
            assert L.shp_shard_partition_soa(n, ts.data_ptr(), key.data_ptr(), price.data_ptr(), None, G,
                                             o[0].data_ptr(), o[1].data_ptr(), o[2].data_ptr(), None, counts,
                                             ws.data_ptr(), cur) == 0

        res[f"G{G}"] = {"partition_packed_ms": timed(part_packed), "unpack_ms": timed(unpack),
                        "partition_soa_ms": timed(part_soa)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
