#!/usr/bin/env python3
"""Headline benchmark: input events/s of the keyed 2-state pattern (BASELINE.json configs[1], C2).

Workload: `partition with (symbol of StockStream) begin from every
e1=StockStream[price>20] -> e2=StockStream[price>e1.price] within 1 sec ... end`, 10k keys,
100M synthetic events per GPU per step (PCG32 stream, generated in HBM before the timed region).
A step = one shp_push_batch_device of the next 100M events of the stream through the engine
(partition by key + NFA + match compaction into HBM), per-key state carried across steps.
N>1: one process per GPU; each rank ingests its slice of the global stream and the events are
redistributed by key owner (key % N) with one RCCL all-to-all per step (torch.distributed nccl),
so per-GPU work is fixed (weak scaling).

Prints ONE JSON line (rank 0) with roofline (dominant kernel, HIP events on the engine stream)
and cpu_baseline (the oracle, single-threaded, on a bounded sample of the same stream).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md: 8.0 TB/s)
BYTES_PER_EVENT = 16    # ts 8 + key 4 + price 4
BYTES_PER_MATCH = 16    # one (e1 seq, e2 seq) pair of int64 (SHP_LAYOUT_PAIRS)
KERNELS = ("sw_count", "sw_scan", "sw_scatter", "sw_solve", "sw_expand",
           "radix_sort", "clock_scan", "key_hist", "key_scan", "sort_keys", "iota", "clamp_clock",
           "fast_gather", "fast_search", "nclose_scan", "fast_total", "fast_emit", "fast_carry", "nfa_lanes")
PATHS = {2: "sweep (owner partition + LDS sweep)", 1: "scan kernels over a key-sorted batch", 0: "general NFA lanes"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--events", type=int, default=100_000_000, help="events per GPU per step")
    ap.add_argument("--keys", type=int, default=10_000)
    ap.add_argument("--cpu-sample", type=int, default=2_500_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--path", choices=["auto", "general", "scan"], default="auto",
                    help="auto = sweep path (default); scan = round-1 scan kernels; general = NFA lanes")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_r01.json"))
    return ap.parse_args()


def main():
    a = parse()
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from siddhi_amd import native, synth
    from siddhi_amd.query.compiler import compile_app

    _, qs, _ = compile_app(synth.QUERIES[2])
    cq = qs[0]
    N, K, G = a.events, a.keys, world
    cap = int(N * 1.08) + 4096 if G > 1 else N
    force = {"auto": 0, "general": 1, "scan": 2}[a.path]
    eng = native.HipEngine(cq.program_json(), 0, max_keys=K, max_batch=cap, max_matches=cap,
                           device=local, force_general=force, profile_kernels=True,
                           match_layout=native.LAYOUT_PAIRS if force == 0 else native.LAYOUT_FULL)
    L = native.lib()
    steps = a.warmup + a.steps

    # synthetic input for every step, resident in HBM before timing
    def gen(step):
        start = (step * G + rank) * N
        ts = torch.empty(N, dtype=torch.int64, device="cuda")
        key = torch.empty(N, dtype=torch.int32, device="cuda")
        price = torch.empty(N, dtype=torch.float32, device="cuda")
        rc = L.shp_synth_fill(2, start, N, K, 1, 0, ts.data_ptr(), key.data_ptr(), price.data_ptr(),
                              None, None, None)
        assert rc == 0
        return ts, key, price

    batches = [gen(s) for s in range(steps)]
    torch.cuda.synchronize()

    def exchange(ts, key, price):
        """RCCL all-to-all of the SoA columns by key owner (key % G); order within a source kept."""
        owner = key % G
        order = torch.argsort(owner, stable=True)
        send_counts = torch.bincount(owner, minlength=G)
        recv_counts = torch.empty_like(send_counts)
        dist.all_to_all_single(recv_counts, send_counts)
        sc = send_counts.tolist()
        rc_ = recv_counts.tolist()
        tot = sum(rc_)
        out = []
        for col in (ts, key, price):
            src = col[order]
            dst = torch.empty(tot, dtype=col.dtype, device=col.device)
            dist.all_to_all_single(dst, src, rc_, sc)
            out.append(dst)
        return out

    def step(i):
        ts, key, price = batches[i]
        if G > 1:
            ts, key, price = exchange(ts, key, price)
            torch.cuda.current_stream().synchronize()  # engine runs on its own HIP stream
        n = ts.numel()
        colp = (ctypes.c_void_p * 1)(price.data_ptr())
        # one input stream: the stream column is NULL (= every event on stream 0)
        b = native.ShpBatch(n, ts.data_ptr(), key.data_ptr(), None, ctypes.cast(colp, ctypes.c_void_p), None)
        mt = native.ShpMatches()
        rc = L.shp_push_batch_device(eng.h, ctypes.byref(b), ctypes.byref(mt))
        if rc != 0:
            raise native.ShpError(rc, L.shp_last_error(eng.h).decode())
        return n, mt.m

    for i in range(a.warmup):
        step(i)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    kernel_ms = {}
    t0 = time.perf_counter()
    ev_local, m_local = 0, 0
    for i in range(a.warmup, steps):
        n, m = step(i)
        ev_local += n
        m_local += m
        for name in KERNELS:
            kernel_ms[name] = kernel_ms.get(name, 0.0) + eng.kernel_ms(name)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        cnt = torch.tensor([ev_local, m_local], dtype=torch.int64, device="cuda")
        dist.all_reduce(cnt)
        ev_total, m_total = int(cnt[0]), int(cnt[1])
    else:
        ev_total, m_total = ev_local, m_local

    if rank == 0:
        value = ev_total / elapsed
        dom = max(kernel_ms, key=lambda k: kernel_ms[k])
        dom_ms = kernel_ms[dom] / a.steps
        ev_per_launch = ev_local / a.steps
        m_per_launch = m_local / a.steps
        alg_bytes = BYTES_PER_EVENT * ev_per_launch + BYTES_PER_MATCH * m_per_launch
        achieved = alg_bytes / (dom_ms * 1e-3) / 1e9
        traffic = None
        if os.path.exists(a.pmc):
            try:
                pm = json.load(open(a.pmc))
                traffic = pm.get("kernels", {}).get(dom, {}).get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        cpu = None
        if not a.no_cpu_baseline and G == 1:
            cpu = cpu_baseline(cq, a.cpu_sample, K)
        line = {
            "metric": "input events/sec, keyed pattern query, 1/2/4/8 MI355X; p99 batch latency",
            "value": value,
            "unit": "events/s",
            "n_gpus": G,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32 compare / int64 ts",
            "data": "synthetic (PCG32 stream of SURVEY.md §8d, generated in HBM)",
            "config": {
                "workload": "C2: partition with (symbol of StockStream) every e1=StockStream[price>20] -> "
                            "e2=StockStream[price>e1.price] within 1 sec; 10k keys",
                "events_per_gpu_per_step": N,
                "keys": K,
                "parallelism": f"key-sharded x{G}" + (" (RCCL all-to-all by key owner)" if G > 1 else ""),
                "engine_path": PATHS.get(eng.path, str(eng.path)),
                "matches_per_s": m_total / elapsed,
                "matches_per_step_gpu0": m_per_launch,
                "p50_batch_ms": elapsed / a.steps * 1e3,
            },
            "roofline": {
                "bound": "hbm",
                "kernel": dom,
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "algorithmic_bytes_per_launch": alg_bytes,
                "kernel_ms_per_launch": {k: v / a.steps for k, v in sorted(kernel_ms.items()) if v > 0},
            },
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


def cpu_baseline(cq, sample, keys):
    """Oracle (C++ restatement of the reference semantics), one thread, first `sample` C2 events."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from diff_util import run, small_stream
    from oracle.oracle import OracleEngine
    g = small_stream(2, sample, keys)
    e = OracleEngine(cq.program_json(), 0)
    t = time.perf_counter()
    mb = run(e, cq, g)
    dt = time.perf_counter() - t
    return {"value": sample / dt, "unit": "events/s", "cores": 1, "kind": "port",
            "sample": f"first {sample} events of the C2 stream ({keys} keys), oracle/liboracle.so, "
                      f"{len(mb['key'])} matches, {dt:.1f} s"}


if __name__ == "__main__":
    main()
