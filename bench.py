#!/usr/bin/env python3
"""Headline benchmark: input events/s of the keyed 2-state pattern (BASELINE.json configs[1], C2).

Workload: `partition with (symbol of StockStream) begin from every
e1=StockStream[price>20] -> e2=StockStream[price>e1.price] within 1 sec ... end`, 10k keys,
100M synthetic events per GPU per step (PCG32 stream, generated in HBM before the timed region).
A step = one shp_push_batch_device of the next 100M events of the stream through the engine
(partition by key + NFA + match compaction into HBM), per-key state carried across steps.
N>1: one process per GPU; each rank ingests its slice of the global stream and the library's
key-sharded group (shp_group_*, multi-GPU behind the C-ABI) redistributes the events by key owner
(key % N): a HIP stable split into destination-grouped columns, then RCCL ncclSend/ncclRecv over
xGMI from the engine's own communicator; per-GPU work is fixed (weak scaling).  torch.distributed
(gloo) is the control plane only: barriers, the RCCL id broadcast, max-over-ranks timing.

Prints ONE JSON line (rank 0) with roofline (dominant kernel, HIP events on the engine stream)
and cpu_baseline (the oracle, single-threaded, on a bounded sample of the same stream).
"""
from __future__ import annotations

import argparse
import ctypes

import numpy as np
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md: 8.0 TB/s)
BYTES_PER_EVENT = 16    # ts 8 + key 4 + price 4
# SURVEY.md §8d per config: C4 reads the stream id too (17 B/event: ts 8 + key 4 + stream 1 + price 4)
BYTES_PER_EVENT_CFG = {"4": 17}
BYTES_PER_MATCH = {"pairs32": 8,  # (e2 batch index, e2 seq - e1 seq) as two u32 (SHP_LAYOUT_PAIRS32)
                   "pairs": 16,  # one (e1 seq, e2 seq) pair of int64 (SHP_LAYOUT_PAIRS)
                   "agg": 12,    # (key u32, aggregate f64) per match (SHP_LAYOUT_AGG, C5)
                   "chain32": 4,  # e2 batch index | L << 28, the e1 chain implied (SHP_LAYOUT_CHAIN32, C3')
                   "full": 16}
KERNELS = ("sw_count", "sw_scan", "sw_scatter", "sw_win", "sw_win_tail", "sw_lean", "sw_solve", "sw_spill", "sw_expand",
           "radix_sort", "clock_scan", "key_hist", "key_scan", "sort_keys", "iota", "clamp_clock",
           "fast_gather", "fast_search", "nclose_scan", "fast_total", "fast_emit", "fast_carry", "nfa_lanes",
           "cseq_count", "cseq_scan", "cseq", "co_count", "co_scan", "co_scatter", "co_run", "cs_pack", "cs_sort", "cs_count", "cs_scan", "cs_emit", "cs_state", "labs_pack", "labs_sort", "labs_gather", "labs_count", "labs_mscan", "labs_split", "labs_steps", "labs_segcheck", "labs_scan", "labs", "labs_pos", "labs_out",
           "key_bounds")
WORKLOADS = {
    "1": "C1: every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] within 1 sec (one key)",
    "2": "C2: partition with (symbol of StockStream) every e1=StockStream[price>20] -> "
         "e2=StockStream[price>e1.price] within 1 sec",
    "3b": "C3': partition with (k of S) every e1=S[v>20]<1:5>, e2=S[v<e1[last].v]",
    "4": "C4: partition every (e1=S1[price>20] and e2=S2[price>20]) -> not S3[price>e1.price] for 5 sec "
         "within 10 sec",
    "5": "C5: partition every e1 -> e2[price>e1.price] within 1 sec select symbol, avg(e2.price)",
}
PATHS = {2: "sweep (owner partition + LDS sweep)", 1: "scan kernels over a key-sorted batch", 0: "general NFA lanes",
         3: "count-sequence automaton over a key-sorted batch (cseq)",
         4: "logical-absent automaton over a key-sorted batch (labs: k_labs_w, ordered pushes; k_labs, any order)"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--events", type=int, default=100_000_000, help="events per GPU per step")
    ap.add_argument("--keys", type=int, default=0, help="keys (default: the config's, C2 = 10k)")
    ap.add_argument("--config", default="2", help="SURVEY §8d config: 2 (headline), 1, 3b, 4, 5")
    ap.add_argument("--cpu-sample", type=int, default=2_500_000, help="events per CPU thread")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads of the key-sharded CPU baseline (default: the box's CPU share, "
                         "OMP_NUM_THREADS, else os.cpu_count())")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-expanded", action="store_true",
                    help="skip the second timed pass of a compact layout with its words expanded to FULL rows")
    ap.add_argument("--path", choices=["auto", "general", "scan", "labs"], default="auto",
                    help="auto = the engine's default path; scan = round-1 scan kernels; general = NFA lanes; "
                         "labs = the logical-absent automaton (C4, force_general 4; the auto path for C4 too)")
    ap.add_argument("--same-device", action="store_true",
                    help="N>1 rehearsal on a one-GPU box without torchrun: one process, an in-process group of "
                         "--gpus ranks all on cuda:0 (device copies stand in for RCCL)")
    ap.add_argument("--pmc", default=None,
                    help="PMC traffic per kernel (tools/pmc_run.sh, tools/pmc_cfg.sh; default "
                         "profiles/pmc_traffic_c<config>.json); used only when it was measured on this "
                         "library build (lib_sha16), this config and key count")
    ap.add_argument("--latency-batches", type=int, default=200,
                    help="§8d latency: batches of --latency-events, push + D2H of the match payload (0: skip)")
    ap.add_argument("--latency-events", type=int, default=16_000_000)
    ap.add_argument("--pairs-layout", choices=["pairs32", "pairs"], default="pairs32",
                    help="match payload of the 2-state sweep: 8-byte PAIRS32 (default) or 16-byte PAIRS")
    ap.add_argument("--disorder", type=float, default=0.0,
                    help="fraction of events whose ts is moved back by up to 8 s (C4: the exact kernel, k_labs, "
                         "takes such pushes; a measurement of that path, not the headline)")
    ap.add_argument("--cseq-layout", choices=["chain32", "full"], default="chain32",
                    help="match payload of the count-sequence path (C3'): 4-byte CHAIN32 words (default) or FULL")
    ap.add_argument("--e2e-steps", type=int, default=3,
                    help="SURVEY §8d(b) end-to-end host ingest: steps of N events from page-locked host columns "
                         "through shp_stage_batch / shp_run_staged (records back to host memory); 0: skip")
    ap.add_argument("--e2e-batch", type=int, default=12_500_000, help="events per staged host batch")
    ap.add_argument("--e2e-modes", default=None,
                    help="comma list of end-to-end forms to run (default all: serial, pipelined, pipelined_ts32, "
                         "pipelined_narrow); tools/gpu_e2e_trace.sh traces one at a time")
    return ap.parse_args()


def main():
    a = parse()
    if a.pmc is None:
        a.pmc = os.path.join(ROOT, "profiles", f"pmc_traffic_c{a.config}.json")
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    G = a.gpus if a.same_device else world
    if a.same_device:  # rehearsal of the N>1 path on a one-GPU box: an in-process group, every rank on cuda:0
        local, world, rank = 0, 1, 0
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        # control plane only (barriers, the RCCL id broadcast, max-over-ranks timing): the data-path
        # exchange is the engine's own RCCL communicator inside libsiddhi_hip.so (shp_group_*)
        import torch.distributed as dist
        dist.init_process_group("gloo")

    from siddhi_amd import native, synth
    from siddhi_amd.query.compiler import compile_app

    cfg_id = int(a.config) if a.config.isdigit() else a.config
    spec = synth.CONFIGS[3 if cfg_id == "3b" else cfg_id]
    _, qs, _ = compile_app(synth.QUERIES[cfg_id])
    cq = qs[0]
    assert all(c[1] == 1 and c[2] == "float" for c in cq.columns), "bench configs read price only"
    N = a.events
    K = a.keys if a.keys else spec.keys
    K_local = -(-K // G)  # each rank's engine holds a dense dictionary of the keys it owns
    cap = int(N * 1.08) + 4096 if G > 1 else N
    force = {"auto": 0, "general": 1, "scan": 2, "labs": 4}[a.path]
    sweep = force == 0 and _sweep_shape(cq, local, K_local)
    layout = ("agg" if "aggregate" in cq.program else a.pairs_layout) if sweep else "full"
    if cfg_id in (3, "3b") and force == 0:  # the count-sequence path takes C3 and C3' by default
        layout = a.cseq_layout
    mlay = {"agg": native.LAYOUT_AGG, "pairs": native.LAYOUT_PAIRS, "pairs32": native.LAYOUT_PAIRS32,
            "chain32": native.LAYOUT_CHAIN32, "full": native.LAYOUT_FULL}[layout]
    L = native.lib()
    grp = None
    if G == 1:
        eng = native.HipEngine(cq.program_json(), 0, max_keys=K_local, max_batch=cap, max_matches=cap,
                               device=local, force_general=force, profile_kernels=True, match_layout=mlay)
        engines = [eng]
    else:
        if a.same_device:
            grp = native.HipGroup(cq.program_json(), 0, max_keys=K, max_batch=cap, max_matches=cap,
                                  devices=[0] * G, force_general=force, profile_kernels=True, match_layout=mlay)
        else:
            cid = torch.zeros(native.COMM_ID_BYTES, dtype=torch.uint8)
            if rank == 0:
                cid = torch.frombuffer(bytearray(native.comm_id()), dtype=torch.uint8)
            dist.broadcast(cid, 0)
            grp = native.HipGroup(cq.program_json(), 0, max_keys=K, max_batch=cap, max_matches=cap, world=G,
                                  rank=rank, comm=bytes(cid.numpy().tobytes()), device=local, force_general=force,
                                  profile_kernels=True, match_layout=mlay)
        engines = [_EngineView(grp, i) for i in range(grp.nlocal)]
    eng = engines[0]
    steps = a.warmup + a.steps
    my_ranks = list(range(G)) if a.same_device else [rank]

    # synthetic input for every step, resident in HBM before timing: step s of the global stream is
    # G consecutive slices of N events, slice r ingested by rank r
    def gen(step, r):
        start = (step * G + r) * N
        ts = torch.empty(N, dtype=torch.int64, device="cuda")
        key = torch.empty(N, dtype=torch.int32, device="cuda")
        price = torch.empty(N, dtype=torch.float32, device="cuda")
        stream = torch.empty(N, dtype=torch.int32, device="cuda") if spec.n_streams > 1 else None
        rc = L.shp_synth_fill(spec.config, start, N, K, spec.n_streams, int(spec.dense), ts.data_ptr(),
                              key.data_ptr(), price.data_ptr(), None,
                              stream.data_ptr() if stream is not None else None, None)
        assert rc == 0
        if a.disorder > 0:  # events going back in time (seeded by the step, so every run is the same stream)
            gg = torch.Generator(device="cuda").manual_seed(1000 + start)
            back = torch.rand(N, device="cuda", generator=gg) < a.disorder
            ts -= back.to(torch.int64) * torch.randint(0, 8000, (N,), device="cuda", generator=gg)
        return ts, key, price, stream

    batches = [[gen(s, r) for r in my_ranks] for s in range(steps)]
    torch.cuda.synchronize()
    ncol = max(1, len(cq.columns))

    def push(ts, key, price, stream, e=None):
        e = e or eng
        n = ts.numel()
        # one pointer per program column (cq.columns: (stream, attr, type)); every stream's
        # predicate attribute is the synthetic price column
        colp = (ctypes.c_void_p * ncol)(*([price.data_ptr()] * ncol))
        b = native.ShpBatch(n, ts.data_ptr(), key.data_ptr(), stream.data_ptr() if stream is not None else None,
                            ctypes.cast(colp, ctypes.c_void_p), None)
        mt = native.ShpMatches()
        rc = L.shp_push_batch_device(e.h, ctypes.byref(b), ctypes.byref(mt))
        if rc != 0:
            raise native.ShpError(rc, L.shp_last_error(e.h).decode())
        return n, mt.m

    def slices(i):
        return [(ts, key, stream, [price] * ncol) for (ts, key, price, stream) in batches[i]]

    staged = []

    def step(i):
        """One batch through the hot path.  N>1: shp_group_run runs batch i (split, exchanged by key
        owner and landed in a receive slot earlier) on a worker thread -- the blocking C call
        releases the GIL -- while this thread stages batch i + 2 (HIP split + RCCL exchange inside
        the library), so the exchange overlaps the engines instead of adding to them."""
        if G == 1:
            return push(*batches[i][0])
        out = {}

        def work():
            try:
                out["r"] = grp.run()
            except BaseException as ex:  # re-raised on the main thread
                out["e"] = ex

        th = threading.Thread(target=work)
        th.start()
        try:
            if i + 2 < steps:
                staged.append(grp.stage_device(slices(i + 2)))
        finally:
            th.join()
        if "e" in out:
            raise out["e"]
        return N * len(my_ranks), sum(out["r"])

    if G > 1:  # fill the pipeline (untimed)
        for i in range(min(2, steps)):
            staged.append(grp.stage_device(slices(i)))
    for i in range(a.warmup):
        step(i)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    kernel_ms = {}
    t0 = time.perf_counter()
    ev_local, m_local = 0, 0
    lat = []
    for i in range(a.warmup, steps):
        ts0 = time.perf_counter()
        n, m = step(i)  # synchronous: matches are counted on the host when it returns
        lat.append((time.perf_counter() - ts0) * 1e3)
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
        tt = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        cnt = torch.tensor([ev_local, m_local], dtype=torch.int64)
        dist.all_reduce(cnt)
        ev_total, m_total = int(cnt[0]), int(cnt[1])
    else:
        ev_total, m_total = ev_local, m_local

    expanded = None
    if G == 1 and layout in ("chain32", "pairs32") and not a.no_expanded:
        fresh = [gen(steps + s, 0) for s in range(1 + a.steps)]
        torch.cuda.synchronize()  # (generated on torch's stream: complete before the engine reads them)
        if layout == "chain32":  # the same path with FULL rows written by its run kernel (k_co_run)
            full = native.HipEngine(cq.program_json(), 0, max_keys=K_local, max_batch=cap, max_matches=cap,
                                    device=local, force_general=force, match_layout=native.LAYOUT_FULL)
            try:
                expanded = full_rate(full, fresh, push)
            finally:
                full.close()
        else:
            expanded = expanded_rate(eng, L, native, fresh, push, layout)
        del fresh

    latency = None
    if rank == 0 and G == 1 and a.latency_batches > 0 and layout != "full":
        latency = batch_latency(eng, L, native, spec, K, layout, a.latency_events, a.latency_batches,
                                (a.warmup + a.steps + 1) * N)

    e2e = None
    if rank == 0 and G == 1 and a.e2e_steps > 0 and layout != "full" and a.disorder == 0:
        del batches
        torch.cuda.empty_cache()
        e2e = end_to_end(cq, L, native, spec, K, a.e2e_batch, N, a.e2e_steps, (a.warmup + 2 * a.steps + 4) * N,
                         force, mlay, layout, local, a.e2e_modes)

    if rank == 0:
        value = ev_total / elapsed
        dom = max(kernel_ms, key=lambda k: kernel_ms[k])
        dom_ms = kernel_ms[dom] / a.steps
        # per launch of the dominant kernel on rank 0's (first local) engine: the events it received
        ev_per_launch = ev_total / G / a.steps
        m_per_launch = m_total / G / a.steps
        bpe = BYTES_PER_EVENT_CFG.get(str(cfg_id), BYTES_PER_EVENT)
        alg_bytes = bpe * ev_per_launch + BYTES_PER_MATCH[layout] * m_per_launch
        achieved = alg_bytes / (dom_ms * 1e-3) / 1e9
        traffic = step_traffic = None
        pmc_src = None
        if os.path.exists(a.pmc):
            try:
                pm = json.load(open(a.pmc))
                # PMC passes are of one bench command (tools/pmc_run.sh) on one library build: used
                # only for that config, key count and build (the same .so as this run loaded)
                if (str(pm.get("config", "2")) == str(cfg_id) and int(pm.get("keys", K)) == K and G == 1
                        and float(pm.get("disorder", 0.0)) == a.disorder
                        and pm.get("lib_sha16") == _lib_sha16(native.LIB_PATH)):
                    ks = pm.get("kernels", {})
                    traffic = ks.get(dom, {}).get("hbm_bytes_per_launch")
                    # the whole push: every kernel of the run but the input generator, the torch
                    # kernels that move events back for --disorder (both before timing) and the
                    # one-time state initialisation (one launch each per push)
                    step_traffic = sum(v["hbm_bytes_per_launch"] for k, v in ks.items()
                                       if k not in ("synth", "sw_init", "labs_init", "cseq_init", "fast_init", "iota")
                                       and not k.startswith("__amd_rocclr") and "at::native" not in k)
                    pmc_src = os.path.relpath(a.pmc, ROOT)
            except Exception:
                traffic = step_traffic = None
        cpu = None
        if not a.no_cpu_baseline and G == 1:
            cpu = cpu_baseline(cq, a.cpu_sample, K, spec.config, a.cpu_threads)
        step_ms = elapsed / a.steps * 1e3
        step_achieved = alg_bytes / (step_ms * 1e-3) / 1e9
        par = f"key-sharded x{G}"
        if G > 1:
            par += (" (shp_group: HIP split by key owner + " +
                    ("device copies, every rank on cuda:0 (rehearsal)" if a.same_device else
                     "RCCL ncclSend/ncclRecv over xGMI") +
                    " inside libsiddhi_hip.so, batch i+2 exchanged while the engines run batch i)")
        line = {
            "metric": "input events/sec, keyed pattern query, 1/2/4/8 MI355X; p99 batch latency",
            "value": value,
            "unit": "events/s",
            "n_gpus": G,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": step_ms,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32 compare / int64 ts",
            "data": "synthetic (PCG32 stream of SURVEY.md §8d, generated in HBM)",
            "config": {
                "workload": WORKLOADS.get(str(cfg_id), f"C{cfg_id}") + f"; {K} keys" + (f"; {a.disorder:g} of events moved back by up to 8 s" if a.disorder else ""),
                "events_per_gpu_per_step": N,
                "keys": K,
                "parallelism": par,
                "engine_path": _path_desc(eng, layout),
                # monitoring counters since create (shp_engine_stat): hand-backs and re-runs of the push
                "engine_stats": ({k: native_stat(eng, k) for k in ("pushes", "lean_fallbacks", "labs_fallbacks",
                                                                 "labs_segmiss", "sweep_r16_reruns", "spill_reruns")}
                                 if G == 1 else None),
                "matches_per_s": m_total / elapsed,
                "matches_per_step_gpu0": m_per_launch,
                "p50_batch_ms": float(np.percentile(lat, 50)),
                "p99_batch_ms": float(np.percentile(lat, 99)),
                "match_layout": layout,
                "latency": latency,
                # host columns in, match records in host memory out (what the Java host
                # drives), beside the device-resident `value`
                "end_to_end": e2e,
                # the compact words are not self-contained (a CHAIN32 word names its e2 event; the
                # chain needs the batch's key column and the engine's pre-push history): the same
                # path with each push's words expanded to FULL rows in HBM, timed the same way
                "expanded": expanded,
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
                "bytes_per_event": bpe,
                "bytes_per_match": BYTES_PER_MATCH[layout],
                "kernel_ms_per_launch": {k: v / a.steps for k, v in sorted(kernel_ms.items()) if v > 0},
                # the same algorithmic bytes over the whole step (every kernel of the push, plus the
                # host round trip), the fraction the headline `value` corresponds to
                "step": {"achieved": step_achieved, "frac": step_achieved / HBM_PEAK_GBS, "ms": step_ms,
                         "traffic": step_traffic,
                         "traffic_x": (step_traffic / alg_bytes) if step_traffic else None},
                "traffic_source": pmc_src,
            },
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if grp is not None:
        grp.close()
    if dist:
        dist.destroy_process_group()


class _EngineView:
    """A group member's engine, for the per-kernel timings and the path (shp_group_engine)."""

    def __init__(self, grp, i):
        from siddhi_amd import native
        self.h = ctypes.c_void_p(native.lib().shp_group_engine(grp.h, i))

    @property
    def path(self):
        from siddhi_amd import native
        return native.lib().shp_engine_path(self.h)

    def kernel_ms(self, which="total"):
        from siddhi_amd import native
        return native.lib().shp_last_kernel_ms(self.h, which.encode())


def _path_desc(eng, layout):
    d = PATHS.get(eng.path, str(eng.path))
    if eng.path == 3:
        own = native_stat(eng, "cseq_owner")
        d = ("count-sequence automaton by owners (owner multisplit + per-owner key order in LDS, cseq_own.h)"
             if own else d) + (", CHAIN32 words" if layout == "chain32" else ", FULL rows")
    return d


def native_stat(eng, which):
    from siddhi_amd import native
    return native.lib().shp_engine_stat(eng.h, which.encode())


def full_rate(full, bats, push):
    """The count sequence with FULL rows (self-contained: e1's chain refs written by k_co_run) on a
    second engine over fresh batches: events/s and ms per step, beside the CHAIN32 headline."""
    import torch
    push(*bats[0], e=full)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev = 0
    for b in bats[1:]:
        ev += push(*b, e=full)[0]
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    k = len(bats) - 1
    return {"value": ev / el, "ms_per_step": el / k * 1e3, "layout": "full (rows and refs written by the run kernel)"}


def expanded_rate(eng, L, native, bats, push, layout):
    """Pushes of fresh batches, each followed by the engine's expansion of its compact words into
    FULL match rows in HBM (shp_engine_device_records: k_cs_expand / the sweep's pair expansion),
    synchronously: events/s and ms per step of the self-contained form."""
    import torch
    out = native.ShpMatches()
    nrefs = ctypes.c_int64(0)
    L.shp_engine_device_records.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    L.shp_engine_device_records.restype = ctypes.c_int

    def one(b):
        n, m = push(*b)
        rc = L.shp_engine_device_records(eng.h, ctypes.byref(out), ctypes.byref(nrefs))
        if rc != 0:
            raise native.ShpError(rc, L.shp_last_error(eng.h).decode())
        return n, m
    one(bats[0])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev = 0
    for b in bats[1:]:
        ev += one(b)[0]
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    k = len(bats) - 1
    return {"value": ev / el, "ms_per_step": el / k * 1e3, "layout": f"{layout} + expansion to FULL rows"}


def batch_latency(eng, L, native, spec, K, layout, n, batches, start):
    """SURVEY §8d latency: batches of n events (device-resident input, generated untimed), each
    timed from shp_push_batch_device entry until its match payload (pairs, or (key, aggregate)
    rows) is in host memory, over `batches` batches.  The payload lands in page-locked memory
    (shp_host_alloc = hipHostMalloc, as a Java host would pin its receive segment with
    shp_host_register); the same batches into pageable memory are reported beside it."""
    import torch
    bufs = [(torch.empty(n, dtype=torch.int64, device="cuda"), torch.empty(n, dtype=torch.int32, device="cuda"),
             torch.empty(n, dtype=torch.float32, device="cuda")) for _ in range(2)]
    per = BYTES_PER_MATCH[layout]
    hbytes = int(n * 1.1) * 16
    pinned = L.shp_host_alloc(hbytes)
    if not pinned:
        raise RuntimeError("shp_host_alloc failed")
    pageable = np.empty(hbytes // 8, dtype=np.int64)
    res = {}
    try:
        for kind, dst in (("pinned", pinned), ("pageable", pageable.ctypes.data)):
            lat = []
            for b in range(batches):
                ts, key, price = bufs[b & 1]
                assert L.shp_synth_fill(spec.config, start + b * n, n, K, 1, int(spec.dense), ts.data_ptr(),
                                        key.data_ptr(), price.data_ptr(), None, None, None) == 0
                torch.cuda.synchronize()
                colp = (ctypes.c_void_p * 1)(price.data_ptr())
                bt = native.ShpBatch(n, ts.data_ptr(), key.data_ptr(), None, ctypes.cast(colp, ctypes.c_void_p), None)
                mt = native.ShpMatches()
                t0 = time.perf_counter()
                rc = L.shp_push_batch_device(eng.h, ctypes.byref(bt), ctypes.byref(mt))
                if rc != 0:
                    raise native.ShpError(rc, L.shp_last_error(eng.h).decode())
                if mt.m * per > hbytes:
                    raise RuntimeError("latency host buffer too small")
                if layout == "agg":
                    assert L.shp_dev_to_host(dst, mt.key, mt.m * 4) == 0
                    assert L.shp_dev_to_host(dst + mt.m * 4, mt.agg, mt.m * 8) == 0
                else:
                    assert L.shp_dev_to_host(dst, mt.refs, mt.m * per) == 0
                lat.append((time.perf_counter() - t0) * 1e3)
            res[kind] = lat
            start += batches * n
    finally:
        L.shp_host_free(pinned)
    pl, pg = res["pinned"], res["pageable"]
    return {"batch_events": n, "batches": batches, "bytes_per_match_to_host": per,
            "p50_ms": float(np.percentile(pl, 50)), "p99_ms": float(np.percentile(pl, 99)),
            "host_buffer": "page-locked (shp_host_alloc)",
            "pageable_p50_ms": float(np.percentile(pg, 50)), "pageable_p99_ms": float(np.percentile(pg, 99)),
            "what": "shp_push_batch_device entry -> match payload in host memory"}


def end_to_end(cq, L, native, spec, K, nb, N, steps, start, force, mlay, layout, device, only=None):
    """the step's N events from page-locked host SoA columns (the Java host's
    ColumnarBatch segments, pinned with shp_host_register) to match records in host memory, in
    batches of nb events: (1) serial -- shp_push_batch_compact per batch, the copy, the run and the
    records' copy back one after the other; (2) pipelined -- shp_stage_batch of batch i+1 (H2D on the
    engine's copy stream) while shp_run_staged runs batch i; (3) the same with the narrow ingest form
    (shp_stage_batch_ts32: 4-byte ts offsets, 12 B/event).  Fresh events every step (the stream goes
    on); each form on its own engine, one untimed warm-up step each.  Achieved PCIe GB/s counts the
    H2D input bytes plus the D2H record bytes over the wall time."""
    import torch
    nsub = -(-N // nb)
    per = BYTES_PER_MATCH[layout]
    total_steps = 1 + steps
    # page-locked host input for every step: generated in HBM, copied down untimed
    host = []
    for s in range(total_steps):
        ts = torch.empty(N, dtype=torch.int64, pin_memory=True)
        key = torch.empty(N, dtype=torch.int32, pin_memory=True)
        price = torch.empty(N, dtype=torch.float32, pin_memory=True)
        ts32 = torch.empty(N, dtype=torch.int32, pin_memory=True)
        key16 = torch.empty(N, dtype=torch.int16, pin_memory=True) if K <= 65536 else None
        dts = torch.empty(N, dtype=torch.int64, device="cuda")
        dkey = torch.empty(N, dtype=torch.int32, device="cuda")
        dpr = torch.empty(N, dtype=torch.float32, device="cuda")
        assert L.shp_synth_fill(spec.config, start + s * N, N, K, 1, int(spec.dense), dts.data_ptr(), dkey.data_ptr(),
                                dpr.data_ptr(), None, None, None) == 0
        torch.cuda.synchronize()
        base = torch.empty(nsub, dtype=torch.int64)
        d32 = torch.empty(N, dtype=torch.int32, device="cuda")
        for j in range(nsub):
            lo, hi = j * nb, min(N, (j + 1) * nb)
            b0 = dts[lo]
            d32[lo:hi] = (dts[lo:hi] - b0).to(torch.int32)
            base[j] = b0.item()
        ts.copy_(dts)
        key.copy_(dkey)
        price.copy_(dpr)
        ts32.copy_(d32)
        if key16 is not None:
            key16.copy_(dkey.to(torch.int16))  # (the ids as 16 bits: uint16 on the C side)
        host.append((ts, key, price, ts32, base, key16))
        del dts, dkey, dpr, d32
    torch.cuda.synchronize()

    def batch(s, j):
        ts, key, price, ts32, base, key16 = host[s]
        lo, hi = j * nb, min(N, (j + 1) * nb)
        colp = (ctypes.c_void_p * 1)(price.data_ptr() + lo * 4)
        b = native.ShpBatch(hi - lo, ts.data_ptr() + lo * 8, key.data_ptr() + lo * 4, None,
                            ctypes.cast(colp, ctypes.c_void_p), None)
        return b, colp, ts32.data_ptr() + lo * 4, int(base[j]), (key16.data_ptr() + lo * 2 if key16 is not None else None)

    def check(rc, e):
        if rc != 0:
            raise native.ShpError(rc, L.shp_last_error(e.h).decode())

    res = {}
    modes = ("serial", "pipelined", "pipelined_ts32") + (("pipelined_narrow",) if K <= 65536 else ())
    if only:
        modes = tuple(m for m in modes if m in only.split(","))
    for mode in modes:
        e = native.HipEngine(cq.program_json(), 0, max_keys=K, max_batch=nb, max_matches=int(nb * 1.1) + 4096,
                             device=device, force_general=force, match_layout=native.LAYOUT_COMPACT)
        try:
            def stage(s, j):
                b, colp, p32, b0, p16 = batch(s, j)
                if mode == "pipelined_narrow":
                    check(L.shp_stage_batch_narrow(e.h, ctypes.byref(b), b0, p32, p16), e)
                elif mode == "pipelined_ts32":
                    check(L.shp_stage_batch_ts32(e.h, ctypes.byref(b), b0, p32), e)
                else:
                    check(L.shp_stage_batch(e.h, ctypes.byref(b)), e)

            def one_step(s):
                m = 0
                mt = native.ShpMatches()
                if mode == "serial":
                    for j in range(nsub):
                        b, colp, _, _, _ = batch(s, j)
                        check(L.shp_push_batch_compact(e.h, ctypes.byref(b), ctypes.byref(mt)), e)
                        m += mt.m
                    return m
                for j in range(nsub):
                    if j + 1 < nsub:
                        stage(s, j + 1)  # batch j+1's copies run while batch j runs
                    elif s + 1 < total_steps:
                        stage(s + 1, 0)  # the next step's first batch
                    check(L.shp_run_staged(e.h, ctypes.byref(mt)), e)
                    m += mt.m
                return m
            if mode != "serial":
                stage(0, 0)
            one_step(0)  # warm-up
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            m = 0
            for s in range(1, total_steps):
                m += one_step(s)
            el = time.perf_counter() - t0
            inb = {"pipelined_ts32": 12, "pipelined_narrow": 10}.get(mode, 16)
            ev = N * steps
            res[mode] = {"value": ev / el, "ms_per_step": el / steps * 1e3, "matches_per_s": m / el,
                         "h2d_bytes_per_event": inb, "d2h_bytes_per_match": per,
                         "pcie_gbs": (ev * inb + m * per) / el / 1e9}
        finally:
            e.close()
    # the host link alone: one page-locked 1 GiB H2D copy (torch), for scale
    hb = torch.empty(1 << 28, dtype=torch.float32, pin_memory=True)
    db = torch.empty(1 << 28, dtype=torch.float32, device="cuda")
    db.copy_(hb, non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(4):
        db.copy_(hb, non_blocking=True)
    torch.cuda.synchronize()
    h2d = 4 * (1 << 30) / (time.perf_counter() - t0) / 1e9
    del hb, db, host
    best = max([m for m in modes if m != "serial"] or list(modes), key=lambda k: res[k]["value"])
    return {"value": res[best]["value"], "unit": "events/s", "ms_per_step": res[best]["ms_per_step"],
            "mode": best, "batch_events": nb, "batches_per_step": nsub, "steps": steps, "forms": res,
            "h2d_copy_gbs": h2d,
            "what": "page-locked host SoA columns -> shp_stage_batch[_ts32|_narrow] / shp_run_staged -> compact records "
                    "in page-locked host memory; serial = shp_push_batch_compact per batch; ts32 = 4-byte ts offsets "
                    "(12 B/event), narrow = also 2-byte key ids (10 B/event)"}


def _lib_sha16(path):
    import hashlib
    try:
        return hashlib.sha256(open(path, "rb").read()).hexdigest()[:16]
    except OSError:
        return None


def _sweep_shape(cq, device, keys):
    """Does the engine pick the sweep path (and so allow the PAIRS layout) for this query?"""
    from siddhi_amd import native
    e = native.HipEngine(cq.program_json(), 0, max_keys=keys, max_batch=16, device=device)
    try:
        return e.path == 2
    finally:
        e.close()


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(cq, sample, keys, config=2, threads=0):
    """The oracle (C++ restatement of the reference semantics, oracle/liboracle.so) on the box's
    host cores, two ways: one thread over the first `sample` events of the
    stream, and key-sharded over T threads (one oracle engine per shard, keys k % T == t; each
    ctypes call releases the GIL) over the first T * `sample` events.  The sharded rate is the
    reported value; the single-thread run sits beside it."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from diff_util import run, small_stream
    from oracle.oracle import OracleEngine
    if threads <= 0:
        threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    threads = max(1, min(threads, os.cpu_count() or 1, 64, keys))
    g1 = small_stream(config, sample, keys)
    e = OracleEngine(cq.program_json(), 0)
    t = time.perf_counter()
    mb = run(e, cq, g1)
    dt1 = time.perf_counter() - t
    single = {"value": sample / dt1, "cores": 1, "events": sample, "matches": int(len(mb["key"])), "s": dt1}
    del e, mb, g1
    total = sample * threads
    g = small_stream(config, total, keys)
    shard = g["key"] % threads
    parts = [{k: v[shard == r] for k, v in g.items()} for r in range(threads)]
    del g, shard
    engines = [OracleEngine(cq.program_json(), 0) for _ in range(threads)]
    out = [None] * threads

    def work(r):
        out[r] = run(engines[r], cq, parts[r])

    ths = [threading.Thread(target=work, args=(r,)) for r in range(threads)]
    t = time.perf_counter()
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    dtn = time.perf_counter() - t
    nm = sum(len(o["key"]) for o in out)
    return {"value": total / dtn, "unit": "events/s", "cores": threads, "kind": "port",
            "cpu_model": _cpu_model(), "cpus_visible": os.cpu_count(),
            "sample": f"first {total} events of the C{config} stream ({keys} keys) key-sharded over {threads} "
                      f"threads (one oracle/liboracle.so engine per shard, key % {threads}), {nm} matches, "
                      f"{dtn:.1f} s; single thread: first {sample} events, {single['value']:.3e} events/s",
            "single_thread": single}


if __name__ == "__main__":
    main()
