"""ctypes binding of libsiddhi_hip.so (include/siddhi_hip.h).

This is the product path: there is no CPU fallback.  Loading fails loudly when
the library is missing, and engine creation fails when no HIP device is present.
"""
from __future__ import annotations

import ctypes
import json
import sys
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libsiddhi_hip.so")
# diagnostics only (tools/sweep_probe.py): load the stamps build instead of the product library
if os.environ.get("SIDDHI_HIP_DIAG_LIB"):
    LIB_PATH = os.environ["SIDDHI_HIP_DIAG_LIB"]
_lib = None

SHP_ERRORS = {-1: "SHP_ERR_ARG", -2: "SHP_ERR_UNSUPPORTED", -3: "SHP_ERR_CAPACITY",
              -4: "SHP_ERR_OUTPUT", -5: "SHP_ERR_DEVICE", -6: "SHP_ERR_KEYS"}

SYMBOLS = ["shp_engine_create", "shp_push_batch", "shp_push_batch_device", "shp_fetch_matches", "shp_push_batch_compact", "shp_engine_oldest_live_seq",
           "shp_engine_next_due", "shp_stage_batch", "shp_stage_batch_ts32", "shp_stage_batch_narrow", "shp_run_staged",
           "shp_advance_clock", "shp_engine_num_states", "shp_engine_state_stream", "shp_engine_path", "shp_last_kernel_ms", "shp_engine_stat",
           "shp_last_error", "shp_engine_destroy", "shp_synth_fill", "shp_dev_alloc", "shp_dev_free",
           "shp_dev_to_host", "shp_host_alloc", "shp_host_free", "shp_host_register",
           "shp_host_unregister", "shp_snapshot", "shp_restore", "shp_snapshot_describe", "shp_shard_workspace_bytes",
           "shp_shard_partition", "shp_shard_unpack", "shp_shard_partition_soa", "shp_comm_id",
           "shp_group_create", "shp_group_create_rank", "shp_group_push", "shp_group_stage", "shp_group_run",
           "shp_group_fetch_matches", "shp_group_gather_matches",
           "shp_group_local_engines", "shp_group_engine", "shp_group_last_error", "shp_group_destroy",
           "shp_dict_create", "shp_dict_intern", "shp_dict_size", "shp_dict_string", "shp_dict_destroy",
           "shp_compile_siddhiql", "shp_siddhiql_queries", "shp_compile_last_error", "shp_engine_create_siddhiql"]


class ShpConfig(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("max_keys", ctypes.c_int32), ("max_batch", ctypes.c_int64),
                ("max_matches", ctypes.c_int64), ("start_clock", ctypes.c_int64),
                ("force_general", ctypes.c_int32), ("profile_kernels", ctypes.c_int32),
                ("match_layout", ctypes.c_int32)]

LAYOUT_FULL, LAYOUT_PAIRS, LAYOUT_AGG, LAYOUT_PAIRS32, LAYOUT_CHAIN32, LAYOUT_COMPACT = 0, 1, 2, 3, 4, 5


class ShpBatch(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int64), ("ts", ctypes.c_void_p), ("key", ctypes.c_void_p),
                ("stream", ctypes.c_void_p), ("cols", ctypes.c_void_p), ("nulls", ctypes.c_void_p),
                ("clock", ctypes.c_void_p), ("seq", ctypes.c_void_p)]


class ShpMatches(ctypes.Structure):
    _fields_ = [("m", ctypes.c_int64), ("num_states", ctypes.c_int32),
                ("key", ctypes.c_void_p), ("ts", ctypes.c_void_p), ("type", ctypes.c_void_p),
                ("pos", ctypes.c_void_p), ("ref_off", ctypes.c_void_p), ("slot_len", ctypes.c_void_p),
                ("refs", ctypes.c_void_p), ("layout", ctypes.c_int32), ("agg", ctypes.c_void_p)]


class ShpError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{SHP_ERRORS.get(code, code)}: {msg}")
        self.code = code


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: run `python -m siddhi_amd.build` "
                              f"(there is no CPU fallback for the state path)")
        # PyTorch-ROCm ships its own HIP runtime. When the caller uses torch as well, its runtime
        # must initialise the device first: the two coexist in that order, not the other.
        torch = sys.modules.get("torch")
        if torch is not None and hasattr(torch, "cuda"):
            torch.cuda.is_available()
        L = ctypes.CDLL(LIB_PATH)
        L.shp_engine_create.argtypes = [ctypes.c_char_p, ctypes.POINTER(ShpConfig), ctypes.POINTER(ctypes.c_void_p)]
        for f in ("shp_push_batch", "shp_push_batch_device"):
            getattr(L, f).argtypes = [ctypes.c_void_p, ctypes.POINTER(ShpBatch), ctypes.POINTER(ShpMatches)]
        L.shp_fetch_matches.argtypes = [ctypes.c_void_p, ctypes.POINTER(ShpMatches)]
        L.shp_push_batch_compact.argtypes = [ctypes.c_void_p, ctypes.POINTER(ShpBatch), ctypes.POINTER(ShpMatches)]
        L.shp_engine_oldest_live_seq.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64)]
        L.shp_stage_batch.argtypes = [ctypes.c_void_p, ctypes.POINTER(ShpBatch)]
        L.shp_stage_batch_ts32.argtypes = [ctypes.c_void_p, ctypes.POINTER(ShpBatch), ctypes.c_int64, ctypes.c_void_p]
        L.shp_stage_batch_narrow.argtypes = [ctypes.c_void_p, ctypes.POINTER(ShpBatch), ctypes.c_int64, ctypes.c_void_p,
                                             ctypes.c_void_p]
        L.shp_run_staged.argtypes = [ctypes.c_void_p, ctypes.POINTER(ShpMatches)]
        L.shp_engine_next_due.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64)]
        L.shp_advance_clock.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ShpMatches)]
        L.shp_engine_num_states.argtypes = [ctypes.c_void_p]
        L.shp_engine_state_stream.argtypes = [ctypes.c_void_p, ctypes.c_int32]
        L.shp_engine_path.argtypes = [ctypes.c_void_p]
        L.shp_last_kernel_ms.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
        L.shp_last_kernel_ms.restype = ctypes.c_double
        L.shp_engine_stat.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
        L.shp_engine_stat.restype = ctypes.c_int64
        L.shp_last_error.argtypes = [ctypes.c_void_p]
        L.shp_last_error.restype = ctypes.c_char_p
        L.shp_engine_destroy.argtypes = [ctypes.c_void_p]
        L.shp_synth_fill.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                     ctypes.c_int] + [ctypes.c_void_p] * 6
        L.shp_dev_alloc.restype = ctypes.c_void_p
        L.shp_dev_alloc.argtypes = [ctypes.c_int64]
        L.shp_dev_free.argtypes = [ctypes.c_void_p]
        L.shp_dev_to_host.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
        L.shp_host_alloc.restype = ctypes.c_void_p
        L.shp_host_alloc.argtypes = [ctypes.c_int64]
        L.shp_host_free.argtypes = [ctypes.c_void_p]
        L.shp_host_register.argtypes = [ctypes.c_void_p, ctypes.c_int64]
        L.shp_host_unregister.argtypes = [ctypes.c_void_p]
        L.shp_snapshot.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t)]
        L.shp_restore.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        L.shp_snapshot_describe.restype = ctypes.c_int64
        L.shp_snapshot_describe.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                            ctypes.c_size_t]
        L.shp_shard_workspace_bytes.restype = ctypes.c_int64
        L.shp_shard_workspace_bytes.argtypes = [ctypes.c_int64, ctypes.c_int]
        L.shp_shard_partition.argtypes = [ctypes.c_int64] + [ctypes.c_void_p] * 4 + [ctypes.c_int] + \
            [ctypes.c_void_p] * 4
        L.shp_shard_unpack.argtypes = [ctypes.c_int64] + [ctypes.c_void_p] * 6
        L.shp_shard_partition_soa.argtypes = [ctypes.c_int64] + [ctypes.c_void_p] * 4 + [ctypes.c_int] + \
            [ctypes.c_void_p] * 7
        L.shp_comm_id.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        L.shp_group_create.argtypes = [ctypes.c_char_p, ctypes.POINTER(ShpConfig), ctypes.c_int32, ctypes.c_void_p,
                                       ctypes.POINTER(ctypes.c_void_p)]
        L.shp_group_create_rank.argtypes = [ctypes.c_char_p, ctypes.POINTER(ShpConfig), ctypes.c_int32, ctypes.c_int32,
                                            ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]
        L.shp_group_push.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.shp_group_stage.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.shp_group_run.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.shp_group_fetch_matches.argtypes = [ctypes.c_void_p, ctypes.POINTER(ShpMatches)]
        L.shp_group_gather_matches.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(ShpMatches)]
        L.shp_group_local_engines.argtypes = [ctypes.c_void_p]
        L.shp_group_engine.restype = ctypes.c_void_p
        L.shp_group_engine.argtypes = [ctypes.c_void_p, ctypes.c_int32]
        L.shp_group_last_error.restype = ctypes.c_char_p
        L.shp_group_last_error.argtypes = [ctypes.c_void_p]
        L.shp_group_destroy.argtypes = [ctypes.c_void_p]
        L.shp_dict_create.restype = ctypes.c_void_p
        L.shp_dict_create.argtypes = [ctypes.c_int32]
        L.shp_dict_intern.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int64]
        L.shp_dict_intern.restype = ctypes.c_int32
        L.shp_dict_size.argtypes = [ctypes.c_void_p]
        L.shp_dict_size.restype = ctypes.c_int32
        L.shp_dict_string.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_char_p, ctypes.c_size_t]
        L.shp_dict_string.restype = ctypes.c_int64
        L.shp_dict_destroy.argtypes = [ctypes.c_void_p]
        L.shp_compile_siddhiql.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_char_p,
                                           ctypes.c_size_t]
        L.shp_compile_siddhiql.restype = ctypes.c_int64
        L.shp_siddhiql_queries.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t]
        L.shp_siddhiql_queries.restype = ctypes.c_int64
        L.shp_compile_last_error.restype = ctypes.c_char_p
        L.shp_engine_create_siddhiql.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_void_p,
                                                 ctypes.POINTER(ShpConfig), ctypes.POINTER(ctypes.c_void_p)]
        _lib = L
    return _lib


def _arr(ptr, n, dtype):
    if n == 0 or not ptr:
        return np.zeros(0, dtype)
    buf = (ctypes.c_char * (n * np.dtype(dtype).itemsize)).from_address(ptr)
    return np.frombuffer(buf, dtype=dtype, count=n).copy()


def matches_to_numpy(mt: ShpMatches):
    m, S = mt.m, mt.num_states
    if mt.layout == LAYOUT_AGG:  # one output row per match: (partition key, aggregate value)
        return {"key": _arr(mt.key, m, np.int32), "agg": _arr(mt.agg, m, np.float64)}
    slot_len = _arr(mt.slot_len, m * S, np.int16).reshape(m, S).astype(np.int32)
    nrefs = int(slot_len.sum())
    return {
        "key": _arr(mt.key, m, np.int32), "ts": _arr(mt.ts, m, np.int64), "type": _arr(mt.type, m, np.int8),
        "pos": _arr(mt.pos, m, np.int64), "slot_len": slot_len, "refs": _arr(mt.refs, nrefs, np.int64),
    }


_TYPE_BYTES = {"int": 4, "long": 8, "float": 4, "double": 8, "bool": 1, "string": 4}


def _column_bytes(program_json: str):
    """Element size of each program column (shp_batch.cols holds one pointer per column, in order)."""
    return [_TYPE_BYTES[c["type"]] for c in json.loads(program_json)["columns"]]


def _check_columns(cols, nulls, col_bytes, n):
    """The C-ABI reads one column pointer (and one null pointer) per program column: a short list
    would make it read past the caller's pointer array, so refuse it here."""
    if len(cols) != len(col_bytes) or len(nulls) != len(col_bytes):
        raise ValueError(f"the program has {len(col_bytes)} columns; got {len(cols)} columns, {len(nulls)} null arrays")
    for i, (c, b) in enumerate(zip(cols, col_bytes)):
        if c.itemsize != b or len(c) < n:
            raise ValueError(f"column {i}: need {n} elements of {b} bytes, got {len(c)} of {c.itemsize}")
    for i, m in enumerate(nulls):
        if m is not None and len(m) < n:
            raise ValueError(f"null array {i}: need {n} elements, got {len(m)}")


class NativeDictionary:
    """A string dictionary held by the library (shp_dict): the SiddhiQL lowering interns filter
    constants in it, and the host encodes string column values with the same ids.  Callable like
    query.compiler.Dictionary (str -> id)."""

    def __init__(self, max_ids: int = 0):
        self.h = lib().shp_dict_create(int(max_ids))

    def __call__(self, s: str) -> int:
        b = s.encode()
        i = lib().shp_dict_intern(self.h, b, len(b))
        if i < 0:
            raise ShpError(i, "string dictionary full")
        return i

    @property
    def strings(self):
        L = lib()
        out = []
        for i in range(L.shp_dict_size(self.h)):
            n = L.shp_dict_string(self.h, i, None, 0)
            b = ctypes.create_string_buffer(n + 1)
            L.shp_dict_string(self.h, i, b, n + 1)
            out.append(b.raw[:n].decode())
        return out

    def __del__(self):
        try:
            if getattr(self, "h", None):
                lib().shp_dict_destroy(self.h)
                self.h = None
        except Exception:
            pass


def compile_siddhiql(app_text: str, query_name, ndict: NativeDictionary) -> str:
    """The library's lowering of one query of a SiddhiQL app to its program JSON."""
    L = lib()
    q = None if query_name is None else query_name.encode()
    n = L.shp_compile_siddhiql(app_text.encode(), q, ndict.h, None, 0)
    if n < 0:
        raise ShpError(int(n), L.shp_compile_last_error().decode())
    buf = ctypes.create_string_buffer(n + 1)
    L.shp_compile_siddhiql(app_text.encode(), q, ndict.h, buf, n + 1)
    return buf.raw[:n].decode()


class HipEngine:
    """One engine per query (libsiddhi_hip.so). Same interface as the test oracle."""

    def __init__(self, program_json: str, start_clock: int = 0, max_keys: int = 1 << 16,
                 max_batch: int = 1 << 20, max_matches: int = 0, device: int = 0, force_general: int = 0,
                 profile_kernels: bool = False, match_layout: int = LAYOUT_FULL, siddhiql=None):
        """force_general: 0 auto path, 1 general NFA lanes only, 2 no sweep path, 3 sweep whenever possible.
        siddhiql = (app_text, query_name, NativeDictionary): the engine is created from the SiddhiQL text
        through shp_engine_create_siddhiql (the library lowers it); program_json is then ignored."""
        L = lib()
        cfg = ShpConfig(device, max_keys, max_batch, max_matches, int(start_clock), int(force_general),
                        int(profile_kernels), int(match_layout))
        h = ctypes.c_void_p()
        if siddhiql is not None:
            app_text, qname, ndict = siddhiql
            program_json = compile_siddhiql(app_text, qname, ndict)
            rc = L.shp_engine_create_siddhiql(app_text.encode(), None if qname is None else qname.encode(), ndict.h,
                                              ctypes.byref(cfg), ctypes.byref(h))
        else:
            rc = L.shp_engine_create(program_json.encode(), ctypes.byref(cfg), ctypes.byref(h))
        if rc != 0:
            raise ShpError(rc, "shp_engine_create failed (see stderr)")
        self.program_json = program_json
        self.h = h
        self.S = L.shp_engine_num_states(h)
        self.col_bytes = _column_bytes(program_json)
        self.max_batch = max_batch
        self.max_keys = max_keys
        self.layout = int(match_layout)
        self._pending = None

    @property
    def path(self):
        return lib().shp_engine_path(self.h)

    @property
    def state_streams(self):
        """shp_engine_state_stream per state: the receiver (program stream index) of each state, in
        MetaStateEvent order."""
        return [lib().shp_engine_state_stream(self.h, s) for s in range(self.S)]

    def _check(self, rc):
        if rc != 0:
            raise ShpError(rc, lib().shp_last_error(self.h).decode())

    def push(self, ts, key, stream, cols, nulls, clock=None, seq=None):
        """Host arrays; clock / seq: the optional shp_batch columns (global playback clock, sequence numbers)."""
        L = lib()
        n = len(ts)
        out_all = []
        for lo in range(0, max(n, 1), self.max_batch):
            hi = min(n, lo + self.max_batch)
            if hi <= lo:
                break
            t = np.ascontiguousarray(ts[lo:hi], np.int64)
            k = np.ascontiguousarray(key[lo:hi], np.int32)
            s = np.ascontiguousarray(stream[lo:hi], np.int32)
            cs = [np.ascontiguousarray(c[lo:hi]) for c in cols]
            ns = [None if m is None else np.ascontiguousarray(m[lo:hi], np.uint8) for m in nulls]
            _check_columns(cs, ns, self.col_bytes, hi - lo)
            colp = (ctypes.c_void_p * max(1, len(cs)))(*[c.ctypes.data for c in cs])
            nulp = (ctypes.c_void_p * max(1, len(ns)))(*[0 if m is None else m.ctypes.data for m in ns])
            ck = None if clock is None else np.ascontiguousarray(clock[lo:hi], np.int64)
            sq = None if seq is None else np.ascontiguousarray(seq[lo:hi], np.int64)
            b = ShpBatch(hi - lo, t.ctypes.data, k.ctypes.data, s.ctypes.data,
                         ctypes.cast(colp, ctypes.c_void_p), ctypes.cast(nulp, ctypes.c_void_p),
                         None if ck is None else ck.ctypes.data, None if sq is None else sq.ctypes.data)
            mt = ShpMatches()
            self._check(L.shp_push_batch(self.h, ctypes.byref(b), ctypes.byref(mt)))
            out_all.append(matches_to_numpy(mt))
        self._pending = _concat(out_all, self._pending, self.S, self.layout)

    def push_compact(self, ts, key, stream, cols, nulls, clock=None, seq=None):
        """One push of host arrays through shp_push_batch_compact (the Java binding's push): the
        records come back in the layout the engine produced them in, without expansion.  Returns
        {"layout": L, "m": m, "words": uint32 array} for PAIRS32 (2 words per match) / CHAIN32 (1)
        / PAIRS (4), or the FULL / AGG dict of fetch() with its "layout"."""
        L = lib()
        n = len(ts)
        if n > self.max_batch:
            raise ValueError("push_compact: batch larger than max_batch")
        t = np.ascontiguousarray(ts, np.int64)
        k = np.ascontiguousarray(key, np.int32)
        s = np.ascontiguousarray(stream, np.int32)
        cs = [np.ascontiguousarray(c) for c in cols]
        ns = [None if m is None else np.ascontiguousarray(m, np.uint8) for m in nulls]
        _check_columns(cs, ns, self.col_bytes, n)
        colp = (ctypes.c_void_p * max(1, len(cs)))(*[c.ctypes.data for c in cs])
        nulp = (ctypes.c_void_p * max(1, len(ns)))(*[0 if m is None else m.ctypes.data for m in ns])
        ck = None if clock is None else np.ascontiguousarray(clock, np.int64)
        sq = None if seq is None else np.ascontiguousarray(seq, np.int64)
        b = ShpBatch(n, t.ctypes.data, k.ctypes.data, s.ctypes.data, ctypes.cast(colp, ctypes.c_void_p),
                     ctypes.cast(nulp, ctypes.c_void_p), None if ck is None else ck.ctypes.data,
                     None if sq is None else sq.ctypes.data)
        mt = ShpMatches()
        self._check(L.shp_push_batch_compact(self.h, ctypes.byref(b), ctypes.byref(mt)))
        lay = int(mt.layout)
        if lay in (LAYOUT_PAIRS32, LAYOUT_CHAIN32, LAYOUT_PAIRS):
            per = {LAYOUT_PAIRS32: 2, LAYOUT_CHAIN32: 1, LAYOUT_PAIRS: 4}[lay]
            return {"layout": lay, "m": int(mt.m), "words": _arr(mt.refs, int(mt.m) * per, np.uint32)}
        out = matches_to_numpy(mt)
        out["layout"] = lay
        out["m"] = int(mt.m)
        return out

    def stage(self, ts, key, stream, cols, nulls, clock=None, seq=None, ts32=None, ts_base=0, key16=None):
        """shp_stage_batch (or, with ts32 = int32 offsets from ts_base, shp_stage_batch_ts32; with key16 =
        uint16 key ids too, shp_stage_batch_narrow): the H2D copies of one host batch, enqueued on the
        engine's copy stream.  The arrays are held until the shp_run_staged that consumes them
        (page-locked arrays make the copies asynchronous)."""
        L = lib()
        n = len(ts) if ts32 is None else len(ts32)
        if n > self.max_batch:
            raise ValueError("stage: batch larger than max_batch")
        keep = [np.ascontiguousarray(x) if x is not None else None for x in (ts, key, stream, clock, seq, ts32, key16)]
        t, k, s_, ck, sq, t32, k16 = keep
        cs = [np.ascontiguousarray(c) for c in cols]
        ns = [None if m is None else np.ascontiguousarray(m, np.uint8) for m in nulls]
        _check_columns(cs, ns, self.col_bytes, n)
        colp = (ctypes.c_void_p * max(1, len(cs)))(*[c.ctypes.data for c in cs])
        nulp = (ctypes.c_void_p * max(1, len(ns)))(*[0 if m is None else m.ctypes.data for m in ns])
        ptr = lambda a: None if a is None else a.ctypes.data  # noqa: E731
        b = ShpBatch(n, ptr(t), ptr(k), ptr(s_), ctypes.cast(colp, ctypes.c_void_p), ctypes.cast(nulp, ctypes.c_void_p),
                     ptr(ck), ptr(sq))
        if k16 is not None:
            self._check(L.shp_stage_batch_narrow(self.h, ctypes.byref(b), int(ts_base), ptr(t32), ptr(k16)))
        elif t32 is None:
            self._check(L.shp_stage_batch(self.h, ctypes.byref(b)))
        else:
            self._check(L.shp_stage_batch_ts32(self.h, ctypes.byref(b), int(ts_base), ptr(t32)))
        if not hasattr(self, "_staged"):
            self._staged = []
        self._staged.append((keep, cs, ns, colp, nulp))

    def run_staged(self):
        """shp_run_staged: the oldest staged batch; records as push_compact returns them."""
        mt = ShpMatches()
        try:
            self._check(lib().shp_run_staged(self.h, ctypes.byref(mt)))
        finally:
            if getattr(self, "_staged", None):
                self._staged.pop(0)
        lay = int(mt.layout)
        if lay in (LAYOUT_PAIRS32, LAYOUT_CHAIN32, LAYOUT_PAIRS):
            per = {LAYOUT_PAIRS32: 2, LAYOUT_CHAIN32: 1, LAYOUT_PAIRS: 4}[lay]
            return {"layout": lay, "m": int(mt.m), "words": _arr(mt.refs, int(mt.m) * per, np.uint32)}
        out = matches_to_numpy(mt)
        out["layout"] = lay
        out["m"] = int(mt.m)
        return out

    def oldest_live_seq(self) -> int:
        """shp_engine_oldest_live_seq: the oldest event an open partial of the committed state holds."""
        v = ctypes.c_int64()
        self._check(lib().shp_engine_oldest_live_seq(self.h, ctypes.byref(v)))
        return int(v.value)

    def next_due(self):
        """shp_engine_next_due: the earliest due time of any key's timer queue, or None."""
        v = ctypes.c_int64()
        rc = lib().shp_engine_next_due(self.h, ctypes.byref(v))
        if rc < 0:
            self._check(rc)
        return int(v.value) if rc == 1 else None

    def advance(self, now):
        mt = ShpMatches()
        self._check(lib().shp_advance_clock(self.h, int(now), ctypes.byref(mt)))
        self._pending = _concat([matches_to_numpy(mt)], self._pending, self.S, self.layout)

    def fetch(self):
        out = self._pending if self._pending is not None else _concat([], None, self.S, self.layout)
        self._pending = None
        return out

    def snapshot(self) -> bytes:
        """Engine state as bytes (shp_snapshot)."""
        buf, n = ctypes.c_void_p(), ctypes.c_size_t()
        self._check(lib().shp_snapshot(self.h, ctypes.byref(buf), ctypes.byref(n)))
        return ctypes.string_at(buf, n.value)

    def restore(self, blob: bytes):
        """Load a snapshot taken from an engine of the same query (shp_restore)."""
        b = ctypes.create_string_buffer(blob, len(blob))
        self._check(lib().shp_restore(self.h, b, len(blob)))

    def describe(self, blob: bytes) -> dict:
        """A snapshot in the reference's State.snapshot() key names (shp_snapshot_describe)."""
        import json
        b = ctypes.create_string_buffer(blob, len(blob))
        need = lib().shp_snapshot_describe(self.h, b, len(blob), None, 0)
        if need < 0:
            raise ShpError(int(need), lib().shp_last_error(self.h).decode())
        out = ctypes.create_string_buffer(need + 1)
        lib().shp_snapshot_describe(self.h, b, len(blob), out, need + 1)
        return json.loads(out.value.decode())

    def kernel_ms(self, which="total"):
        return lib().shp_last_kernel_ms(self.h, which.encode())

    def stat(self, which):
        """shp_engine_stat: "pushes", "lean_pushes", "lean_fallbacks" or "labs_fallbacks"."""
        return int(lib().shp_engine_stat(self.h, which.encode()))

    def close(self):
        if getattr(self, "h", None):
            lib().shp_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _concat(parts, prev, S, layout=LAYOUT_FULL):
    parts = ([prev] if prev is not None else []) + list(parts)
    if not parts and layout == LAYOUT_AGG:
        return {"key": np.zeros(0, np.int32), "agg": np.zeros(0, np.float64)}
    if not parts:
        return {"key": np.zeros(0, np.int32), "ts": np.zeros(0, np.int64), "type": np.zeros(0, np.int8),
                "pos": np.zeros(0, np.int64), "slot_len": np.zeros((0, S), np.int32),
                "refs": np.zeros(0, np.int64)}
    return {k: np.concatenate([p[k] for p in parts]) for k in parts[0]}


COMM_ID_BYTES = 128


def comm_id() -> bytes:
    """RCCL unique id for a per-process group (rank 0 makes it; broadcast it to the other ranks)."""
    buf = ctypes.create_string_buffer(COMM_ID_BYTES)
    rc = lib().shp_comm_id(buf, COMM_ID_BYTES)
    if rc != 0:
        raise ShpError(rc, "shp_comm_id failed")
    return buf.raw


class HipGroup:
    """Key-sharded engines (shp_group_*): in one process over `devices`, or one member per process
    (rank, comm id).  push() takes one slice per local rank as device tensors (torch) or host arrays."""

    def __init__(self, program_json: str, start_clock: int = 0, max_keys: int = 1 << 16, max_batch: int = 1 << 20,
                 max_matches: int = 0, devices=None, world: int = 0, rank: int = 0, comm: bytes = None,
                 device: int = 0, force_general: int = 0, profile_kernels: bool = False,
                 match_layout: int = LAYOUT_FULL):
        L = lib()
        cfg = ShpConfig(device, max_keys, max_batch, max_matches, int(start_clock), int(force_general),
                        int(profile_kernels), int(match_layout))
        h = ctypes.c_void_p()
        if comm is None:
            devs = list(devices or [0])
            arr = (ctypes.c_int32 * len(devs))(*devs)
            rc = L.shp_group_create(program_json.encode(), ctypes.byref(cfg), len(devs), arr, ctypes.byref(h))
            self.world = len(devs)
        else:
            rc = L.shp_group_create_rank(program_json.encode(), ctypes.byref(cfg), world, rank, comm, ctypes.byref(h))
            self.world = world
        if rc != 0:
            raise ShpError(rc, "shp_group_create failed (see stderr)")
        self.h = h
        self.nlocal = L.shp_group_local_engines(h)
        self.layout = int(match_layout)

    def _check(self, rc):
        if rc != 0:
            raise ShpError(rc, lib().shp_group_last_error(self.h).decode())

    def _batches(self, slices):
        """slices: per local rank (ts, key, stream-or-None, [cols]) or (..., [cols], [nulls-or-None])."""
        arr = (ShpBatch * self.nlocal)()
        keep = []
        for i, sl in enumerate(slices):
            ts, key, stream, cols = sl[:4]
            nulls = sl[4] if len(sl) > 4 else None
            colp = (ctypes.c_void_p * max(1, len(cols)))(*[c.data_ptr() for c in cols])
            keep.append(colp)
            nulp = None
            if nulls is not None:
                nulp = (ctypes.c_void_p * max(1, len(cols)))(*[0 if m is None else m.data_ptr() for m in nulls])
                keep.append(nulp)
            arr[i] = ShpBatch(ts.numel(), ts.data_ptr(), key.data_ptr(), None if stream is None else stream.data_ptr(),
                              ctypes.cast(colp, ctypes.c_void_p),
                              None if nulp is None else ctypes.cast(nulp, ctypes.c_void_p))
        return arr, keep

    def push_device(self, slices):
        """slices: per local rank, (ts, key, stream-or-None, [cols]) torch tensors on that rank's device."""
        arr, keep = self._batches(slices)
        counts = (ctypes.c_int64 * self.nlocal)()
        self._check(lib().shp_group_push(self.h, arr, counts))
        return list(counts)

    def stage_device(self, slices):
        """Split + exchange one batch into a receive slot (the inputs may be reused once this returns
        only after the next run(): the exchange reads them asynchronously)."""
        arr, keep = self._batches(slices)
        self._check(lib().shp_group_stage(self.h, arr))
        return keep

    def run(self):
        counts = (ctypes.c_int64 * self.nlocal)()
        self._check(lib().shp_group_run(self.h, counts))
        return list(counts)

    def fetch(self):
        mt = ShpMatches()
        self._check(lib().shp_group_fetch_matches(self.h, ctypes.byref(mt)))
        return matches_to_numpy(mt)

    def gather(self, root=0):
        """shp_group_gather_matches: every rank's matches of the last push at `root` (collective)."""
        mt = ShpMatches()
        self._check(lib().shp_group_gather_matches(self.h, int(root), ctypes.byref(mt)))
        return matches_to_numpy(mt)

    def engine_ms(self, i, which="total"):
        e = lib().shp_group_engine(self.h, i)
        return lib().shp_last_kernel_ms(e, which.encode())

    def engine_stat(self, i, which):
        """shp_engine_stat of local engine i (shp_group_engine)."""
        return lib().shp_engine_stat(lib().shp_group_engine(self.h, i), which.encode())

    def close(self):
        if getattr(self, "h", None):
            lib().shp_group_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
