"""ctypes binding for liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module.  The oracle is the CPU restatement of the reference semantics
(oracle/oracle.cpp) used as the parity checker; it is never the product path.
"""
from __future__ import annotations

import ctypes
import json
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liboracle.so")
_lib = None


def build(force=False):
    if force or not os.path.exists(_LIB) or \
            os.path.getmtime(_LIB) < os.path.getmtime(os.path.join(_HERE, "oracle.cpp")):
        subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB)
        L.oracle_create.restype = ctypes.c_void_p
        L.oracle_create.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_char_p, ctypes.c_int]
        L.oracle_push.argtypes = [ctypes.c_void_p, ctypes.c_int64] + [ctypes.c_void_p] * 5
        L.oracle_push2.argtypes = [ctypes.c_void_p, ctypes.c_int64] + [ctypes.c_void_p] * 7
        L.oracle_advance.argtypes = [ctypes.c_void_p, ctypes.c_int64]
        for f in ("oracle_num_matches", "oracle_num_refs", "oracle_timer_ties", "oracle_dropped_returns",
                  "oracle_oldest_live_seq"):
            getattr(L, f).restype = ctypes.c_int64
            getattr(L, f).argtypes = [ctypes.c_void_p]
        L.oracle_next_due.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64)]
        L.oracle_num_states.argtypes = [ctypes.c_void_p]
        L.oracle_fetch.argtypes = [ctypes.c_void_p] + [ctypes.c_void_p] * 6
        L.oracle_destroy.argtypes = [ctypes.c_void_p]
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


class OracleEngine:
    """Same Python-side interface as siddhi_amd.native.HipEngine."""

    def __init__(self, program_json: str, start_clock: int = 0):
        L = lib()
        err = ctypes.create_string_buffer(512)
        self.h = L.oracle_create(program_json.encode(), int(start_clock), err, 512)
        if not self.h:
            raise ValueError(err.value.decode())
        self.S = L.oracle_num_states(self.h)
        self.ncol = len(json.loads(program_json)["columns"])
        self._keep = []

    def push(self, ts, key, stream, cols, nulls, clock=None, seq=None):
        L = lib()
        n = len(ts)
        if len(cols) != self.ncol or len(nulls) != self.ncol:  # the C side reads one pointer per column
            raise ValueError(f"the program has {self.ncol} columns; got {len(cols)} columns, {len(nulls)} null arrays")
        ts = np.ascontiguousarray(ts, np.int64)
        key = np.ascontiguousarray(key, np.int32)
        stream = np.ascontiguousarray(stream, np.int32)
        cols = [np.ascontiguousarray(c) for c in cols]
        colp = (ctypes.c_void_p * max(1, len(cols)))(*[c.ctypes.data for c in cols])
        nul = [None if m is None else np.ascontiguousarray(m, np.uint8) for m in nulls]
        nulp = (ctypes.c_void_p * max(1, len(nul)))(*[None if m is None else m.ctypes.data for m in nul])
        clock = None if clock is None else np.ascontiguousarray(clock, np.int64)
        seq = None if seq is None else np.ascontiguousarray(seq, np.int64)
        L.oracle_push2(self.h, n, _ptr(ts), _ptr(key), _ptr(stream), ctypes.cast(colp, ctypes.c_void_p),
                       ctypes.cast(nulp, ctypes.c_void_p), _ptr(clock), _ptr(seq))

    def advance(self, now):
        lib().oracle_advance(self.h, int(now))

    def timer_ties(self):
        return lib().oracle_timer_ties(self.h)

    def dropped_returns(self):
        return lib().oracle_dropped_returns(self.h)

    def next_due(self):
        """The earliest head of any key's timer queue (oracle_next_due), or None."""
        v = ctypes.c_int64()
        return int(v.value) if lib().oracle_next_due(self.h, ctypes.byref(v)) == 1 else None

    def oldest_live_seq(self):
        """The oldest event any open partial holds (oracle_oldest_live_seq)."""
        return lib().oracle_oldest_live_seq(self.h)

    def fetch(self):
        L = lib()
        m = L.oracle_num_matches(self.h)
        r = L.oracle_num_refs(self.h)
        out = {
            "key": np.zeros(m, np.int32), "ts": np.zeros(m, np.int64), "type": np.zeros(m, np.int8),
            "pos": np.zeros(m, np.int64), "slot_len": np.zeros((m, self.S), np.int32),
            "refs": np.zeros(max(r, 1), np.int64),
        }
        L.oracle_fetch(self.h, _ptr(out["key"]), _ptr(out["ts"]), _ptr(out["type"]), _ptr(out["pos"]),
                       _ptr(out["slot_len"]), _ptr(out["refs"]))
        out["refs"] = out["refs"][:r]
        return out

    def __del__(self):
        try:
            if getattr(self, "h", None):
                lib().oracle_destroy(self.h)
                self.h = None
        except Exception:
            pass
