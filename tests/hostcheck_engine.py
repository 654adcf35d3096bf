"""Python side of the CPU debug harness for the lane interpreter (tests only).

Runs siddhi_amd/csrc/nfa_lane.h compiled for the host (tests/hostcheck/lane_host.cpp)
with the same driver logic as k_nfa_lanes, so lane-logic parity with the oracle can be
checked without a GPU.  The product path (libsiddhi_hip.so) never loads this.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "hostcheck")
_L = None


def lib():
    global _L
    if _L is None:
        subprocess.check_call(["make", "-s", "-C", HERE])
        L = ctypes.CDLL(os.path.join(HERE, "liblane_host.so"))
        L.hc_create.restype = ctypes.c_void_p
        L.hc_create.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_int]
        L.hc_push.argtypes = [ctypes.c_void_p, ctypes.c_int64] + [ctypes.c_void_p] * 5 + [ctypes.c_int]
        for f in ("hc_num_matches", "hc_num_refs"):
            getattr(L, f).restype = ctypes.c_int64
            getattr(L, f).argtypes = [ctypes.c_void_p]
        L.hc_num_states.argtypes = [ctypes.c_void_p]
        L.hc_fast.argtypes = [ctypes.c_void_p]
        L.hc_fetch.argtypes = [ctypes.c_void_p] + [ctypes.c_void_p] * 6
        L.hc_destroy.argtypes = [ctypes.c_void_p]
        L.hc_set_tier.argtypes = [ctypes.c_void_p, ctypes.c_int]
        _L = L
    return _L


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class HostCheckEngine:
    def __init__(self, program_json, start_clock=0, max_keys=256, tier=0):
        self.h = lib().hc_create(program_json.encode(), int(start_clock), max_keys)
        if not self.h:
            raise ValueError("hc_create failed")
        if tier and lib().hc_set_tier(self.h, int(tier)) != 0:
            raise ValueError("bad capacity tier")
        self.S = lib().hc_num_states(self.h)

    def _push(self, ts, key, stream, cols, nulls, clock_only=0):
        ts = np.ascontiguousarray(ts, np.int64)
        key = np.ascontiguousarray(key, np.int32)
        stream = np.ascontiguousarray(stream, np.int32)
        cols = [np.ascontiguousarray(c) for c in cols]
        nul = [None if m is None else np.ascontiguousarray(m, np.uint8) for m in nulls]
        colp = (ctypes.c_void_p * max(1, len(cols)))(*[c.ctypes.data for c in cols])
        nulp = (ctypes.c_void_p * max(1, len(nul)))(*[None if m is None else m.ctypes.data for m in nul])
        err = lib().hc_push(self.h, len(ts), _p(ts), _p(key), _p(stream), ctypes.cast(colp, ctypes.c_void_p),
                            ctypes.cast(nulp, ctypes.c_void_p), clock_only)
        if err:
            raise RuntimeError(f"lane error {err}")
        self._keep = (ts, key, stream, cols, nul)

    def push(self, ts, key, stream, cols, nulls):
        self._push(ts, key, stream, cols, nulls)

    def advance(self, now):
        self._push(np.array([now]), np.zeros(1, np.int32), np.array([-1], np.int32),
                   [np.zeros(1, np.int64) for _ in range(8)], [None] * 8, clock_only=1)

    def fetch(self):
        L = lib()
        m = L.hc_num_matches(self.h)
        r = L.hc_num_refs(self.h)
        out = {"key": np.zeros(m, np.int32), "ts": np.zeros(m, np.int64), "type": np.zeros(m, np.int8),
               "pos": np.zeros(m, np.int64), "slot_len": np.zeros((m, self.S), np.int32),
               "refs": np.zeros(max(r, 1), np.int64)}
        L.hc_fetch(self.h, _p(out["key"]), _p(out["ts"]), _p(out["type"]), _p(out["pos"]), _p(out["slot_len"]),
                   _p(out["refs"]))
        out["refs"] = out["refs"][:r]
        return out

    def __del__(self):
        try:
            lib().hc_destroy(self.h)
        except Exception:
            pass


_F = None


def fast_lib():
    """tests/hostcheck/libfast_host.so: fast_core.h's per-item bodies (the scan kernels) in host loops."""
    global _F
    if _F is None:
        subprocess.check_call(["make", "-s", "-C", HERE])
        L = ctypes.CDLL(os.path.join(HERE, "libfast_host.so"))
        L.fh_create.restype = ctypes.c_void_p
        L.fh_create.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int64]
        L.fh_push.argtypes = [ctypes.c_void_p, ctypes.c_int64] + [ctypes.c_void_p] * 5
        for f in ("fh_num_matches", "fh_num_refs"):
            getattr(L, f).restype = ctypes.c_int64
            getattr(L, f).argtypes = [ctypes.c_void_p]
        L.fh_num_states.argtypes = [ctypes.c_void_p]
        L.fh_fetch.argtypes = [ctypes.c_void_p] + [ctypes.c_void_p] * 6
        L.fh_destroy.argtypes = [ctypes.c_void_p]
        _F = L
    return _F


class FastHostEngine:
    """The 2-state scan kernels' item bodies (fast_core.h) run on the host, same interface as the oracle."""

    def __init__(self, program_json, max_keys=256, max_batch=1 << 16, max_matches=1 << 18):
        self.h = fast_lib().fh_create(program_json.encode(), max_keys, max_batch, max_matches)
        if not self.h:
            raise ValueError("fh_create failed (not a 2-state every/within shape?)")
        self.S = fast_lib().fh_num_states(self.h)

    def push(self, ts, key, stream, cols, nulls):
        ts = np.ascontiguousarray(ts, np.int64)
        key = np.ascontiguousarray(key, np.int32)
        stream = np.ascontiguousarray(stream, np.int32)
        cols = [np.ascontiguousarray(c) for c in cols]
        nul = [None if m is None else np.ascontiguousarray(m, np.uint8) for m in nulls]
        colp = (ctypes.c_void_p * max(1, len(cols)))(*[c.ctypes.data for c in cols])
        nulp = (ctypes.c_void_p * max(1, len(nul)))(*[None if m is None else m.ctypes.data for m in nul])
        err = fast_lib().fh_push(self.h, len(ts), _p(ts), _p(key), _p(stream), ctypes.cast(colp, ctypes.c_void_p),
                                 ctypes.cast(nulp, ctypes.c_void_p))
        if err:
            raise RuntimeError(f"scan-kernel error {err}")

    def fetch(self):
        L = fast_lib()
        m = L.fh_num_matches(self.h)
        r = L.fh_num_refs(self.h)
        out = {"key": np.zeros(m, np.int32), "ts": np.zeros(m, np.int64), "type": np.zeros(m, np.int8),
               "pos": np.zeros(m, np.int64), "slot_len": np.zeros((m, self.S), np.int32),
               "refs": np.zeros(max(r, 1), np.int64)}
        L.fh_fetch(self.h, _p(out["key"]), _p(out["ts"]), _p(out["type"]), _p(out["pos"]), _p(out["slot_len"]),
                   _p(out["refs"]))
        out["refs"] = out["refs"][:r]
        return out

    def __del__(self):
        try:
            fast_lib().fh_destroy(self.h)
        except Exception:
            pass
