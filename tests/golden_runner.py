"""Replays a transcribed reference known-answer test (tests/golden/*.json).

Each fixture holds the reference test's SiddhiQL app, its ordered sends (with the
timestamps the reference would have stamped), its ``Thread.sleep`` / wait helpers
as clock advances, and the rows/count it asserted.  ``run_fixture`` drives the
host-side runtime mirror with any engine (the HIP engine, or the oracle in tests)
and returns (ok, message, rows).
"""
from __future__ import annotations

import glob
import json
import os

import numpy as np

from siddhi_amd.runtime import SiddhiManager

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_fixtures(pattern="*.json"):
    out = []
    for path in sorted(glob.glob(os.path.join(GOLDEN, pattern))):
        d = json.load(open(path))
        out.extend(d["fixtures"])
    return out


def jval(v):
    if v is None or isinstance(v, bool):
        return v
    (k, x), = v.items()
    if k == "s":
        return x
    if k == "f":
        return float(np.float32(x))
    if k == "d":
        return float(x)
    return int(x)


def _eq(a, b):
    if isinstance(a, list) or isinstance(b, list):
        return isinstance(a, list) and isinstance(b, list) and len(a) == len(b) and all(
            _eq(x, y) for x, y in zip(a, b))
    if a is None or b is None:
        return a is None and b is None
    if isinstance(a, (int, float)) and isinstance(b, (int, float)) and not isinstance(a, bool):
        return float(a) == float(b) or (float(np.float32(a)) == float(np.float32(b)))
    return a == b


def rows_equal(r1, r2):
    return len(r1) == len(r2) and all(_eq(a, b) for a, b in zip(r1, r2))


def run_fixture(fx, engine_factory, native_lowering=False):
    mgr = SiddhiManager(engine_factory)
    rt = mgr.createSiddhiAppRuntime(fx["app"], start_clock=fx["start_clock"], batch_size=1,
                                    native_lowering=native_lowering)
    rows = []
    cb = fx["callback"]["name"]
    rt.addCallback(cb, lambda ts, ins, rem: rows.extend(list(e.data) for e in (ins or [])))
    rt.start()
    handlers = {}
    now = fx["start_clock"]
    for op in fx["ops"]:
        if "send" in op:
            h = handlers.setdefault(op["send"], rt.getInputHandler(op["send"]))
            h.send(op["ts"], [jval(v) for v in op["data"]])
            rt.flush()
            now = max(now, op["ts"])
        elif "advance" in op:
            now = op["advance"]
            rt.advance_time(now)
        elif "expect_count" in op:  # an intermediate count assert of the reference test
            rt.flush()
            if len(rows) != op["expect_count"]:
                return False, f"count {len(rows)} != expected {op['expect_count']} at op {fx['ops'].index(op)}", rows
        elif "wait_in_events" in op:
            w = op["wait_in_events"]
            for i in range(w["retry"]):
                now += w["sleep"]
                rt.advance_time(now)
                if len(rows) == 1:
                    break
        elif "wait_events" in op:
            w = op["wait_events"]
            waited = 0
            while len(rows) < w["expected"] and waited < w["timeout"]:
                now += w["sleep"]
                waited += w["sleep"]
                rt.advance_time(now)
    rt.shutdown()
    exp = fx["expected"]
    erows = [[jval(v) for v in r] for r in exp["rows"]]
    if len(rows) != exp["count"]:
        return False, f"count {len(rows)} != expected {exp['count']}; rows={rows[:6]}", rows
    mode = exp["mode"]
    if mode == "ordered" and not all(rows_equal(a, b) for a, b in zip(rows, erows)):
        return False, f"rows {rows} != expected {erows}", rows
    if mode == "each" and not all(rows_equal(r, erows[0]) for r in rows):
        return False, f"rows {rows} != expected each {erows[0]}", rows
    if mode == "prefix" and not all(rows_equal(a, b) for a, b in zip(rows, erows)):
        return False, f"rows {rows} != expected prefix {erows}", rows
    if mode == "contains":
        for e in erows:
            if not any(rows_equal(r, e) for r in rows):
                return False, f"expected row {e} not in {rows}", rows
    return True, "ok", rows
