"""Differential helpers: run a synthetic stream through two engines and compare matches per key."""
import json

import numpy as np

from siddhi_amd import synth
from siddhi_amd.query.compiler import compile_app


def program_for(query_key):
    app, qs, _ = compile_app(synth.QUERIES[query_key])
    return qs[0]


def columns_for(cq, g):
    cols = []
    for (s, a, t) in cq.columns:
        name = list(cq.program["streams"][s]["attrs"])[a][0]
        name = {"v": "price"}.get(name, name)
        arr = g[name]
        cols.append(np.ascontiguousarray(arr.astype({"float": np.float32, "double": np.float64,
                                                     "int": np.int32, "long": np.int64}[t])))
    return cols


def run(engine, cq, g, batch=None):
    n = len(g["ts"])
    batch = batch or n
    cols = columns_for(cq, g)
    for lo in range(0, n, batch):
        hi = min(n, lo + batch)
        engine.push(g["ts"][lo:hi], g["key"][lo:hi], g["stream"][lo:hi], [c[lo:hi] for c in cols],
                    [None] * len(cols))
    return engine.fetch()


def per_key(mb):
    """{key: [(ts, type, pos, slots...)]} preserving per-key order."""
    out = {}
    S = mb["slot_len"].shape[1] if len(mb["key"]) else 0
    off = 0
    for i in range(len(mb["key"])):
        slots = []
        for s in range(S):
            ln = int(mb["slot_len"][i, s])
            slots.append(tuple(int(x) for x in mb["refs"][off:off + ln]))
            off += ln
        out.setdefault(int(mb["key"][i]), []).append(
            (int(mb["ts"][i]), int(mb["type"][i]), int(mb["pos"][i]), tuple(slots)))
    return out


def compare(a, b):
    ka, kb = set(a), set(b)
    if ka != kb:
        return f"key sets differ: only-a {sorted(ka - kb)[:5]} only-b {sorted(kb - ka)[:5]}"
    for k in sorted(ka):
        if a[k] != b[k]:
            la, lb = a[k], b[k]
            for i, (x, y) in enumerate(zip(la, lb)):
                if x != y:
                    return f"key {k} idx {i}: {x} != {y} (len {len(la)} vs {len(lb)})"
            return f"key {k}: lengths {len(la)} vs {len(lb)}"
    return None


def small_stream(config, n, keys=None, dense=None):
    spec = synth.CONFIGS[config if isinstance(config, int) else 3]
    spec = synth.StreamSpec(spec.config, n, keys or spec.keys, spec.n_streams,
                            spec.dense if dense is None else dense)
    return synth.generate(spec)
