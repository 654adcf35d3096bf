"""GPU diagnostic: the spill test's AGG stream through the FULL layout against the oracle, per push."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from diff_util import compare, per_key  # noqa: E402
from oracle.oracle import OracleEngine  # noqa: E402
from test_spill import _app, _cq, _falling_stream  # noqa: E402
from siddhi_amd.native import HipEngine  # noqa: E402

cq = _cq(_app())
ts, key, v = _falling_stream(400, 40_000, 4, hot=(5,), fall=6000)
st = np.zeros(len(ts), np.int32)
ora = OracleEngine(cq.program_json(), 0)
eng = HipEngine(cq.program_json(), 0, max_keys=400, max_batch=1 << 14, max_matches=1 << 18, force_general=3)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 9_973
for lo in range(0, len(ts), B):
    hi = min(len(ts), lo + B)
    for e in (ora, eng):
        e.push(ts[lo:hi], key[lo:hi], st[lo:hi], [v[lo:hi]], [None])
    a, b = per_key(ora.fetch()), per_key(eng.fetch())
    msg = compare(a, b)
    print(f"push [{lo},{hi}) oracle {sum(len(x) for x in a.values())} device {sum(len(x) for x in b.values())}"
          f" lean={eng.stat('lean_pushes')} fb={eng.stat('lean_fallbacks')} spill={eng.stat('spill_reruns')}"
          f" spilled={eng.stat('spilled_owners')} : {msg}", flush=True)
    if msg:
        k = int(msg.split()[1]) if msg.startswith("key") else None
        if k is not None:
            sa, sb = set(a.get(k, [])), set(b.get(k, []))
            print("  only oracle:", sorted(sa - sb)[:5], " only device:", sorted(sb - sa)[:5])
            idx = np.nonzero(key[:hi] == k)[0]
            print("  key events (idx, ts, v) last 12:", [(int(i), int(ts[i]), float(v[i])) for i in idx[-12:]])
            from siddhi_amd.native import LAYOUT_FULL  # noqa: F401
            print("  owner of key", k, "=", (k * 2654435769 % (1 << 32)) >> (32 - 9))
