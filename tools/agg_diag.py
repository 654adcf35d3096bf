"""GPU diagnostic: per-key match counts of the AGG layout against the PAIRS layout on the spill test's
stream, with k_sw_lean on and off (SHP_NO_LEAN), and with the spill path avoided (fewer open)."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

if len(sys.argv) < 2:
    for fall in ("6000", "300"):
        for nolean in ("0", "1"):
            env = dict(os.environ)
            if nolean == "1":
                env["SHP_NO_LEAN"] = "1"
            subprocess.check_call([sys.executable, __file__, fall, nolean], env=env)
    sys.exit(0)

from test_spill import _app, _cq, _falling_stream  # noqa: E402
from siddhi_amd.native import HipEngine, LAYOUT_AGG, LAYOUT_PAIRS32  # noqa: E402

fall = int(sys.argv[1])
cq = _cq(_app(select="e1.k as k, avg(e2.v) as a"))
ts, key, v = _falling_stream(400, 40_000, 4, hot=(5,), fall=fall)
st = np.zeros(len(ts), np.int32)
out = {}
for name, lay in (("agg", LAYOUT_AGG), ("pairs", LAYOUT_PAIRS32)):
    e = HipEngine(cq.program_json(), 0, max_keys=400, max_batch=1 << 14, max_matches=1 << 18, force_general=3,
                  match_layout=lay)
    cnt = np.zeros(400, np.int64)
    for lo in range(0, len(ts), 9_973):
        hi = min(len(ts), lo + 9_973)
        e.push(ts[lo:hi], key[lo:hi], st[lo:hi], [v[lo:hi]], [None])
        got = e.fetch()
        np.add.at(cnt, got["key"].astype(np.int64), 1)
    out[name] = (cnt, e.stat("lean_pushes"), e.stat("lean_fallbacks"), e.stat("spill_reruns"))
a, p = out["agg"], out["pairs"]
bad = np.nonzero(a[0] != p[0])[0]
print(f"fall={fall} nolean={sys.argv[2]} agg stats={a[1:]} pairs stats={p[1:]} total agg={a[0].sum()} pairs={p[0].sum()}"
      f" bad keys={bad[:10].tolist()} agg={a[0][bad[:10]].tolist()} pairs={p[0][bad[:10]].tolist()}", flush=True)
