"""Unbounded partial lists on the sweep path (GPU): spilled owners against the oracle.

The reference keeps each state's pending partials in an unbounded LinkedList
(StreamPreStateProcessor.java:437-438).  The sweep's LDS solves carry at most SWS_CCAP = 512 open
candidates per owner; an owner whose carry would outgrow that is re-run on k_sw_spill
(siddhi_amd/csrc/sweep_spill.h) with its open candidates in an HBM pool, and returns to the LDS
solves once its carry is back under SWS_CCAP / 2.  These streams hold thousands of open candidates
on one key -- a price that falls for a whole `within` window -- next to ordinary keys, and compare
every record with the oracle, bit-exact per key.
"""
import numpy as np
import pytest

from diff_util import compare, per_key
from oracle.oracle import OracleEngine

pytestmark = pytest.mark.gpu


def _app(within="5 sec", select="e1.v as a, e2.v as b"):
    return ("define stream S (k string, v float); partition with (k of S) begin @info(name='q') "
            f"from every e1=S[v > 20] -> e2=S[v > e1.v] within {within} select {select} "
            "insert into Out; end;")


def _cq(app):
    from siddhi_amd.query.compiler import compile_app
    return compile_app(app)[1][0]


def _eng(cq, keys, batch, **kw):
    from siddhi_amd.native import HipEngine
    e = HipEngine(cq.program_json(), 0, max_keys=keys, max_batch=batch, force_general=3, **kw)
    assert e.path == 2
    return e


def _falling_stream(keys, n, seed, hot=(0,), fall=6000, rise_at=None):
    """n events 1 ms apart over `keys` keys (random values); the `hot` keys get a run of `fall`
    strictly falling prices (every one opens a candidate, none closes: the open list grows to the
    whole window), then a high price that closes every open one at `rise_at`."""
    rng = np.random.default_rng(seed)
    key = rng.integers(0, keys, n).astype(np.int32)
    v = (rng.integers(0, 10000, n) / 100.0).astype(np.float32)
    ts = (1_000_000 + np.arange(n)).astype(np.int64)
    nh = len(hot)
    start = n // 10
    pos = np.arange(start, start + fall * nh)
    key[pos] = np.tile(np.asarray(hot, np.int32), fall)
    v[pos] = np.repeat(np.linspace(99.0, 21.0, fall).astype(np.float32), nh)
    r = start + fall * nh if rise_at is None else rise_at
    for j, h in enumerate(hot):
        key[r + j] = h
        v[r + j] = np.float32(99.5)
    return ts, key, v


def _push_all(eng, ts, key, v, batch):
    st = np.zeros(len(ts), np.int32)
    for lo in range(0, len(ts), batch):
        hi = min(len(ts), lo + batch)
        eng.push(ts[lo:hi], key[lo:hi], st[lo:hi], [v[lo:hi]], [None])
    return per_key(eng.fetch())


@pytest.mark.parametrize("batch", [40_000, 1_999], ids=["whole", "split"])
def test_one_key_with_thousands_of_open_candidates(batch):
    """One key holds ~5000 open candidates (falling for the whole 5 s window at 1 event/ms), then
    a rise closes all of them at once; 300 ordinary keys around it."""
    cq = _cq(_app())
    ts, key, v = _falling_stream(300, 40_000, 1, hot=(7,), fall=6000)
    want = _push_all(OracleEngine(cq.program_json(), 0), ts, key, v, batch)
    eng = _eng(cq, 300, 1 << 16, max_matches=1 << 18)
    got = _push_all(eng, ts, key, v, batch)
    assert compare(want, got) is None, compare(want, got)
    assert len(want[7]) > 4000  # the rise closed the window's candidates
    assert eng.stat("spill_reruns") >= 1
    assert eng.stat("spilled_owners") == 0  # back on the LDS solves after the stretch


def test_several_hot_keys_and_pairs32():
    """Three keys of different owners spill at once; the PAIRS32 layout (the bench's)."""
    from siddhi_amd.native import LAYOUT_PAIRS32
    cq = _cq(_app(within="3 sec"))
    ts, key, v = _falling_stream(1000, 60_000, 2, hot=(3, 500, 999), fall=3500)
    want = _push_all(OracleEngine(cq.program_json(), 0), ts, key, v, 7_919)
    eng = _eng(cq, 1000, 1 << 14, max_matches=1 << 18, match_layout=LAYOUT_PAIRS32)
    got = _push_all(eng, ts, key, v, 7_919)
    assert compare(want, got) is None, compare(want, got)
    assert eng.stat("spill_reruns") >= 1


def test_spilled_owner_snapshot_restore():
    """A snapshot taken while an owner is spilled (its carry in the HBM pool) restores into a
    fresh engine that continues exactly as the oracle."""
    cq = _cq(_app())
    ts, key, v = _falling_stream(200, 30_000, 3, hot=(11,), fall=5000)
    cut = 3000 + 4000  # inside the falling run: the open list is in the pool
    eng = _eng(cq, 200, 1 << 15, max_matches=1 << 18)
    first = _push_all(eng, ts[:cut], key[:cut], v[:cut], 2_500)
    assert eng.stat("spilled_owners") >= 1
    blob = eng.snapshot()
    d = eng.describe(blob)
    e2 = d["keys"]["11"]["e2"]  # e1-filled partials wait at e2's pre-processor
    opens = len(e2["PendingStateEventList"]) + len(e2["NewAndEveryStateEventList"])
    fresh = _eng(cq, 200, 1 << 15, max_matches=1 << 18)
    fresh.restore(blob)
    want = _push_all(OracleEngine(cq.program_json(), 0), ts, key, v, 2_500)
    rest = _push_all(fresh, ts[cut:], key[cut:], v[cut:], 2_500)
    got = {}
    for part in (first, rest):
        for k, recs in part.items():
            got.setdefault(k, []).extend(recs)
    assert compare(want, got) is None, compare(want, got)
    assert opens > 3000


def test_rejected_restore_leaves_spilled_state():
    """A truncated blob, and one whose pool sections disagree with each other, are rejected before
    anything changes: the engine holding a spilled owner (its carry in the HBM pool) then goes on
    exactly as the oracle (restore used to resize the pool before validating)."""
    from siddhi_amd.native import ShpError
    cq = _cq(_app())
    ts, key, v = _falling_stream(200, 30_000, 3, hot=(11,), fall=5000)
    cut = 3000 + 4000
    eng = _eng(cq, 200, 1 << 15, max_matches=1 << 18)
    first = _push_all(eng, ts[:cut], key[:cut], v[:cut], 2_500)
    assert eng.stat("spilled_owners") >= 1
    blob = eng.snapshot()
    for bad in (blob[:-1], blob[:-9] + blob[-8:], blob + b"\0"):
        with pytest.raises(ShpError):
            eng.restore(bad)
    assert eng.stat("spilled_owners") >= 1
    want = _push_all(OracleEngine(cq.program_json(), 0), ts, key, v, 2_500)
    rest = _push_all(eng, ts[cut:], key[cut:], v[cut:], 2_500)
    got = {}
    for part in (first, rest):
        for k, recs in part.items():
            got.setdefault(k, []).extend(recs)
    assert compare(want, got) is None, compare(want, got)


def test_spill_with_device_average():
    """C5's selector (avg over e2's value) folded on a spilled owner in emission order."""
    from siddhi_amd.native import LAYOUT_AGG
    cq = _cq(_app(select="e1.k as k, avg(e2.v) as a"))
    ts, key, v = _falling_stream(400, 40_000, 4, hot=(5,), fall=6000)
    ora = OracleEngine(cq.program_json(), 0)
    want = _push_all(ora, ts, key, v, 9_973)
    eng = _eng(cq, 400, 1 << 14, max_matches=1 << 18, match_layout=LAYOUT_AGG)
    st = np.zeros(len(ts), np.int32)
    rows = {}
    for lo in range(0, len(ts), 9_973):
        hi = min(len(ts), lo + 9_973)
        eng.push(ts[lo:hi], key[lo:hi], st[lo:hi], [v[lo:hi]], [None])
        got = eng.fetch()
        for k, a in zip(got["key"], got["agg"]):
            rows.setdefault(int(k), []).append(float(a))
    assert eng.stat("spill_reruns") >= 1
    # expected running average per key over e2's values in emission order (the oracle's records)
    for k, recs in want.items():
        vals = [float(v[r[3][1][0] - 0]) for r in recs]  # e2's batch-global seq = stream index
        acc, exp = 0.0, []
        for i, x in enumerate(vals):
            acc += x
            exp.append(acc / (i + 1))
        np.testing.assert_allclose(rows.get(k, []), exp, rtol=1e-9, atol=0)
