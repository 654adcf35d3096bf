"""Per-key capacity growth on the general lanes (GPU).

The reference keeps pending / new-and-every lists as unbounded LinkedLists
(StreamPreStateProcessor.java:437-438) and its timer queue unbounded (Scheduler.java).  The lanes
keep fixed per-key pools in capacity tiers (nfa_lane.h LaneCaps: x1, x4, x16); a push that
overflows a tier is re-run from the committed state at the next tier, with the arena migrated
(engine.hip set_tier / k_lane_migrate).  These tests drive keys far past tier 0 (32 list entries,
64 StateEvents, 64 queued timers per key) and compare with the oracle, bit-exact per key.
"""
import json

import numpy as np
import pytest

from diff_util import compare, per_key
from oracle.oracle import OracleEngine

pytestmark = pytest.mark.gpu

NEVER_CLOSES = ("define stream S (k string, v float); partition with (k of S) begin @info(name='q') "
                "from every e1=S[v > 0] -> e2=S[v > 1000] select e1.v as a, e2.v as b insert into Out; end;")

ABSENT = ("@app:playback define stream S1 (k string, v float); define stream S2 (k string, v float); "
          "partition with (k of S1, k of S2) begin @info(name='q') "
          "from every e1=S1[v > 0] -> not S2[v > e1.v] for 10 sec "
          "select e1.v as a insert into Out; end;")


def _cq(app):
    from siddhi_amd.query.compiler import compile_app
    return compile_app(app)[1][0]


def _lanes(cq, keys, max_batch=1 << 14):
    from siddhi_amd.native import HipEngine
    return HipEngine(cq.program_json(), 0, max_keys=keys, max_batch=max_batch, max_matches=1 << 18,
                     force_general=1)


def _tier(eng):
    return eng.describe(eng.snapshot())["engine"]["tier"]


def _pending_stream(keys, opens, seed):
    """`opens` events per key with 0 < v <= 100 (each opens a partial that stays pending), then
    one v > 1000 per key, which closes every one of them."""
    rng = np.random.default_rng(seed)
    key = np.concatenate([rng.permutation(np.repeat(np.arange(keys), opens)), rng.permutation(keys)]).astype(np.int32)
    v = np.concatenate([rng.integers(1, 101, keys * opens), np.full(keys, 5000)]).astype(np.float32)
    ts = (1_000 + np.arange(len(key))).astype(np.int64)
    return ts, key, v


def _push_all(e, ts, key, v, step, streams=None, ncol=1):
    """v feeds every program column (one float attribute per stream here)."""
    st = np.zeros(len(ts), np.int32) if streams is None else streams
    for lo in range(0, len(ts), step):
        hi = min(len(ts), lo + step)
        e.push(ts[lo:hi], key[lo:hi], st[lo:hi], [v[lo:hi]] * ncol, [None] * ncol)


@pytest.mark.parametrize("step", [100_000, 97], ids=["whole", "split"])
def test_pending_lists_grow_past_tier0(step):
    """300 open partials per key: past tier 0 (32) and tier 1 (128), held at tier 2 (512).  Split
    pushes grow mid-stream, so the committed arena is migrated twice."""
    cq = _cq(NEVER_CLOSES)
    keys, opens = 6, 300
    ts, key, v = _pending_stream(keys, opens, 3)
    eng = _lanes(cq, keys)
    assert eng.path == 0
    ora = OracleEngine(cq.program_json(), 0)
    for e in (ora, eng):
        _push_all(e, ts, key, v, step)
    a, b = per_key(ora.fetch()), per_key(eng.fetch())
    assert compare(a, b) is None, compare(a, b)
    assert sum(len(x) for x in a.values()) == keys * opens
    assert _tier(eng) == 2


def test_tier_survives_snapshot_restore():
    """A snapshot taken at tier 1 restores into a fresh engine (tier 0, grown to the snapshot's
    tier) and continues exactly as the oracle does."""
    cq = _cq(NEVER_CLOSES)
    keys, opens = 4, 100
    ts, key, v = _pending_stream(keys, opens, 8)
    cut = keys * opens  # every partial open, none closed yet
    eng = _lanes(cq, keys)
    _push_all(eng, ts[:cut], key[:cut], v[:cut], 1 << 14)
    assert _tier(eng) == 1
    blob = eng.snapshot()
    d = eng.describe(blob)
    assert d["engine"]["tier"] == 1
    fresh = _lanes(cq, keys)
    assert _tier(fresh) == 0
    fresh.restore(blob)
    assert _tier(fresh) == 1
    ora = OracleEngine(cq.program_json(), 0)
    _push_all(ora, ts, key, v, 1 << 14)
    _push_all(fresh, ts[cut:], key[cut:], v[cut:], 1 << 14)
    a, b = per_key(ora.fetch()), per_key(fresh.fetch())
    assert compare(a, b) is None, compare(a, b)
    assert sum(len(x) for x in b.values()) == keys * opens


def test_timer_queue_grows_past_tier0():
    """An absent state queues one timer per open partial (Scheduler.notifyAt): 150 partials of
    one key within the 10 s wait overflow the tier-0 queue (64) and the lists (32)."""
    cq = _cq(ABSENT)
    keys, per = 3, 150
    rng = np.random.default_rng(11)
    n1 = keys * per
    key = rng.permutation(np.repeat(np.arange(keys), per)).astype(np.int32)
    v = rng.integers(1, 100, n1).astype(np.float32)
    ts = (10_000 + 5 * np.arange(n1)).astype(np.int64)  # all within 2.25 s
    # later events far apart on S1 fire the timers; no S2 events at all
    tail_key = np.arange(keys).astype(np.int32)
    key = np.concatenate([key, tail_key])
    v = np.concatenate([v, np.full(keys, 50)]).astype(np.float32)
    ts = np.concatenate([ts, 40_000 + np.arange(keys) * 1000]).astype(np.int64)
    streams = np.zeros(len(ts), np.int32)
    eng = _lanes(cq, keys)
    ora = OracleEngine(cq.program_json(), 0)
    for e in (ora, eng):
        _push_all(e, ts, key, v, 1 << 14, streams, ncol=2)
    a, b = per_key(ora.fetch()), per_key(eng.fetch())
    assert compare(a, b) is None, compare(a, b)
    assert sum(len(x) for x in a.values()) >= n1
    assert _tier(eng) >= 1


def test_tier0_workload_stays_at_tier0():
    """A workload within tier 0 never grows (the grown tiers only cost when needed)."""
    cq = _cq(NEVER_CLOSES)
    ts, key, v = _pending_stream(8, 20, 4)
    eng = _lanes(cq, 8)
    ora = OracleEngine(cq.program_json(), 0)
    for e in (ora, eng):
        _push_all(e, ts, key, v, 1 << 14)
    assert compare(per_key(ora.fetch()), per_key(eng.fetch())) is None
    assert _tier(eng) == 0


def test_pending_lists_grow_past_x16():
    """2500 open partials on each of 3 keys: past tier 2 (512 per list) and tier 3 (2048), held at
    tier 4 (x128: 4096 per list); the reference's lists are unbounded LinkedLists."""
    cq = _cq(NEVER_CLOSES)
    keys, opens = 3, 2500
    ts, key, v = _pending_stream(keys, opens, 12)
    eng = _lanes(cq, keys, max_batch=1 << 14)
    ora = OracleEngine(cq.program_json(), 0)
    for e in (ora, eng):
        _push_all(e, ts, key, v, 4_001)
    a, b = per_key(ora.fetch()), per_key(eng.fetch())
    assert compare(a, b) is None, compare(a, b)
    assert sum(len(x) for x in a.values()) == keys * opens
    assert _tier(eng) == 4
