"""k_sw_win, the unit-parallel sweep solve (round 4), against the oracle and against k_sw_lean (GPU).

k_sw_win (siddhi_amd/csrc/sweep_win.h) cuts the owner-major record array into fixed units, one
wave each; a unit rebuilds the open candidates at its start by replaying a halo of the owner's
earlier records (exact once each key's events in it span more than `within`, or from the owner's
start), and finds its output offset by a decoupled look-back over the earlier units.  The per-owner
state after a push comes from a tail replay per owner.  These tests pin each of those pieces
against the oracle (StreamPreStateProcessor.processAndReturn / expireEvents :326-403 restated in
oracle/oracle.cpp): halos too short for the keys (forced with SHP_WIN_HALO), units that straddle
many short owner regions, keys idle in a push (their state passes through the tail), rare keys
whose halo reaches back to the owner's start, both pair layouts, and snapshots equal to the ones
k_sw_lean leaves.
"""
import numpy as np
import pytest

from diff_util import compare, per_key, program_for, run, small_stream
from oracle.oracle import OracleEngine

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _win_on(monkeypatch):
    """k_sw_win is opt-in (SHP_WIN=1): it is exact but slower than k_sw_lean on C2."""
    monkeypatch.setenv("SHP_WIN", "1")


def _eng(cq, keys, batch, **kw):
    from siddhi_amd.native import HipEngine
    e = HipEngine(cq.program_json(), 0, max_keys=keys, max_batch=batch, force_general=3, **kw)
    assert e.path == 2
    return e


def _push_all(eng, ts, key, v, batch):
    st = np.zeros(len(ts), np.int32)
    for lo in range(0, len(ts), batch):
        hi = min(len(ts), lo + batch)
        eng.push(ts[lo:hi], key[lo:hi], st[lo:hi], [v[lo:hi]], [None])
    return per_key(eng.fetch())


def _app(within="1 sec"):
    return ("define stream S (k string, v float); partition with (k of S) begin @info(name='q') "
            f"from every e1=S[v > 20] -> e2=S[v > e1.v] within {within} select e1.v as a, e2.v as b "
            "insert into Out; end;")


def _cq(app):
    from siddhi_amd.query.compiler import compile_app
    return compile_app(app)[1][0]


def test_win_c2_10k_keys_no_fallback():
    """The headline stream (10k keys, three pushes): every push on k_sw_win, bit-exact per key."""
    cq = program_for(2)
    g = small_stream(2, 3_000_000, 10_000)
    want = per_key(run(OracleEngine(cq.program_json(), 0), cq, g))
    eng = _eng(cq, 10_000, 1 << 21)
    got = per_key(run(eng, cq, g, 1_000_003))
    assert compare(want, got) is None, compare(want, got)
    assert eng.stat("win_pushes") == 3 and eng.stat("win_fallbacks") == 0
    assert sum(len(v) for v in want.values()) > 1_000_000


@pytest.mark.parametrize("halo", [8, 64, 1 << 20])
def test_win_halo_lengths(halo, monkeypatch):
    """Halos far too short for the keys (every unit widens its own, several times), the default,
    and one that always reaches the owner's start: the same records."""
    monkeypatch.setenv("SHP_WIN_HALO", str(halo))
    cq = program_for(2)
    g = small_stream(2, 600_000, 2_000)
    want = per_key(run(OracleEngine(cq.program_json(), 0), cq, g))
    eng = _eng(cq, 2_000, 1 << 18)
    got = per_key(run(eng, cq, g, 200_003))
    assert compare(want, got) is None, compare(want, got)
    assert eng.stat("win_pushes") == 3 and eng.stat("win_fallbacks") == 0


def test_win_units_straddle_short_owner_regions():
    """40k keys over 2048 owners and pushes of ~20k events: about ten records per owner, so one
    unit covers a hundred owners' segments, each with its own halo and presence mask."""
    rng = np.random.default_rng(3)
    n, keys = 120_000, 40_000
    ts = 2_000_000 + np.arange(n, dtype=np.int64) // 4
    key = rng.integers(0, keys, n).astype(np.int32)
    v = (rng.integers(0, 10000, n) / 100.0).astype(np.float32)
    cq = _cq(_app(within="30 sec"))
    want = _push_all(OracleEngine(cq.program_json(), 0), ts, key, v, 20_011)
    eng = _eng(cq, keys, 1 << 15)
    got = _push_all(eng, ts, key, v, 20_011)
    assert compare(want, got) is None, compare(want, got)
    assert eng.stat("win_fallbacks") == 0 and eng.stat("win_pushes") == eng.stat("pushes")


def test_win_idle_and_rare_keys_snapshot_like_lean(monkeypatch):
    """Keys silent for whole pushes (their carry and lastc pass through the tail), keys with one
    event per push (their halo reaches back to the owner's start), and the snapshot each push
    leaves: describe() equal to k_sw_lean's after every push."""
    rng = np.random.default_rng(11)
    keys, per = 3_000, 60_000
    parts = []
    t = 5_000_000
    for p in range(4):
        active = np.arange(keys) if p % 2 == 0 else np.arange(0, keys, 7)  # most keys idle in odd pushes
        k = rng.choice(active, per).astype(np.int32)
        k[:40] = np.arange(2_900, 2_940)  # rare keys: one event each, at the push's start
        k[40:] = np.where(k[40:] >= 2_900, k[40:] - 100, k[40:])
        ts = t + np.arange(per, dtype=np.int64) // 3
        t = int(ts[-1]) + 50
        v = (rng.integers(0, 10000, per) / 100.0).astype(np.float32)
        parts.append((ts, k, v))
    cq = _cq(_app(within="5 sec"))
    o = OracleEngine(cq.program_json(), 0)
    win = _eng(cq, keys, 1 << 17)
    monkeypatch.delenv("SHP_WIN")
    lean = _eng(cq, keys, 1 << 17)
    monkeypatch.setenv("SHP_WIN", "1")
    st = np.zeros(per, np.int32)
    for ts, k, v in parts:
        for e in (o, win, lean):
            e.push(ts, k, st, [v], [None])
        assert win.describe(win.snapshot()) == lean.describe(lean.snapshot())
    want, got = per_key(o.fetch()), per_key(win.fetch())
    assert compare(want, got) is None, compare(want, got)
    assert win.stat("win_pushes") == 4 and win.stat("win_fallbacks") == 0
    assert lean.stat("win_pushes") == 0


@pytest.mark.parametrize("layout", ["pairs", "pairs32"])
def test_win_pair_layouts(layout):
    """Both pair layouts from k_sw_win (the bench's PAIRS32 and the 16-byte PAIRS), expanded on
    fetch, against the oracle."""
    from siddhi_amd import native
    lay = native.LAYOUT_PAIRS if layout == "pairs" else native.LAYOUT_PAIRS32
    cq = program_for(2)
    g = small_stream(2, 500_000, 4_000)
    want = per_key(run(OracleEngine(cq.program_json(), 0), cq, g))
    eng = _eng(cq, 4_000, 1 << 18, match_layout=lay)
    got = per_key(run(eng, cq, g, 170_001))
    assert compare(want, got) is None, compare(want, got)
    assert eng.stat("win_pushes") == 3 and eng.stat("win_fallbacks") == 0


def test_win_hands_back_to_lean_then_exact():
    """A key with hundreds of open candidates (falling prices over one hour's window) overflows
    the wave's list: k_sw_win hands the push to k_sw_lean, which hands it on to the exact solve;
    later ordinary pushes return to k_sw_win from the state the exact solve left."""
    rng = np.random.default_rng(4)
    keys = 200
    n1 = 30_000
    ts = 1_000_000 + np.arange(3 * n1, dtype=np.int64)
    key = rng.integers(0, keys, 3 * n1).astype(np.int32)
    v = (rng.integers(0, 10000, 3 * n1) / 100.0).astype(np.float32)
    hot = key[:n1] == 7
    v[:n1][hot] = np.linspace(95.0, 21.0, hot.sum()).astype(np.float32)  # ~150 open candidates
    cq = _cq(_app(within="1 hour"))
    want = _push_all(OracleEngine(cq.program_json(), 0), ts, key, v, n1)
    eng = _eng(cq, keys, 1 << 16)
    got = _push_all(eng, ts, key, v, n1)
    assert compare(want, got) is None, compare(want, got)
    assert eng.stat("win_fallbacks") >= 1 and eng.stat("win_pushes") == 3
