"""k_sw_lean, the sweep solve for the headline 2-state shape, against the oracle (GPU).

k_sw_lean (siddhi_amd/csrc/sweep_lean.h) covers `every e1=S[f1] -> e2=S[e2.v OP x] within W`
with one typed compare and no nulls; anything else it meets in a push (a ts decrease within a
key, a push spanning more than 2^30 ms, more than 384 open candidates on an owner, more than 255
far candidates closed by one event) hands the push back to the exact k_sw_solve.  These tests
check both kernels against the oracle (StreamPreStateProcessor.processAndReturn / expireEvents
:326-403 restated in oracle/oracle.cpp), that the headline stream never falls back, that the
fallbacks do happen where they should, and that state handed between the two kernels across
pushes continues exactly.
"""
import numpy as np
import pytest

from diff_util import compare, per_key, program_for, run, small_stream
from oracle.oracle import OracleEngine

pytestmark = pytest.mark.gpu


def _eng(cq, keys, batch, **kw):
    from siddhi_amd.native import HipEngine
    e = HipEngine(cq.program_json(), 0, max_keys=keys, max_batch=batch, force_general=3, **kw)
    assert e.path == 2
    return e


def _push_all(eng, ts, key, v, batch, nul=None):
    st = np.zeros(len(ts), np.int32)
    for lo in range(0, len(ts), batch):
        hi = min(len(ts), lo + batch)
        eng.push(ts[lo:hi], key[lo:hi], st[lo:hi], [v[lo:hi]], [None if nul is None else nul[lo:hi]])
    return per_key(eng.fetch())


def _app(op="> e1.v", typ="float", f1="v > 20", within="1 sec"):
    return (f"define stream S (k string, v {typ}); partition with (k of S) begin @info(name='q') "
            f"from every e1=S[{f1}] -> e2=S[v {op}] within {within} select e1.v as a, e2.v as b "
            f"insert into Out; end;")


def _cq(app):
    from siddhi_amd.query.compiler import compile_app
    return compile_app(app)[1][0]


def test_c2_10k_keys_runs_lean_without_fallback():
    """The headline stream (10k keys) through k_sw_lean: bit-exact per key, no push handed back."""
    cq = program_for(2)
    g = small_stream(2, 3_000_000, 10_000)
    want = per_key(run(OracleEngine(cq.program_json(), 0), cq, g))
    eng = _eng(cq, 10_000, 1 << 21)
    got = per_key(run(eng, cq, g, 1_000_003))
    assert compare(want, got) is None, compare(want, got)
    assert eng.stat("pushes") == 3 and eng.stat("lean_pushes") == 3 and eng.stat("lean_fallbacks") == 0
    assert sum(len(v) for v in want.values()) > 1_000_000


@pytest.mark.parametrize("typ", ["float", "int"])
@pytest.mark.parametrize("op", ["<", "<=", ">", ">=", "==", "!="])
@pytest.mark.parametrize("rhs", ["e1", "const"])
def test_lean_comparisons_vs_oracle(op, typ, rhs):
    """Every comparison class of k_sw_lean (float and int compares), e1.v or a constant on the
    right, ties and -0.0, split batches; the lean kernel takes every push."""
    rng = np.random.default_rng(len(op) * 13 + (typ == "int") * 5 + (rhs == "e1"))
    n, keys = 80_000, 700
    ts = np.cumsum(rng.integers(0, 3, n)).astype(np.int64) + 5_000
    key = rng.integers(0, keys, n).astype(np.int32)
    small = rng.integers(0, 10, n)
    if typ == "float":
        v = small.astype(np.float32) + np.where(rng.random(n) < 0.3, np.float32(0.5), np.float32(0))
        v[rng.random(n) < 0.02] = -0.0
    else:
        v = (small - 2).astype(np.int32)
    cq = _cq(_app(op=f"{op} {'e1.v' if rhs == 'e1' else '4'}", typ=typ, f1="v > 3", within="300 milliseconds"))
    want = _push_all(OracleEngine(cq.program_json(), 0), ts, key, v, 19_997)
    eng = _eng(cq, keys, 1 << 15)
    got = _push_all(eng, ts, key, v, 19_997)
    assert compare(want, got) is None, compare(want, got)
    assert eng.stat("lean_pushes") == eng.stat("pushes") and eng.stat("lean_fallbacks") == 0
    assert sum(len(x) for x in want.values()) > 500


def test_lean_matches_exact_kernel_with_env_off(monkeypatch):
    """The same pushes with k_sw_lean disabled (SHP_NO_LEAN): identical per-key records."""
    cq = program_for(2)
    g = small_stream(2, 400_000, 3_000)
    a = per_key(run(_eng(cq, 3_000, 1 << 18), cq, g, 123_457))
    monkeypatch.setenv("SHP_NO_LEAN", "1")
    b = per_key(run(_eng(cq, 3_000, 1 << 18), cq, g, 123_457))
    assert compare(a, b) is None, compare(a, b)


def test_fallback_and_back_keeps_state_exact():
    """Pushes alternate between ordered input (k_sw_lean) and input whose ts decrease within a
    key (handed back to k_sw_solve): the carry each kernel writes is read by the other."""
    rng = np.random.default_rng(21)
    n, keys, batch = 120_000, 16, 10_000
    ts = 1_000_000 + np.arange(n, dtype=np.int64) * 3
    bad = np.zeros(n, bool)
    for b0 in range(0, n, 2 * batch):  # every other push has out-of-order events
        bad[b0:b0 + batch] = rng.random(min(batch, n - b0)) < 0.05
    ts[bad] -= rng.integers(1, 800, bad.sum())
    key = rng.integers(0, keys, n).astype(np.int32)
    v = (rng.integers(0, 10000, n) / 100.0).astype(np.float32)
    cq = program_for(2)
    want = _push_all(OracleEngine(cq.program_json(), 0), ts, key, v, batch)
    eng = _eng(cq, keys, 1 << 15)
    got = _push_all(eng, ts, key, v, batch)
    assert compare(want, got) is None, compare(want, got)
    fb = eng.stat("lean_fallbacks")
    assert 0 < fb < eng.stat("pushes"), (fb, eng.stat("pushes"))


def test_far_closers_and_many_open_candidates():
    """Keys whose candidates stay open over long runs: a falling price for hundreds of events,
    then one event that closes all of them (distances beyond the 24 near bits, more than 255
    far closers on one event, and carries beyond the lean kernel's 384 per owner)."""
    rng = np.random.default_rng(5)
    keys = 300
    parts_ts, parts_key, parts_v = [], [], []
    t = 10_000
    for rnd in range(6):
        run_len = [30, 120, 300, 500, 60, 260][rnd]
        hot = rng.choice(keys, 3, replace=False)
        for i in range(run_len):  # the hot keys fall, background keys are random
            for k in hot:
                parts_ts.append(t)
                parts_key.append(k)
                parts_v.append(90.0 - 60.0 * i / run_len)
            bg = rng.choice(np.setdiff1d(np.arange(keys), hot), 4)  # background keys never close a hot key's run
            for k in bg:
                parts_ts.append(t)
                parts_key.append(int(k))
                parts_v.append(float(rng.integers(0, 10000)) / 100.0)
            t += 1
        for k in hot:  # one high price closes every open candidate of the key
            parts_ts.append(t)
            parts_key.append(k)
            parts_v.append(99.5)
        t += 5
    ts = np.array(parts_ts, np.int64)
    key = np.array(parts_key, np.int32)
    v = np.array(parts_v, np.float32)
    cq = _cq(_app(within="1 hour"))
    want = _push_all(OracleEngine(cq.program_json(), 0), ts, key, v, 1_700)
    eng = _eng(cq, keys, 1 << 14)
    got = _push_all(eng, ts, key, v, 1_700)
    assert compare(want, got) is None, compare(want, got)
    assert max(len(x) for x in want.values()) > 300
    assert eng.stat("lean_fallbacks") > 0  # the 500-long run overflows the lean carry


def test_wide_push_falls_back_exactly():
    """One push whose timestamps span more than 2^30 ms (about 12 days): the exact kernel runs it,
    and the next (narrow) push continues in k_sw_lean from the state it left."""
    rng = np.random.default_rng(8)
    n, keys = 40_000, 500
    ts = 1_000_000 + np.arange(n, dtype=np.int64) * 5
    ts[n // 2:] += 1 << 31  # a jump of ~25 days in the middle of the first push
    key = rng.integers(0, keys, n).astype(np.int32)
    v = (rng.integers(0, 10000, n) / 100.0).astype(np.float32)
    cq = _cq(_app(within="5 days"))
    want = _push_all(OracleEngine(cq.program_json(), 0), ts, key, v, 30_000)
    eng = _eng(cq, keys, 1 << 15)
    got = _push_all(eng, ts, key, v, 30_000)
    assert compare(want, got) is None, compare(want, got)
    assert eng.stat("pushes") == 2 and eng.stat("lean_pushes") == 2 and eng.stat("lean_fallbacks") == 1


@pytest.mark.parametrize("agg", [False, True], ids=["pairs", "avg"])
def test_push_beyond_12_byte_records_rescatters(agg):
    """The scatter writes 12-byte records (ts in 23 bits around the push's first ts) for the lean
    solve; a push spanning more than 2^22 ms (a jump of ~2.3 h in its middle) overflows them and is
    scattered again in the 16-byte form, the lean solve re-running it (no exact-kernel fallback);
    the next, narrow push is back on the 12-byte records.  Output equal to the oracle's."""
    rng = np.random.default_rng(9)
    n, keys = 40_000, 500
    ts = 1_000_000 + np.arange(n, dtype=np.int64) * 5
    ts[n // 2:] += 1 << 23
    key = rng.integers(0, keys, n).astype(np.int32)
    v = (rng.integers(0, 10000, n) / 100.0).astype(np.float32)
    app = _app(within="1 sec")
    if agg:
        app = app.replace("select e1.v as a, e2.v as b", "select avg(e2.v) as a")
    cq = _cq(app)
    want = _push_all(OracleEngine(cq.program_json(), 0), ts, key, v, 30_000)
    eng = _eng(cq, keys, 1 << 15)
    got = _push_all(eng, ts, key, v, 30_000)
    if not agg:
        assert compare(want, got) is None, compare(want, got)
        assert sum(len(x) for x in want.values()) > 1000
    assert eng.stat("pushes") == 2 and eng.stat("lean_fallbacks") == 0
    assert eng.stat("sweep_r16_reruns") == 1


@pytest.mark.parametrize("fn", ["avg", "max"])
def test_lean_agg_closers_with_many_matches(fn):
    """SHP_LAYOUT_AGG through k_sw_lean where one event closes up to ~200 candidates of its key
    (falling prices, then one high price): the one-lane-per-match emission (sl_expand_block) takes
    a closing position's matches over several 64-match windows, with blocks of 64 positions holding
    far more than 64 matches.  Per key, the running aggregate equals the reference aggregator's fold
    over the oracle's matches (avg to 1e-9 relative, max exact)."""
    from siddhi_amd.native import LAYOUT_AGG, HipEngine
    from siddhi_amd.query.compiler import compile_app
    from test_gpu_parity import _agg_app, _expected_agg
    rng = np.random.default_rng(17)
    keys = 300
    ts_, key_, v_ = [], [], []
    t = 50_000
    for rnd, run_len in enumerate([30, 70, 130, 200, 90, 160]):
        hot = 3 * rnd + np.arange(3)  # consecutive ids: three different owners
        for i in range(run_len):
            for k in hot:
                ts_.append(t)
                key_.append(int(k))
                v_.append(90.0 - 60.0 * i / run_len)
            for k in rng.choice(np.arange(20, keys), 4):  # background keys
                ts_.append(t)
                key_.append(int(k))
                v_.append(float(rng.integers(2100, 10000)) / 100.0)
            t += 1
        for k in hot:
            ts_.append(t)
            key_.append(int(k))
            v_.append(99.5)
        t += 2_000  # past the window: the next round starts from empty keys
    n = len(ts_)
    g = {"ts": np.array(ts_, np.int64), "key": np.array(key_, np.int32), "stream": np.zeros(n, np.int32),
         "price": np.array(v_, np.float32), "volume": np.zeros(n, np.int64)}
    cq = compile_app(_agg_app(fn))[1][0]
    a = run(OracleEngine(cq.program_json(), 0), cq, g)
    want = _expected_agg(a, g["price"], fn)
    e2 = {}
    S = a["slot_len"].shape[1]
    off = 0
    for i in range(len(a["key"])):  # matches per closing event
        lens = [int(x) for x in a["slot_len"][i]]
        e2[int(a["refs"][off + lens[0]])] = e2.get(int(a["refs"][off + lens[0]]), 0) + 1
        off += sum(lens)
    assert max(e2.values()) >= 150
    eng = HipEngine(cq.program_json(), 0, max_keys=keys, max_batch=1 << 14, force_general=3,
                    match_layout=LAYOUT_AGG)
    assert eng.path == 2
    b = run(eng, cq, g, 1_700)
    assert eng.stat("lean_pushes") == eng.stat("pushes") and eng.stat("lean_fallbacks") == 0
    got = {}
    for k, x in zip(b["key"], b["agg"]):
        got.setdefault(int(k), []).append(float(x))
    assert set(got) == set(want)
    for k in want:
        assert len(got[k]) == len(want[k]), k
        if fn == "max":
            assert got[k] == want[k], k
        else:
            np.testing.assert_allclose(got[k], want[k], rtol=1e-9, atol=0)
