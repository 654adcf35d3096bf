"""Device aggregates off the sweep: SHP_LAYOUT_AGG on the general NFA lanes.

The lanes fold the select's aggregate as each match is emitted (siddhi_amd/csrc/nfa_lane.h
aggregate(): QuerySelector.processInBatchNoGroupBy :271-313 with the Avg / Sum / Count / Min / Max
AttributeAggregatorExecutors), one running state per partition key, in emission order.  Every
query shape whose aggregate the sweep does not cover runs it there: count sequences (C3'), the
logical-absent playback pattern (C4, timer matches), aggregates over e1.  Expected values: the
oracle's matches folded by the reference aggregator arithmetic (per key, in emission order); the
first event of the aggregated state's chain (the selector's default index 0) is the argument.
"""
import numpy as np
import pytest

from diff_util import columns_for, run, small_stream
from oracle.oracle import OracleEngine

pytestmark = pytest.mark.gpu


def _cq(app):
    from siddhi_amd.query.compiler import compile_app
    return compile_app(app)[1][0]


def _fold(ora, cq, g, values_by_seq):
    """Per key: the running aggregate over the oracle's matches (reference arithmetic)."""
    agg = cq.program["aggregate"]
    fn, st = agg["fn"], agg.get("state")
    S = ora["slot_len"].shape[1]
    out, state = {}, {}
    off = 0
    for i in range(len(ora["key"])):
        k = int(ora["key"][i])
        lens = [int(x) for x in ora["slot_len"][i]]
        x = None
        if fn != "count":
            o = off + sum(lens[:st])
            if lens[st] > 0:
                x = values_by_seq(int(ora["refs"][o]))
        off += sum(lens)
        s, c = state.get(k, (None, 0))
        if fn == "count":
            c += 1
            val = float(c)
        else:
            if x is not None:
                if fn in ("avg", "sum"):
                    s = (s or 0.0) + x
                elif c == 0:
                    s = x
                elif not np.isnan(s) and not np.isnan(x):
                    s = x if (fn == "min" and s > x) or (fn == "max" and s < x) else s
                c += 1
            assert c > 0, "a null first value (the engine fails such a push)"
            val = s / c if fn == "avg" else s
        state[k] = (s, c)
        out.setdefault(k, []).append(val)
    return out


def _got(b):
    got = {}
    for k, v in zip(b["key"], b["agg"]):
        got.setdefault(int(k), []).append(float(v))
    return got


def _check(want, got, exact):
    assert set(got) == set(want)
    for k in want:
        w, h = np.array(want[k]), np.array(got[k])
        assert len(w) == len(h), k
        if exact:
            assert (np.isnan(w) == np.isnan(h)).all(), k
            ok = ~np.isnan(w)
            assert (w[ok].view(np.uint64) == h[ok].view(np.uint64)).all(), k
        else:
            np.testing.assert_allclose(h, w, rtol=1e-12, atol=0)


@pytest.mark.parametrize("fn", ["avg", "sum", "count", "min", "max"])
def test_lanes_aggregate_over_e1_of_the_two_state_pattern(fn):
    """avg/sum/count/min/max over e1's price (the sweep folds only e2's): on the general lanes,
    three pushes, 400 keys; sequential fold per key, so avg / sum match the reference's own
    association exactly."""
    from siddhi_amd.native import LAYOUT_AGG, HipEngine
    arg = "" if fn == "count" else "e1.price"
    cq = _cq("define stream StockStream (symbol string, price float, volume long); "
             "partition with (symbol of StockStream) begin @info(name='q') "
             "from every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] within 1 sec "
             f"select e1.symbol as symbol, {fn}({arg}) as a insert into Out; end;")
    g = small_stream(2, 120_000, 400)
    price = columns_for(cq, g)[0]
    ora = run(OracleEngine(cq.program_json(), 0), cq, g)
    want = _fold(ora, cq, g, lambda q: float(price[q]))
    eng = HipEngine(cq.program_json(), 0, max_keys=400, max_batch=1 << 16, match_layout=LAYOUT_AGG)
    # count() has no argument, so it does not name e1: the sweep folds it (k_sw_lean)
    assert eng.path == (2 if fn == "count" else 0)
    got = _got(run(eng, cq, g, 40_009))
    _check(want, got, exact=True)
    assert sum(len(v) for v in want.values()) > 10_000


def test_lanes_aggregate_count_sequence_c3b():
    """C3' (`every e1=S[v>20]<1:5>, e2=S[v<e1[last].v]`) with avg(e2.v): the count-sequence shape
    hands an aggregate to the lanes."""
    from siddhi_amd.native import LAYOUT_AGG, HipEngine
    cq = _cq("define stream S (k string, v float); partition with (k of S) begin @info(name='q') "
             "from every e1=S[v>20]<1:5>, e2=S[v<e1[last].v] select e1[0].v as a, avg(e2.v) as m "
             "insert into Out; end;")
    g = small_stream(3, 100_000, 1_000)
    v = columns_for(cq, g)[0]
    ora = run(OracleEngine(cq.program_json(), 0), cq, g)
    want = _fold(ora, cq, g, lambda q: float(v[q]))
    eng = HipEngine(cq.program_json(), 0, max_keys=1_000, max_batch=1 << 16, match_layout=LAYOUT_AGG)
    assert eng.path == 0
    got = _got(run(eng, cq, g, 33_331))
    _check(want, got, exact=True)
    assert sum(len(x) for x in want.values()) > 5_000


def test_lanes_aggregate_logical_absent_timer_matches_c4():
    """C4 (logical + absent, playback) with sum(e1.price): every match is a timer match whose
    e1 may come from an earlier push; the lane reads it from its own event nodes."""
    from siddhi_amd.native import LAYOUT_AGG, HipEngine
    cq = _cq("@app:playback define stream S1 (symbol string, price float, volume long); "
             "define stream S2 (symbol string, price float, volume long); "
             "define stream S3 (symbol string, price float, volume long); "
             "partition with (symbol of S1, symbol of S2, symbol of S3) begin @info(name='q') "
             "from every (e1=S1[price>20] and e2=S2[price>20]) -> not S3[price>e1.price] for 5 sec within 10 sec "
             "select e1.symbol as symbol, sum(e1.price) as s insert into Out; end;")
    keys = 200
    g = small_stream(4, 120_000, keys)
    cols = columns_for(cq, g)
    ci = cq.program["aggregate"]["column"]
    col = cols[ci]
    ora = run(OracleEngine(cq.program_json(), 0), cq, g)
    want = _fold(ora, cq, g, lambda q: float(col[q]))
    eng = HipEngine(cq.program_json(), 0, max_keys=keys, max_batch=1 << 16, match_layout=LAYOUT_AGG)
    assert eng.path == 0
    got = _got(run(eng, cq, g, 30_011))
    _check(want, got, exact=True)
    assert sum(len(x) for x in want.values()) > 500


def test_lanes_aggregate_snapshot_restore():
    """The per-key aggregate state is part of the lanes' arena: a snapshot restored into a fresh
    engine continues the running values exactly."""
    from siddhi_amd.native import LAYOUT_AGG, HipEngine
    cq = _cq("define stream StockStream (symbol string, price float, volume long); "
             "partition with (symbol of StockStream) begin @info(name='q') "
             "from every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] within 1 sec "
             "select e1.symbol as symbol, avg(e1.price) as a insert into Out; end;")
    g = small_stream(2, 60_000, 300)
    price = columns_for(cq, g)[0]
    want = _fold(run(OracleEngine(cq.program_json(), 0), cq, g), cq, g, lambda q: float(price[q]))
    half = {k: v[:30_000] for k, v in g.items()}
    rest = {k: v[30_000:] for k, v in g.items()}
    a = HipEngine(cq.program_json(), 0, max_keys=300, max_batch=1 << 16, match_layout=LAYOUT_AGG)
    first = _got(run(a, cq, half))
    b = HipEngine(cq.program_json(), 0, max_keys=300, max_batch=1 << 16, match_layout=LAYOUT_AGG)
    b.restore(a.snapshot())
    # the restored engine continues the stream's sequence numbers from the snapshot
    second = _got(run(b, cq, rest))
    got = {}
    for part in (first, second):
        for k, v in part.items():
            got.setdefault(k, []).extend(v)
    _check(want, got, exact=True)
