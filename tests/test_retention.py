"""Retention of the host's rows by the engine's oldest live sequence number, and the compact record
decoding -- the rules the Java binding follows (ColumnarBatch's history, GpuStateStreamRuntime's
PAIRS32 / CHAIN32 decoding), run through their Python mirror (siddhi_amd/history.py, runtime.py).

The reference keeps a StreamEvent alive exactly as long as a partial holds it
(StreamPreStateProcessor.java:364-403); the host keeps its copy of a row from
shp_engine_oldest_live_seq on.  These tests drive the mirror one push per event
(GpuStateStreamRuntime.FlushPolicy.SYNC with single sends, the case a fixed push history broke) and
require every match to resolve to a held row and the output to equal an unbounded run's.
CPU: the oracle reports the oldest live event (oracle_oldest_live_seq).  GPU: the HIP engine with
SHP_LAYOUT_COMPACT (PAIRS32 on the sweep, CHAIN32 on the count sequence) through
shp_push_batch_compact, against the oracle's rows.
"""
import numpy as np
import pytest

from oracle.oracle import OracleEngine
from siddhi_amd import synth
from siddhi_amd.history import ChainRings, EvictedRow, RowHistory, decode_pairs32
from siddhi_amd.runtime import SiddhiManager


def _oracle_factory(program_json, start, **kw):
    return OracleEngine(program_json, start)


def _events(cfg, n, keys, ms):
    """Synthetic (stream, ts, data) sends of a config's stream shape, `keys` symbols, `ms` apart."""
    spec = synth.StreamSpec(cfg if cfg != "3b" else 3, n, keys, 3 if cfg == 4 else 1, cfg == 4)
    g = synth.generate(spec, 0, n)
    ts = synth.T0 + (np.arange(n) * ms).astype(np.int64)
    streams = {4: ["S1", "S2", "S3"], 3: ["S"], "3b": ["S"]}.get(cfg, ["StockStream"])
    out = []
    for i in range(n):
        sym = f"k{int(g['key'][i])}"
        s = streams[int(g["stream"][i])]
        data = [sym, float(g["price"][i])] if cfg in (3, "3b") else [sym, float(g["price"][i]), int(g["volume"][i])]
        out.append((s, int(ts[i]), data))
    return out


def _run(factory, cfg, evs, **kw):
    rt = SiddhiManager(factory).createSiddhiAppRuntime(synth.QUERIES[cfg], **kw)
    handlers = {}
    for s, t, data in evs:
        h = handlers.get(s) or handlers.setdefault(s, rt.getInputHandler(s))
        h.send(t, data)
    rt.shutdown()
    return rt


def _rows(rt):
    return [(t, tuple(r)) for t, r in rt.queries["q"].rows]


# ------------------------------------------------------------------------------------ unit rules
def test_history_trim_keeps_live_tail_and_raises_below():
    h = RowHistory(min_trim=4)
    for b in ([1, 2, 3], [4], [5, 6, 7, 8]):
        h.add_block(b)
    assert h[0] == 1 and h[7] == 8 and h.kept == 8
    h.trim_below(2)  # block 0 partly below: its tail stays
    assert h.kept == 6 and h[2] == 3 and h[3] == 4
    with pytest.raises(EvictedRow):
        h[1]
    h.trim_below(5)
    assert h.kept == 3 and h[5] == 6 and h[7] == 8
    with pytest.raises(EvictedRow):
        h[8]  # not pushed yet


def test_history_asks_the_engine_only_when_rows_double():
    h = RowHistory(min_trim=10)
    asked = []

    def live():
        asked.append(h.next_seq)
        return h.next_seq - 3  # three rows stay live
    for i in range(1000):
        h.add_block([i])
        h.maybe_trim(live)
    assert h.kept <= 10 and len(asked) <= 1000 // 7 + 1  # a query per >= min_trim - 3 pushes
    assert h[999] == 999 and h[997] == 997


def test_pairs32_decode_restores_arrival_order_stably():
    # owner order: key B's match (e2 at 5) before key A's two (e2 at 2, candidates 0 then 1)
    w = np.array([5, 1, 2, 2, 2, 1], np.uint32)
    got = decode_pairs32(w, 100)
    assert got == [(2, [[100], [102]]), (2, [[101], [102]]), (5, [[104], [105]])]


def test_chain32_rings_follow_each_keys_events_across_pushes():
    r = ChainRings(3)
    keys = np.array([7, 8, 7, 7], np.int32)
    ok = np.ones(4, bool)
    # a match at row 3 (key 7) with L = 2: rows 0 and 2
    assert r.decode(np.array([3 | 2 << 28], np.uint32), keys, ok, 10) == [(3, [[10, 12], [13]])]
    # next push: key 7's chain of 3 reaches back into the first push (rows 12, 13 then row 0 here)
    got = r.decode(np.array([1 | 3 << 28], np.uint32), np.array([7, 7], np.int32), np.ones(2, bool), 14)
    assert got == [(1, [[12, 13, 14], [15]])]


# --------------------------------------------------------------- mirror vs unbounded, on the oracle
@pytest.mark.parametrize("cfg,n,keys,ms", [(2, 24_000, 1_000, 0.5), ("3b", 12_000, 500, 1),
                                            (3, 6_000, 300, 1), (4, 8_000, 50, 5)])
def test_sync_pushes_with_retention_equal_unbounded_run_oracle(cfg, n, keys, ms):
    evs = _events(cfg, n, keys, ms)
    want = _rows(_run(_oracle_factory, cfg, evs, retain=False))
    rt = _run(_oracle_factory, cfg, evs, batch_size=1, min_trim=64)
    h = rt.queries["q"].history
    assert _rows(rt) == want
    assert len(want) > 50 or cfg == 3  # C3 (no `every`) dies at its first failed e2: no output
    assert h.trims > 0 and h.dropped > n // 3, (h.trims, h.dropped)


# ---------------------------------------------------------------------- GPU: the engine's report
def _hip_factory(max_keys):
    from siddhi_amd.native import HipEngine

    def f(program_json, start, **kw):
        return HipEngine(program_json, start, max_keys=max_keys, max_batch=1 << 16, **kw)
    return f


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,n,keys,ms,layout", [(2, 200_000, 10_000, 0.05, 3), ("3b", 100_000, 1_000, 1, 4),
                                                  (5, 60_000, 2_000, 0.2, 3), (3, 20_000, 1_000, 1, 4),
                                                  (4, 20_000, 100, 5, 0)])
def test_sync_pushes_compact_with_engine_retention(cfg, n, keys, ms, layout):
    """C2 (10k keys, 2*10^5 pushes) and C3' (10^5 pushes) one event per push (C5, C3 and C4 shorter):
    the HIP engine's compact records decoded on the host, rows kept from shp_engine_oldest_live_seq on,
    the output equal to the oracle's.  A candidate the reference leaves on a pending list stays there
    until its key's next event, so at 10k keys the live rows span ~10^5 events (the least recently
    seen key's): the C2 run is long enough for the history to be trimmed well below what it pushed."""
    evs = _events(cfg, n, keys, ms)
    want = _rows(_run(_oracle_factory, cfg, evs, retain=False))
    rt = _run(_hip_factory(max(keys, 256)), cfg, evs, batch_size=1, compact=True, min_trim=256)
    q = rt.queries["q"]
    assert q.layout == layout
    assert _rows(rt) == want
    assert len(want) > 100 or cfg == 3
    # kept <= 2x the live span (trims when the rows double): at 10k keys C2's live span is ~8*10^4 events
    assert q.history.trims > 0 and q.history.dropped > n // 6, (q.history.trims, q.history.dropped)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,keys,ms", [(2, 2_000, 0.25), ("3b", 500, 1), (3, 300, 1), (4, 40, 2)])
def test_engine_oldest_live_seq_against_oracle(cfg, keys, ms):
    """After every push of a split stream: the engine's oldest live event is never before the
    oracle's (it holds no more than the reference), every match of later pushes names an event at or
    after it, and on the count sequence (no expiry) the two are equal."""
    from diff_util import columns_for, program_for
    from siddhi_amd.native import HipEngine
    spec = synth.StreamSpec(cfg if cfg != "3b" else 3, 40_000, keys, 3 if cfg == 4 else 1, cfg == 4)
    g = synth.generate(spec)
    g["ts"] = synth.T0 + (np.arange(len(g["ts"])) * ms).astype(np.int64)
    cq = program_for(cfg)
    cols = columns_for(cq, g)
    o = OracleEngine(cq.program_json(), 0)
    e = HipEngine(cq.program_json(), 0, max_keys=max(keys, 256), max_batch=1 << 16)
    n, step, floor = len(g["ts"]), 1_000, 0
    for lo in range(0, n, step):
        hi = min(n, lo + step)
        args = (g["ts"][lo:hi], g["key"][lo:hi], g["stream"][lo:hi], [c[lo:hi] for c in cols], [None] * len(cols))
        o.push(*args)
        e.push(*args)
        mb = e.fetch()
        o.fetch()
        refs = mb["refs"][mb["refs"] >= 0]
        assert refs.size == 0 or refs.min() >= floor, (lo, int(refs.min()), floor)
        floor = e.oldest_live_seq()
        want = o.oldest_live_seq()
        assert floor >= want, (lo, floor, want)
        if cfg in (3, "3b"):
            assert floor == want, (lo, floor, want)
        assert floor <= hi


@pytest.mark.gpu
@pytest.mark.parametrize("narrow", [False, True])
@pytest.mark.parametrize("cfg,n,keys,ms,layout", [(2, 60_000, 2_000, 0.25, 3), ("3b", 40_000, 500, 1, 4),
                                                  (5, 40_000, 1_500, 0.2, 3), (4, 20_000, 100, 5, 0)])
def test_pipelined_batches_compact_with_engine_retention(cfg, n, keys, ms, layout, narrow):
    """The pipelined flush (FlushPolicy.PIPELINED's mirror: shp_stage_batch[_narrow] / shp_run_staged,
    one batch in flight) with compact records decoded per run -- PAIRS32, CHAIN32 (the rings walk the
    runs in stage order), FULL for C4 -- rows kept from shp_engine_oldest_live_seq on: the output equal
    to the oracle's."""
    evs = _events(cfg, n, keys, ms)
    want = _rows(_run(_oracle_factory, cfg, evs, retain=False))
    rt = _run(_hip_factory(max(keys, 256)), cfg, evs, batch_size=997, compact=True, min_trim=256, pipelined=True,
              narrow=narrow)
    q = rt.queries["q"]
    assert q.layout == layout and q.pipelined and q.inflight is None
    assert (q.narrow_batches > 0) == narrow
    assert _rows(rt) == want
    assert len(want) > 100 or cfg == 3
