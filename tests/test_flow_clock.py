"""Match egress inside the match's partition flow, and the app clock reaching absent-state timers --
the rules the Java drop-in follows (GpuStateStreamRuntime.emit / onTimeChange / scheduleWake), run
through their Python mirror (siddhi_amd/flow.py, runtime.py), against the oracle driven directly.

* Egress: the reference emits every match inside its key's flow (PartitionStreamReceiver.java:262-272,
  Scheduler.java:88-97) and the selector's aggregators are per flow (PartitionStateHolder.java:43-48).
  The mirror's selector reads the flow, so a delivery outside it aggregates under the wrong key: C5's
  avg with many keys per push (FlushPolicy.DEFERRED) is compared per key with a running mean computed
  here from the oracle's raw matches (1e-6 relative, the north_star bound), and the same run with the
  flow removed must differ (the test sees the defect class).
* Clock: a playback send on a stream the query does not read moves the app clock before anything else
  (InputHandler.java:59-92); the query's TimeChangeListener (Scheduler.java:71-103) fires the timers.
  So does the idle.time heartbeat (TimestampGeneratorImpl.java:165-185; the fixture
  AbsentWithEveryPatternTestCase.java:277-310), and in live mode the wall-clock wake-up at
  shp_engine_next_due (Scheduler.java:129-155, 287-326).  Expected rows: the oracle pushed one send
  at a time, other streams' sends as clock-only rows, clock moves as oracle advances.
"""
import numpy as np
import pytest

from oracle.oracle import OracleEngine
from siddhi_amd import synth
from siddhi_amd.flow import get_partition_flow_id, in_partition_flow, start_partition_flow, stop_partition_flow
from siddhi_amd.query.compiler import compile_app
from siddhi_amd.runtime import SiddhiManager

F32 = lambda x: float(np.float32(x))  # noqa: E731


def _oracle_factory(program_json, start, **kw):
    return OracleEngine(program_json, start)


def _hip_factory(max_keys):
    from siddhi_amd.native import HipEngine

    def f(program_json, start, **kw):
        return HipEngine(program_json, start, max_keys=max_keys, max_batch=1 << 16, **kw)
    return f


def _c_sends(cfg, n, keys, ms, t0=synth.T0):
    """(stream, ts, data) sends of config cfg's stream shape (symbols 'k<id>'), `ms` apart."""
    spec = synth.StreamSpec(cfg, n, keys, 3 if cfg == 4 else 1, cfg == 4)
    g = synth.generate(spec, 0, n)
    names = ["S1", "S2", "S3"] if cfg == 4 else ["StockStream"]
    return [(names[int(g["stream"][i])], int(t0 + round(i * ms)),
             [f"k{int(g['key'][i])}", float(g["price"][i]), int(g["volume"][i])]) for i in range(n)]


class Direct:
    """The oracle driven without the mirror: one push per send (the query's streams as events,
    every other stream as a clock-only row), clock moves as oracle advances.  Keeps every row so
    match slots resolve to the sent data, and the matches in emission order with their key string."""

    def __init__(self, app_text, start_clock=0):
        self.app, qs, self.strings = compile_app(app_text)
        self.cq = qs[0]
        self.names = [s["name"] for s in self.cq.program["streams"]]
        self.eng = OracleEngine(self.cq.program_json(), start_clock)
        self.keys, self.rows, self.matches = {}, [], []

    def send(self, stream, ts, data):
        cq = self.cq
        n = len(cq.columns)
        cols = [np.zeros(1, {"float": np.float32, "double": np.float64, "int": np.int32, "long": np.int64,
                             "string": np.int32, "bool": np.uint8}[t]) for (_, _, t) in cq.columns]
        nul = [np.ones(1, np.uint8) for _ in range(n)]
        key = 0
        mine = set(cq.partition_keys) if cq.partition_keys else {lf.stream for lf in cq.leaves}
        sidx = self.names.index(stream) if stream in mine else -1
        if sidx >= 0:
            for c, (cs, ca, ct) in enumerate(cq.columns):
                if cs == sidx and data[ca] is not None:
                    cols[c][0] = self.strings(data[ca]) if ct == "string" else data[ca]
                    nul[c][0] = 0
            if cq.partition_keys is not None:
                attrs = [a[0] for a in self.app.streams[stream].attrs]
                k = str(data[attrs.index(cq.partition_keys[stream])])
                key = self.keys.setdefault(k, len(self.keys))
        self.rows.append((stream, ts, data))
        self.eng.push(np.array([ts], np.int64), np.array([key], np.int32), np.array([sidx], np.int32), cols, nul)
        self._take()

    def advance(self, now):
        self.eng.advance(int(now))
        self._take()

    def _take(self):
        mb = self.eng.fetch()
        names = {v: k for k, v in self.keys.items()}
        off = 0
        for i in range(len(mb["key"])):
            slots = []
            for s in range(mb["slot_len"].shape[1]):
                ln = int(mb["slot_len"][i, s])
                slots.append([self.rows[int(x)][2] for x in mb["refs"][off:off + ln]])
                off += ln
            self.matches.append((names.get(int(mb["key"][i])), int(mb["ts"][i]), int(mb["type"][i]), slots))


def _by_key(rows, kpos=0):
    out = {}
    for ts, r in rows:
        out.setdefault(r[kpos], []).append((ts, r))
    return out


def _run_mirror(factory, app, sends, batch, compact=False, advances=None, **kw):
    rt = SiddhiManager(factory).createSiddhiAppRuntime(app, batch_size=batch, compact=compact, **kw)
    rt.start()
    handlers = {}
    for i, (s, t, data) in enumerate(sends):
        h = handlers.get(s) or handlers.setdefault(s, rt.getInputHandler(s))
        h.send(t, data)
        if advances and i in advances:
            rt.advance_time(advances[i])
    rt.shutdown()
    return rt.queries["q"]


# ----------------------------------------------------------------------------------- flow rules
def test_partition_flow_is_thread_local_and_restored():
    import threading
    stop_partition_flow()
    with in_partition_flow("A"):
        assert get_partition_flow_id() == "A"
        with in_partition_flow("B"):
            assert get_partition_flow_id() == "B"
        assert get_partition_flow_id() == "A"  # a delivery inside another key's send leaves it as it was
        seen = []
        th = threading.Thread(target=lambda: seen.append(get_partition_flow_id()))
        th.start()
        th.join()
        assert seen == [None]
    assert get_partition_flow_id() is None
    start_partition_flow(None)


# -------------------------------------------------------------- C5 egress: per-key avg, DEFERRED
C5_N, C5_KEYS = 30_000, 1_500


def _c5_expected(sends):
    """Per symbol: the running mean of e2.price over that key's matches in emission order
    (AvgAttributeAggregatorExecutor: double sum / long count), from the oracle's raw matches."""
    d = Direct(synth.QUERIES[5])
    for s in sends:
        d.send(*s)
    acc, out = {}, {}
    for key, ts, typ, slots in d.matches:
        e1, e2 = slots[0][0], slots[1][0]
        sm, c = acc.get(key, (0.0, 0))
        sm, c = sm + F32(e2[1]), c + 1
        acc[key] = (sm, c)
        out.setdefault(key, []).append((ts, [e1[0], sm / c]))
    assert all(k == v[0][1][0] for k, v in out.items())  # e1.symbol is the key
    return out


def _assert_rows_close(got, want):
    assert set(got) == set(want)
    for k in want:
        assert len(got[k]) == len(want[k]), k
        for (tg, rg), (tw, rw) in zip(got[k], want[k]):
            assert tg == tw and rg[0] == rw[0], (k, tg, tw)
            assert abs(rg[1] - rw[1]) <= 1e-6 * abs(rw[1]), (k, rg, rw)


@pytest.fixture(scope="module")
def c5_case():
    sends = _c_sends(5, C5_N, C5_KEYS, 0.2)
    return sends, _c5_expected(sends)


@pytest.mark.parametrize("batch", [1, 4096])
def test_c5_avg_per_key_in_flow_oracle(c5_case, batch):
    sends, want = c5_case
    q = _run_mirror(_oracle_factory, synth.QUERIES[5], sends, batch)
    got = _by_key(q.rows)
    assert sum(len(v) for v in want.values()) > 2_000
    _assert_rows_close(got, want)


def test_c5_avg_outside_the_flow_is_detected(c5_case):
    """Negative control: deliveries with no flow (the defect of a host that calls selector.process
    outside startPartitionFlow) aggregate every key under one state -- the comparison catches it."""
    sends, want = c5_case
    rt = SiddhiManager(_oracle_factory).createSiddhiAppRuntime(synth.QUERIES[5], batch_size=4096)
    rt._deliver = lambda qr, key, ts, etype, slots: rt._select(qr, ts, etype, slots)
    h = rt.getInputHandler("StockStream")
    for s, t, data in sends:
        h.send(t, data)
    rt.shutdown()
    with pytest.raises(AssertionError):
        _assert_rows_close(_by_key(rt.queries["q"].rows), want)


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [1, 4096, 1 << 16])
def test_c5_avg_per_key_in_flow_hip_compact(c5_case, batch):
    """The HIP engine's PAIRS32 records (many keys per push), decoded on the host and delivered per
    match inside its key's flow: per-key avg equal to the oracle's running mean."""
    sends, want = c5_case
    q = _run_mirror(_hip_factory(C5_KEYS), synth.QUERIES[5], sends, batch, compact=True)
    assert q.layout == 3
    _assert_rows_close(_by_key(q.rows), want)


# ------------------------------------------------ C4 timers fired by a send to another stream
C4_TIMER_APP = synth.QUERIES[4].replace("@app:playback ", "@app:playback define stream TimerStream (symbol string); ")


def _c4_timer_sends():
    """C4 sends for 40 keys, a TimerStream send every 50th, then 12 s of TimerStream sends only: the
    timers armed by the last events fire only through the app clock."""
    base = _c_sends(4, 6_000, 40, 2.0)
    sends = []
    for i, s in enumerate(base):
        sends.append(s)
        if i % 50 == 49:
            sends.append(("TimerStream", s[1], ["tick"]))
    t = base[-1][1]
    for j in range(1, 25):
        sends.append(("TimerStream", t + 500 * j, ["tick"]))
    return sends, base[-1][1]


def _c4_expected(sends):
    d = Direct(C4_TIMER_APP)
    for s in sends:
        d.send(*s)
    sid = {st["ref"]: st["id"] for st in d.cq.program["states"]}  # (Logical: e2's state is numbered first)
    a, b = sid["e1"], sid["e2"]
    rows = [(ts, [sl[a][0][0], F32(sl[a][0][1]), F32(sl[b][0][1])]) for _, ts, typ, sl in d.matches if typ == 0]
    return _by_key(rows)


@pytest.fixture(scope="module")
def c4_case():
    sends, last_event = _c4_timer_sends()
    want = _c4_expected(sends)
    late = sum(1 for v in want.values() for ts, _ in v if ts > last_event)
    assert late > 10  # matches only the TimerStream's clock fires
    return sends, want


@pytest.mark.parametrize("batch", [1, 997])
def test_c4_timers_fire_on_other_stream_sends_oracle(c4_case, batch):
    sends, want = c4_case
    q = _run_mirror(_oracle_factory, C4_TIMER_APP, sends, batch)
    assert _by_key(q.rows) == want


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [1, 997])
def test_c4_timers_fire_on_other_stream_sends_hip(c4_case, batch):
    sends, want = c4_case
    q = _run_mirror(_hip_factory(64), C4_TIMER_APP, sends, batch, compact=True)
    assert q.engine.path == 4
    assert _by_key(q.rows) == want


# ---------------------------------------------------------------- the idle.time heartbeat fixture
HB_APP = ("@app:playback(idle.time = '10 milliseconds', increment = '10 milliseconds') "
          "define stream Stream1 (symbol string, price float, volume int); "
          "@info(name = 'q') from every e1=Stream1[price>20] -> not Stream1[symbol==e1.symbol and "
          "price>e1.price] for 1sec select e1.symbol as symbol insert into OutputStream ;")
HB_SENDS = [("Stream1", 1544512385000, ["WSO2", 55.6, 100]), ("Stream1", 1544512385100, ["GOOG", 55.6, 100]),
            ("Stream1", 1544512385800, ["WSO2", 55.7, 100]), ("Stream1", 1544512386200, ["GOOG", 55.6, 100])]


def _heartbeat_run(factory, batch, **kw):
    wall = [0]
    rt = SiddhiManager(factory).createSiddhiAppRuntime(HB_APP, batch_size=batch, **kw)
    rt.timestamp_generator._wall = lambda: wall[0]
    rt.start()
    h = rt.getInputHandler("Stream1")
    for s, t, data in HB_SENDS:
        h.send(t, data)
        wall[0] += 1
    rt.flush()
    at_sends = [r for _, r in rt.queries["q"].rows]
    clocks = []
    for _ in range(150):  # no event for 1.5 s of wall time: the clock steps 10 ms per heartbeat
        wall[0] += 10
        rt.heartbeat(wall[0])
        clocks.append(rt.timestamp_generator.current_time())
    rt.shutdown()
    return at_sends, rt.queries["q"].rows, clocks


@pytest.mark.parametrize("batch", [1, 64])
def test_idle_heartbeat_fixture_oracle(batch):
    at_sends, rows, clocks = _heartbeat_run(_oracle_factory, batch)
    assert at_sends == [["GOOG"]]  # AbsentWithEveryPatternTestCase.testQuery7's assertion
    assert clocks[0] == HB_SENDS[-1][1] + 10 and clocks[-1] == HB_SENDS[-1][1] + 1500
    d = Direct(HB_APP)
    for s in HB_SENDS:
        d.send(*s)
    for c in clocks:
        d.advance(c)
    want = [(ts, [sl[0][0][0]]) for _, ts, typ, sl in d.matches if typ == 0]
    assert [r for _, r in want] == [["GOOG"], ["WSO2"], ["GOOG"]]
    assert rows == want


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [1, 64])
def test_idle_heartbeat_fixture_hip(batch):
    at_sends, rows, _ = _heartbeat_run(_hip_factory(256), batch, compact=True)
    assert at_sends == [["GOOG"]]
    assert [r for _, r in rows] == [["GOOG"], ["WSO2"], ["GOOG"]]
    assert [t for t, _ in rows] == [1544512386100, 1544512386800, 1544512387200]


# ------------------------------------------------------------- live mode: the wall-clock wake-up
LIVE_APP = ("define stream S1 (symbol string, price float, volume long); "
            "define stream S2 (symbol string, price float, volume long); "
            "partition with (symbol of S1, symbol of S2) begin "
            "@info(name='q') from every e1=S1[price>20] -> not S2[price>e1.price] for 1 sec "
            "select e1.symbol as s, e1.price as p insert into Out; end;")


def _live_case(n=3_000, keys=30):
    g = synth.generate(synth.StreamSpec(4, n, keys, 3, True), 0, n)
    sends, adv = [], {}
    t = 1_700_000_000_000
    for i in range(n):
        t += int(g["volume"][i] % 7)
        st = "S1" if g["stream"][i] != 1 else "S2"
        sends.append((st, t, [f"k{int(g['key'][i])}", float(g["price"][i]), int(g["volume"][i])]))
        if i % 97 == 96:  # Thread.sleep: 0.3 - 2.3 s of wall time with no event
            t += 300 + int(g["volume"][i]) * 2
            adv[i] = t
    return sends, adv


@pytest.fixture(scope="module")
def live_case():
    sends, adv = _live_case()
    d = Direct(LIVE_APP, start_clock=sends[0][1])
    for i, s in enumerate(sends):
        d.send(*s)
        if i in adv:
            d.advance(adv[i])
    want = _by_key([(ts, [sl[0][0][0], F32(sl[0][0][1])]) for _, ts, typ, sl in d.matches if typ == 0])
    assert sum(len(v) for v in want.values()) > 100
    return sends, adv, want


@pytest.mark.parametrize("batch", [1, 500])
def test_live_wakeup_at_next_due_oracle(live_case, batch):
    sends, adv, want = live_case
    q = _run_mirror(_oracle_factory, LIVE_APP, sends, batch, advances=adv, start_clock=sends[0][1])
    assert _by_key(q.rows) == want


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [1, 500])
def test_live_wakeup_at_next_due_hip(live_case, batch):
    sends, adv, want = live_case
    q = _run_mirror(_hip_factory(64), LIVE_APP, sends, batch, compact=True, advances=adv, start_clock=sends[0][1])
    assert q.engine.path == 0
    assert _by_key(q.rows) == want


@pytest.mark.gpu
@pytest.mark.parametrize("app,start", [(synth.QUERIES[4], 0), (LIVE_APP, 1_700_000_000_000)], ids=["labs", "lanes"])
def test_engine_next_due_equals_oracle(app, start):
    """shp_engine_next_due after every push: the earliest head of any key's timer queue, as the oracle's."""
    from siddhi_amd.native import HipEngine
    cq = compile_app(app)[1][0]
    g = synth.generate(synth.StreamSpec(4, 20_000, 50, 3, True), 0, 20_000)
    g["ts"] = start + np.arange(20_000, dtype=np.int64) * 3 if start else synth.T0 + np.arange(20_000) * 3
    if app is LIVE_APP:
        g["stream"] = np.where(g["stream"] == 1, 1, 0).astype(np.int32)
    from diff_util import columns_for
    cols = columns_for(cq, g)
    o = OracleEngine(cq.program_json(), start)
    e = HipEngine(cq.program_json(), start, max_keys=64, max_batch=1 << 14)
    assert e.next_due() is None and o.next_due() is None
    seen = 0
    for lo in range(0, 20_000, 1_999):
        hi = min(20_000, lo + 1_999)
        args = (g["ts"][lo:hi], g["key"][lo:hi], g["stream"][lo:hi], [c[lo:hi] for c in cols], [None] * len(cols))
        o.push(*args)
        e.push(*args)
        assert e.next_due() == o.next_due(), lo
        seen += o.next_due() is not None
    assert seen > 5


# ------------------------------------------- pipelined flush (shp_stage_batch / shp_run_staged)
class _StagedOracle(OracleEngine):
    """The oracle behind the staged-ingest interface (host-logic check of the pipelined flush on the
    CPU): stage() holds a copy of the batch, run_staged() pushes the oldest one.  Like the engine it
    refuses a third staged batch, and a clock move or due-time query with a batch still staged is the
    host's ordering defect, so it fails."""

    def __init__(self, program_json, start, **kw):
        super().__init__(program_json, start)
        self.staged = []
        self.max_staged = 0
        self.narrow = 0

    def stat(self, which):
        assert which == "match_layout"
        return 0  # FULL records

    def push_compact(self, ts, key, stream, cols, nulls):
        self.push(ts, key, stream, cols, nulls)
        out = self.fetch()
        out["layout"] = 0
        return out

    max_keys = 65536  # (so the mirror's narrow form applies)

    def stage(self, ts, key, stream, cols, nulls, ts32=None, ts_base=0, key16=None):
        """The narrow form is pushed as what the engine's k_widen_ts / k_widen_key rebuild from it."""
        assert len(self.staged) < 2, "two batches staged: run one first"
        if ts32 is not None:
            ts = ts_base + ts32.astype(np.int64)
            key = key16.astype(np.int32)
            self.narrow += 1
        self.staged.append(tuple(np.array(a, copy=True) for a in (ts, key, stream)) +
                           ([np.array(c, copy=True) for c in cols], [None if m is None else m.copy() for m in nulls]))
        self.max_staged = max(self.max_staged, len(self.staged))

    def run_staged(self):
        return self.push_compact(*self.staged.pop(0))

    def advance(self, now):
        assert not self.staged, "clock moved past a staged batch"
        super().advance(now)

    def next_due(self):
        assert not self.staged, "due time read with a batch staged"
        return super().next_due()


def _staged_oracle_factory(program_json, start, **kw):
    return _StagedOracle(program_json, start)


def test_pipelined_flush_needs_batches():
    with pytest.raises(ValueError):
        SiddhiManager(_oracle_factory).createSiddhiAppRuntime(synth.QUERIES[5], batch_size=1, compact=True,
                                                             pipelined=True)


@pytest.mark.parametrize("narrow", [False, True])
@pytest.mark.parametrize("case", ["c5", "c4", "live", "heartbeat"])
def test_pipelined_flush_host_logic(case, narrow, c5_case, c4_case, live_case):
    """The pipelined flush's ordering on the CPU: batch i runs after batch i+1 is staged, the rows join
    the history in run order, and every clock move / drain point runs the staged batch first -- the
    same rows as the unpipelined mirror and the Direct transcription."""
    f = _staged_oracle_factory
    if case == "c5":
        sends, want = c5_case
        q = _run_mirror(f, synth.QUERIES[5], sends, 4096, compact=True, pipelined=True, narrow=narrow)
        _assert_rows_close(_by_key(q.rows), want)
    elif case == "c4":
        sends, want = c4_case
        q = _run_mirror(f, C4_TIMER_APP, sends, 997, compact=True, pipelined=True, narrow=narrow)
        assert _by_key(q.rows) == want
    elif case == "live":
        sends, adv, want = live_case
        q = _run_mirror(f, LIVE_APP, sends, 500, compact=True, pipelined=True, narrow=narrow, advances=adv,
                        start_clock=sends[0][1])
        assert _by_key(q.rows) == want
    else:
        at_sends, rows, _ = _heartbeat_run(f, 64, compact=True, pipelined=True, narrow=narrow)
        assert at_sends == []  # the sends' batch is still staged at the first read (one flush late)
        assert [r for _, r in rows] == [["GOOG"], ["WSO2"], ["GOOG"]]
        q = None
    if q is not None:
        # (live mode's Thread.sleep every 97 sends drains before a 500-row batch fills)
        assert q.pipelined and q.inflight is None and q.engine.max_staged == (1 if case == "live" else 2)
        assert (q.narrow_batches > 0) == narrow and q.engine.narrow == q.narrow_batches


@pytest.mark.gpu
@pytest.mark.parametrize("narrow", [False, True])
@pytest.mark.parametrize("case", ["c5", "c4", "live", "heartbeat"])
def test_pipelined_flush_hip(case, narrow, c5_case, c4_case, live_case):
    """The mirror's pipelined flush through shp_stage_batch / shp_run_staged on the GPU: the same rows
    as the oracle (PAIRS32 for C5, the labs path's FULL records for C4, the lanes for live mode)."""
    if case == "c5":
        sends, want = c5_case
        q = _run_mirror(_hip_factory(C5_KEYS), synth.QUERIES[5], sends, 4096, compact=True, pipelined=True, narrow=narrow)
        assert q.layout == 3 and q.pipelined and (q.narrow_batches > 0) == narrow
        _assert_rows_close(_by_key(q.rows), want)
    elif case == "c4":
        sends, want = c4_case
        q = _run_mirror(_hip_factory(64), C4_TIMER_APP, sends, 997, compact=True, pipelined=True, narrow=narrow)
        assert q.engine.path == 4 and q.pipelined and (q.narrow_batches > 0) == narrow
        assert _by_key(q.rows) == want
    elif case == "live":
        sends, adv, want = live_case
        q = _run_mirror(_hip_factory(64), LIVE_APP, sends, 500, compact=True, pipelined=True, narrow=narrow, advances=adv,
                        start_clock=sends[0][1])
        assert q.pipelined
        assert _by_key(q.rows) == want
    else:
        at_sends, rows, _ = _heartbeat_run(_hip_factory(256), 64, compact=True, pipelined=True, narrow=narrow)
        assert [r for _, r in rows] == [["GOOG"], ["WSO2"], ["GOOG"]]
        assert [t for t, _ in rows] == [1544512386100, 1544512386800, 1544512387200]
