"""Host-side mirror of the reference's embedding API for the state path.

Mirrors the names and argument meaning of ``SiddhiManager.createSiddhiAppRuntime``
(``core/SiddhiManager.java:93-95``), ``SiddhiAppRuntime.getInputHandler/addCallback/
start/shutdown`` (``core/SiddhiAppRuntime.java:115-191``), ``InputHandler.send``
(``core/stream/input/InputHandler.java:50-92``) and ``QueryCallback.receive``
(``core/query/output/callback/QueryCallback.java``), so that parity tests read like
the reference's own TestNG tests.

Events are buffered host-side as SoA columns and pushed to the engine in batches
(the columnar boundary of ``north_star``).  Each event keeps the semantics of one
``InputHandler.send(long, Object[])`` call; batching changes nothing except that
callbacks fire at ``flush()`` (or ``shutdown()``) rather than synchronously.

The engine is ``libsiddhi_hip.so`` (:mod:`siddhi_amd.native`).  There is no CPU
fallback: constructing a runtime without the HIP library raises.
"""
from __future__ import annotations

import time
from typing import Callable, Dict, List, Optional

import numpy as np

from .flow import TimestampGenerator, in_partition_flow
from .query.compiler import Dictionary, compile_app
from .history import ChainRings, RowHistory, decode_pairs32
from .query.selector import Selector

_NP = {"int": np.int32, "long": np.int64, "float": np.float32, "double": np.float64,
       "bool": np.uint8, "string": np.int32}


class Event:
    """Mirrors io.siddhi.core.event.Event (timestamp + data)."""

    __slots__ = ("timestamp", "data")

    def __init__(self, timestamp, data):
        self.timestamp = timestamp
        self.data = data

    def getTimestamp(self):
        return self.timestamp

    def getData(self, i=None):
        return self.data if i is None else self.data[i]

    def __repr__(self):
        return f"Event{{timestamp={self.timestamp}, data={self.data}}}"


def java_key_string(v) -> str:
    """String.valueOf(Object) for partition keys (ValuePartitionExecutor.java:34-40)."""
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float):
        r = repr(float(np.float32(v))) if v == float(np.float32(v)) else repr(v)
        return r
    return str(v)


class InputHandler:
    def __init__(self, runtime: "SiddhiAppRuntime", stream: str):
        self.rt = runtime
        self.stream = stream

    def getStreamId(self):
        return self.stream

    def send(self, *args):
        """send(Object[]) | send(long timestamp, Object[]) | send(Event) | send(Event[]).
        In playback the app clock is set from the event before it enters any junction
        (InputHandler.java:59-92; send(Event[]): from the last event), which is what fires absent
        timers on a send to any stream; send(Object[]) stamps wall-clock time and sets nothing."""
        tg = self.rt.timestamp_generator
        if len(args) == 2:
            if tg.playback:
                tg.set_current_timestamp(int(args[0]))
            self.rt._enqueue(self.stream, int(args[0]), list(args[1]))
            return
        (a,) = args
        if isinstance(a, Event):
            if tg.playback:
                tg.set_current_timestamp(int(a.timestamp))
            self.rt._enqueue(self.stream, int(a.timestamp), list(a.data))
        elif isinstance(a, (list, tuple)) and a and isinstance(a[0], Event):
            if tg.playback:
                tg.set_current_timestamp(int(a[-1].timestamp))
            for ev in a:
                self.rt._enqueue(self.stream, int(ev.timestamp), list(ev.data))
        else:
            self.rt._enqueue(self.stream, self.rt._now_ms(), list(a))


def _count_max(tree) -> int:
    """The largest count bound <min:max> of the program's state tree (CHAIN32's chain length)."""
    if not isinstance(tree, dict):
        return 0
    m = int(tree.get("max", 0)) if tree.get("t") == "count" else 0
    return max([m] + [_count_max(tree[c]) for c in ("a", "b", "x") if c in tree])


class _QueryRun:
    """One query's engine and what GpuStateStreamRuntime holds beside it: the pushed rows by
    sequence number (RowHistory = ColumnarBatch's history, trimmed by the engine's oldest live
    sequence number) and, for CHAIN32, the per-key rings of the last M events."""

    def __init__(self, rt, cq, engine, min_trim):
        self.cq = cq
        self.engine = engine
        self.history = RowHistory(min_trim)
        self.selector = Selector(cq, self.history, rt.strings)
        self.callbacks: List[Callable] = []
        self.streams = set(cq.partition_keys.keys()) if cq.partition_keys else \
            {lf.stream for lf in cq.leaves}
        self.stream_idx = cq.stream_index
        self.rows: List[tuple] = []
        self.compact = hasattr(engine, "push_compact") and rt.compact
        self.layout = engine.stat("match_layout") if self.compact else 0
        self.rings = ChainRings(_count_max(cq.program["tree"])) if self.layout == 4 else None
        self.retain = rt.retain and hasattr(engine, "oldest_live_seq")
        # absent states: the query's Scheduler listens to the app clock (Scheduler.java:71-103)
        self.timers = any(st.get("absent") for st in cq.program["states"])
        # pipelined ingest (shp_stage_batch / shp_run_staged): the batch whose H2D is in flight while
        # the next one is built -- (rows, ts, key, stream) -- run at the next push or at a drain point
        self.pipelined = rt.pipelined and self.compact and hasattr(engine, "stage")
        self.inflight = None
        self.narrow_batches = 0  # staged in the narrow form (tests)


class SiddhiAppRuntime:
    def __init__(self, text: str, engine_factory: Callable, start_clock: Optional[int] = None,
                 batch_size: int = 1 << 20, native_lowering: bool = False, compact: bool = False,
                 retain: bool = True, min_trim: int = 4096, pipelined: bool = False, narrow: bool = False):
        """native_lowering: engines are created from the SiddhiQL text by the library
        (shp_engine_create_siddhiql), as the Java host does; string values then use the library's
        dictionary, shared with the lowering's filter constants.
        batch_size: events per push (1 = GpuStateStreamRuntime's FlushPolicy.SYNC with single sends).
        compact: engines made with SHP_LAYOUT_COMPACT and pushed with shp_push_batch_compact, the
        records decoded on the host (PAIRS32 / CHAIN32), as the Java binding does.
        retain / min_trim: keep the pushed rows only from the engine's oldest live sequence number on
        (history.RowHistory), asking the engine once the kept rows reach min_trim and have doubled.
        pipelined (with compact and batch_size > 1, GpuStateStreamRuntime's PIPELINED flush): each
        flush stages its batch (shp_stage_batch: the H2D on the engine's copy stream) and runs the
        batch staged before it (shp_run_staged), so batch i+1's copies overlap batch i's kernels; the
        callbacks of a batch arrive one flush later, and every drain point
        (shutdown, advance_time, heartbeat) runs the batch still staged first.
        narrow (with pipelined): a staged batch whose ts lie within 2^31 ms of its first goes in the
        narrow form (shp_stage_batch_narrow: 4-byte ts offsets from that first ts, 2-byte key ids, as
        ColumnarBatch's narrow column sets under max_keys <= 65536); other batches in the wide form."""
        if pipelined and batch_size == 1:
            raise ValueError("pipelined ingest needs batched flushes (batch_size > 1)")
        if narrow and not pipelined:
            raise ValueError("the narrow ingest form is a form of the pipelined flush")
        self.pipelined = pipelined
        self.narrow = narrow
        self.compact = compact
        self.retain = retain
        self.min_trim = min_trim
        self.text = text
        self.native_lowering = native_lowering
        if native_lowering:
            from .native import NativeDictionary
            self.strings = NativeDictionary()
        else:
            self.strings = Dictionary()
        self.keydict = Dictionary()
        self.app, self.compiled, _ = compile_app(text, self.strings)
        self.timestamp_generator = TimestampGenerator(self.app.playback, self.app.idle_time, self.app.increment)
        # rows not yet pushed: (stream idx, ts, data, query) -- stream -1 with a query name is that
        # query's clock-only row (its Scheduler heard the app clock move, under DEFERRED batching)
        self._events: List[tuple] = []
        self._pending: List[int] = []
        self._start_clock = start_clock
        self._engine_factory = engine_factory
        self._batch_size = batch_size
        self.queries: Dict[str, _QueryRun] = {}
        self._started = False
        self._t0 = int(time.time() * 1000)

    # ----------------------------------------------------------------- API
    def getInputHandler(self, stream: str) -> InputHandler:
        if stream not in self.app.streams:
            raise KeyError(f"stream {stream} not defined")
        return InputHandler(self, stream)

    def addCallback(self, name: str, callback: Callable):
        """QueryCallback when ``name`` is a query; StreamCallback when it is an output stream."""
        self._ensure_queries()
        if name in self.queries:
            self.queries[name].callbacks.append(callback)
            return
        hit = [qr for qr in self.queries.values() if qr.cq.query.out_stream == name]
        if not hit:
            raise KeyError(f"no query or output stream named {name}")
        for qr in hit:
            qr.callbacks.append(callback)

    def start(self):
        self._ensure_queries()
        self._started = True

    def shutdown(self):
        self.flush()
        self._run_inflight()

    def _run_inflight(self, qr: Optional[_QueryRun] = None):
        """Drain point of the pipelined flush: the batch still staged runs before the clock moves or
        results are read (its sequence numbers precede whatever the engine sees next)."""
        for q in ([qr] if qr is not None else list(self.queries.values())):
            if q.inflight is not None:
                self._finish(q)

    def _now_ms(self):
        return int(time.time() * 1000)

    def _ensure_queries(self):
        if self.queries:
            return
        start = self._start_clock if self._start_clock is not None else (0 if self.app.playback else self._t0)
        kw = {"match_layout": 5} if self.compact else {}  # SHP_LAYOUT_COMPACT
        for cq in self.compiled:
            if self.native_lowering:
                eng = self._engine_factory(cq.program_json(), start, siddhiql=(self.text, cq.name, self.strings), **kw)
                if eng.program_json != cq.program_json():
                    raise AssertionError(f"native lowering of {cq.name} differs from query.compiler")
            else:
                eng = self._engine_factory(cq.program_json(), start, **kw)
            qr = _QueryRun(self, cq, eng, self.min_trim)
            self.queries[cq.name] = qr
            if qr.timers:
                self.timestamp_generator.add_time_change_listener(
                    lambda now, qr=qr: self._on_time_change(qr, now))

    def _enqueue(self, stream: str, ts: int, data: list):
        self._ensure_queries()
        sidx = list(self.app.streams.keys()).index(stream)
        # a query's clock-only row at this ts just before its own stream's event: the event carries
        # the same clock (ColumnarBatch.append absorbs it the same way)
        ev = self._events
        j = len(ev)
        while j > 0 and ev[j - 1][0] < 0 and ev[j - 1][1] == ts:
            j -= 1
        for i in range(len(ev) - 1, j - 1, -1):
            if stream in self.queries[ev[i][3]].streams:
                del ev[i]
                self._pending.pop()
        ev.append((sidx, ts, tuple(data), None))
        self._pending.append(len(ev) - 1)
        if len(self._pending) >= self._batch_size:
            self.flush()

    def _on_time_change(self, qr: _QueryRun, now: int):
        """The query's TimeChangeListener (Scheduler.java:71-103; GpuStateStreamRuntime.onTimeChange):
        one push per send (batch_size 1, FlushPolicy.SYNC) fires the due timers at once, before the
        event that moved the clock; batched (DEFERRED) a clock-only row joins the batch."""
        self._ensure_queries()
        if self._batch_size == 1:
            self.flush()
            self._run_inflight(qr)
            qr.engine.advance(int(now))
            self._drain(qr)
            self._trim(qr)
            return
        self._events.append((-1, int(now), (), qr.cq.name))
        self._pending.append(len(self._events) - 1)
        if len(self._pending) >= self._batch_size:
            self.flush()

    def advance_time(self, now: int):
        """Time passes to `now` with no event (a test's Thread.sleep).  Playback: an injected clock
        move (the idle heartbeat's setCurrentTimestamp), heard by the timer queries' listeners.  Live:
        each timer query's wall-clock wake-up (Scheduler.schedule / EventCaller.run,
        Scheduler.java:129-155, 287-326; GpuStateStreamRuntime.scheduleWake) runs at every due time
        shp_engine_next_due reports up to `now`, and fires the timers due then."""
        self._ensure_queries()
        self.flush()
        if self.app.playback:
            self.timestamp_generator.set_current_timestamp(int(now))
            self.flush()
            self._run_inflight()
            return
        self._run_inflight()
        for qr in self.queries.values():
            if not qr.timers:
                continue
            while True:
                due = qr.engine.next_due() if hasattr(qr.engine, "next_due") else None
                if due is None or due > now:
                    break
                qr.engine.advance(due)
                self._drain(qr)
            self._trim(qr)

    def heartbeat(self, wall_ms: int):
        """The playback idle heartbeat (TimestampGeneratorImpl.TimeInjector) at wall-clock wall_ms."""
        self._ensure_queries()
        self.flush()
        if self.timestamp_generator.heartbeat(int(wall_ms)):
            self.flush()
        self._run_inflight()

    # ---------------------------------------------------------------- flush
    def flush(self):
        if not self._pending:
            return
        ids = self._pending
        self._pending = []
        events = self._events
        self._events = []  # the queries' histories keep what their engines may still name
        ids = [i - ids[0] for i in ids]
        stream_names = list(self.app.streams.keys())
        for qr in self.queries.values():
            # the query's own streams' events and its own clock-only rows (the listener's)
            sel = [i for i in ids if (events[i][3] == qr.cq.name if events[i][0] < 0
                                      else stream_names[events[i][0]] in qr.streams)]
            if not sel:
                continue
            self._push(qr, [events[i][:3] for i in sel], stream_names)

    def _push(self, qr: _QueryRun, evs: List[tuple], stream_names):
        n = len(evs)
        ts = np.empty(n, np.int64)
        key = np.zeros(n, np.int32)
        stream = np.empty(n, np.int32)
        cols = []
        nulls = []
        for (s, a, t) in qr.cq.columns:
            cols.append(np.zeros(n, _NP[t]))
            nulls.append(np.zeros(n, np.uint8))
        pk = qr.cq.partition_keys
        for j, ev in enumerate(evs):
            s, t, data = ev
            ts[j] = t
            stream[j] = s
            if s < 0:  # clock-only: no key, no values (the kernels never read a stream -1 row's
                continue  # values, so its null flags stay 0)
            sname = stream_names[s]
            if pk is not None:
                attr = pk[sname]
                ai = [x[0] for x in self.app.streams[sname].attrs].index(attr)
                key[j] = self.keydict(java_key_string(data[ai]))
            for c, (cs, ca, ct) in enumerate(qr.cq.columns):
                if cs != s:
                    nulls[c][j] = 1
                    continue
                v = data[ca]
                if v is None:
                    nulls[c][j] = 1
                elif ct == "string":
                    cols[c][j] = self.strings(v)
                else:
                    cols[c][j] = v
        null_ptrs = [m if m.any() else None for m in nulls]
        if qr.pipelined:
            # stage this batch, then run the one staged before it: its kernels overlap these copies
            d = ts - ts[0] if n else ts
            if (self.narrow and getattr(qr.engine, "max_keys", 1 << 30) <= 65536 and n
                    and int(d.min()) >= -(1 << 31) and int(d.max()) < (1 << 31)):
                qr.engine.stage(ts, key, stream, cols, null_ptrs, ts32=d.astype(np.int32), ts_base=int(ts[0]),
                                key16=key.astype(np.uint16))
                qr.narrow_batches += 1
            else:
                qr.engine.stage(ts, key, stream, cols, null_ptrs)
            if qr.inflight is not None:
                self._finish(qr)
            qr.inflight = (list(evs), ts, key, stream)
            return
        if qr.compact:
            res = qr.engine.push_compact(ts, key, stream, cols, null_ptrs)
        else:
            qr.engine.push(ts, key, stream, cols, null_ptrs)
            res = None
        self._commit(qr, list(evs), ts, key, stream, res)

    def _finish(self, qr: _QueryRun):
        """shp_run_staged of the query's oldest staged batch, then its records as a push's."""
        evs, ts, key, stream = qr.inflight
        qr.inflight = None
        self._commit(qr, evs, ts, key, stream, qr.engine.run_staged())

    def _commit(self, qr: _QueryRun, evs, ts, key, stream, res):
        # the engine took the push (its sequence counter moved by n): the rows join the history
        seq0 = qr.history.add_block(evs)
        if res is not None and res["layout"] == 3:  # PAIRS32
            for i, slots in decode_pairs32(res["words"], seq0):
                self._deliver(qr, int(key[i]), int(ts[i]), 0, slots)
        elif res is not None and res["layout"] == 4:  # CHAIN32
            for i, slots in qr.rings.decode(res["words"], key, stream >= 0, seq0):
                self._deliver(qr, int(key[i]), int(ts[i]), 0, slots)
        else:
            self._drain(qr, res)
        self._trim(qr)

    def _trim(self, qr: _QueryRun):
        if qr.retain:
            qr.history.maybe_trim(qr.engine.oldest_live_seq)

    def _deliver(self, qr: _QueryRun, key: int, ts: int, etype: int, slots):
        """One match into the selector inside its key's partition flow, as the reference emits it
        (PartitionStreamReceiver.send :262-272 for event matches, Scheduler.java:88-97 for timer
        matches): the selector's per-key state is looked up under the flow (PartitionStateHolder)."""
        flow = self.keydict.strings[key] if qr.cq.partition_keys is not None else None
        if flow is None:
            return self._select(qr, ts, etype, slots)
        with in_partition_flow(flow):
            self._select(qr, ts, etype, slots)

    def _select(self, qr: _QueryRun, ts: int, etype: int, slots):
        row = qr.selector.select(ts, etype, slots)
        if row is None:
            return
        qr.rows.append((ts, row))
        for cb in qr.callbacks:
            cb(ts, [Event(ts, row)], None)

    def _drain(self, qr: _QueryRun, mb=None):
        """FULL records (slots name events by the engine's sequence numbers = history positions)."""
        if mb is None:
            mb = qr.engine.fetch()
        m = len(mb["key"])
        if m == 0:
            return
        S = mb["slot_len"].shape[1] if m else 0
        refs = mb["refs"]
        off = 0
        for i in range(m):
            slots = []
            for s in range(S):
                ln = int(mb["slot_len"][i, s])
                slots.append([int(x) for x in refs[off:off + ln]])
                off += ln
            self._deliver(qr, int(mb["key"][i]), int(mb["ts"][i]), int(mb["type"][i]), slots)


class SiddhiManager:
    """Mirrors io.siddhi.core.SiddhiManager for the state path."""

    def __init__(self, engine_factory: Optional[Callable] = None):
        if engine_factory is None:
            from .native import HipEngine  # fails loudly when libsiddhi_hip.so is missing
            engine_factory = HipEngine
        self.engine_factory = engine_factory

    def createSiddhiAppRuntime(self, text: str, **kw) -> SiddhiAppRuntime:
        return SiddhiAppRuntime(text, self.engine_factory, **kw)

    def shutdown(self):
        pass
