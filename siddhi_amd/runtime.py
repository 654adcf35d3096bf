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

from .query.compiler import Dictionary, compile_app
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
        """send(Object[]) | send(long timestamp, Object[]) | send(Event) | send(Event[])."""
        if len(args) == 2:
            self.rt._enqueue(self.stream, int(args[0]), list(args[1]))
            return
        (a,) = args
        if isinstance(a, Event):
            self.rt._enqueue(self.stream, int(a.timestamp), list(a.data))
        elif isinstance(a, (list, tuple)) and a and isinstance(a[0], Event):
            for ev in a:
                self.rt._enqueue(self.stream, int(ev.timestamp), list(ev.data))
        else:
            self.rt._enqueue(self.stream, self.rt._now_ms(), list(a))


class _QueryRun:
    def __init__(self, rt, cq, engine):
        self.cq = cq
        self.engine = engine
        self.selector = Selector(cq, rt._events, rt.strings)
        self.callbacks: List[Callable] = []
        self.local_to_app: List[int] = []
        self.streams = set(cq.partition_keys.keys()) if cq.partition_keys else \
            {lf.stream for lf in cq.leaves}
        self.stream_idx = cq.stream_index
        self.rows: List[tuple] = []


class SiddhiAppRuntime:
    def __init__(self, text: str, engine_factory: Callable, start_clock: Optional[int] = None,
                 batch_size: int = 1 << 20, native_lowering: bool = False):
        """native_lowering: engines are created from the SiddhiQL text by the library
        (shp_engine_create_siddhiql), as the Java host does; string values then use the library's
        dictionary, shared with the lowering's filter constants."""
        self.text = text
        self.native_lowering = native_lowering
        if native_lowering:
            from .native import NativeDictionary
            self.strings = NativeDictionary()
        else:
            self.strings = Dictionary()
        self.keydict = Dictionary()
        self.app, self.compiled, _ = compile_app(text, self.strings)
        self._events: List[tuple] = []  # app event id -> (stream idx, ts, data)
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

    def _now_ms(self):
        return int(time.time() * 1000)

    def _ensure_queries(self):
        if self.queries:
            return
        start = self._start_clock if self._start_clock is not None else (0 if self.app.playback else self._t0)
        for cq in self.compiled:
            if self.native_lowering:
                eng = self._engine_factory(cq.program_json(), start, siddhiql=(self.text, cq.name, self.strings))
                if eng.program_json != cq.program_json():
                    raise AssertionError(f"native lowering of {cq.name} differs from query.compiler")
            else:
                eng = self._engine_factory(cq.program_json(), start)
            self.queries[cq.name] = _QueryRun(self, cq, eng)

    def _enqueue(self, stream: str, ts: int, data: list):
        self._ensure_queries()
        sidx = list(self.app.streams.keys()).index(stream)
        self._events.append((sidx, ts, tuple(data)))
        self._pending.append(len(self._events) - 1)
        if len(self._pending) >= self._batch_size:
            self.flush()

    def advance_time(self, now: int):
        """Advance the event-time clock (playback heartbeat / live scheduler emulation)."""
        self.flush()
        for qr in self.queries.values():
            qr.engine.advance(int(now))
            self._drain(qr)

    # ---------------------------------------------------------------- flush
    def flush(self):
        if not self._pending:
            return
        ids = self._pending
        self._pending = []
        stream_names = list(self.app.streams.keys())
        for qr in self.queries.values():
            if self.app.playback:
                # the playback clock is the app's: a send on any stream sets it before anything
                # else (InputHandler.java:59-64), so a stream this query does not read still
                # fires its timers -- pushed as clock-only events (stream -1)
                sel = list(ids)
            else:
                sel = [i for i in ids if stream_names[self._events[i][0]] in qr.streams]
            if not sel:
                continue
            self._push(qr, sel, stream_names)
            self._drain(qr)

    def _push(self, qr: _QueryRun, sel: List[int], stream_names):
        n = len(sel)
        ts = np.empty(n, np.int64)
        key = np.zeros(n, np.int32)
        stream = np.empty(n, np.int32)
        cols = []
        nulls = []
        for (s, a, t) in qr.cq.columns:
            cols.append(np.zeros(n, _NP[t]))
            nulls.append(np.zeros(n, np.uint8))
        pk = qr.cq.partition_keys
        for j, i in enumerate(sel):
            s, t, data = self._events[i]
            ts[j] = t
            stream[j] = s
            sname = stream_names[s]
            if sname not in qr.streams:  # clock-only (playback): no key, no values (the kernels never
                stream[j] = -1          # read a stream -1 row's values, so its null flags stay 0)
                continue
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
        qr.engine.push(ts, key, stream, cols, null_ptrs)
        qr.local_to_app.extend(sel)

    def _drain(self, qr: _QueryRun):
        mb = qr.engine.fetch()
        m = len(mb["key"])
        if m == 0:
            return
        S = mb["slot_len"].shape[1] if m else 0
        refs = mb["refs"]
        off = 0
        l2a = qr.local_to_app
        for i in range(m):
            slots = []
            for s in range(S):
                ln = int(mb["slot_len"][i, s])
                chain = [l2a[int(x)] if x >= 0 else -1 for x in refs[off:off + ln]]
                off += ln
                slots.append(chain)
            row = qr.selector.select(int(mb["key"][i]), int(mb["ts"][i]), int(mb["type"][i]), slots)
            if row is None:
                continue
            t = int(mb["ts"][i])
            qr.rows.append((t, row))
            for cb in qr.callbacks:
                cb(t, [Event(t, row)], None)


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
