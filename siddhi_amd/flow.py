"""The partition flow and the app clock of the host mirror -- the two pieces of the reference's
``SiddhiAppContext`` / ``TimestampGeneratorImpl`` the state path's egress and timers depend on.

* Partition flow (``core/config/SiddhiAppContext.java:56,97-111``): a thread-local partition key.
  ``PartitionStreamReceiver.send`` (``core/partition/PartitionStreamReceiver.java:262-272``) and the
  Scheduler's timer loop (``core/util/Scheduler.java:88-97``) set it around everything they run, and
  every per-key state -- the selector's aggregators included -- is looked up under it
  (``PartitionStateHolder.getState``, ``core/util/snapshot/state/PartitionStateHolder.java:43-48``).
  The host's match delivery therefore runs each match inside its key's flow
  (``runtime.SiddhiAppRuntime._deliver``, ``GpuStateStreamRuntime.java`` ``inFlow``); the selector
  reads the flow, it is never handed a key.
* App clock (``core/util/timestamp/TimestampGeneratorImpl.java:77-185``): in playback,
  ``InputHandler.send`` sets it from the event (``core/stream/input/InputHandler.java:59-92``, before
  the event enters any junction) and the idle heartbeat moves it by ``increment`` when no event came
  for ``idle.time``; every change is announced to the registered ``TimeChangeListener``s, which is how
  the Scheduler of an absent state learns the time (``Scheduler.java:71-103``).
"""
from __future__ import annotations

import threading
from typing import Callable, List, Optional

_flow = threading.local()


def start_partition_flow(key: Optional[str]) -> None:
    """SiddhiAppContext.startPartitionFlow (:97-99)."""
    _flow.key = key


def stop_partition_flow() -> None:
    """SiddhiAppContext.stopPartitionFlow (:101-103)."""
    _flow.key = None


def get_partition_flow_id() -> Optional[str]:
    """SiddhiAppContext.getPartitionFlowId (:109-111)."""
    return getattr(_flow, "key", None)


class in_partition_flow:
    """Runs a block inside key's flow and restores the caller's flow after it: a match delivered
    during a PartitionStreamReceiver.send of another key (a batched push, a timer of key A fired by
    key B's event) must not leave the sender's flow changed."""

    __slots__ = ("key", "prev")

    def __init__(self, key: Optional[str]):
        self.key = key

    def __enter__(self):
        self.prev = get_partition_flow_id()
        start_partition_flow(self.key)
        return self

    def __exit__(self, *exc):
        start_partition_flow(self.prev)
        return False


class TimestampGenerator:
    """TimestampGeneratorImpl (core/util/timestamp/TimestampGeneratorImpl.java): the app clock.

    playback: currentTime() is the last event's timestamp; set_current_timestamp only moves it
    forward (:105-122) and notifies every listener.  idle_time / increment
    (``@app:playback(idle.time, increment)``): the heartbeat (TimeInjector, :168-185) adds
    ``increment`` whenever no event arrived for ``idle_time`` wall-clock ms -- driven here by
    ``heartbeat(wall_ms)`` so tests can step it deterministically."""

    def __init__(self, playback: bool, idle_time: int = -1, increment: int = 0, wall: Callable[[], int] = None):
        import time
        self.playback = playback
        self.idle_time = idle_time
        self.increment = increment
        self.last_event_ts = 0
        self._wall = wall or (lambda: int(time.time() * 1000))
        self.last_system_ts = self._wall()
        self.listeners: List[Callable[[int], None]] = []

    def current_time(self) -> int:
        return self.last_event_ts if self.playback else self._wall()

    def add_time_change_listener(self, fn: Callable[[int], None]) -> None:
        self.listeners.append(fn)

    def set_current_timestamp(self, ts: int, wall_ms: Optional[int] = None) -> None:
        if ts >= self.last_event_ts:
            self.last_event_ts = ts
            for fn in self.listeners:
                fn(ts)
            self.last_system_ts = self._wall() if wall_ms is None else wall_ms

    def heartbeat(self, wall_ms: int) -> bool:
        """TimeInjector.run at wall-clock time wall_ms: when no event came for idle_time, the clock
        moves by increment (and the listeners hear it).  Returns whether it moved."""
        if not self.playback or self.idle_time < 0:
            return False
        if wall_ms - self.last_system_ts >= self.idle_time:
            self.set_current_timestamp(self.last_event_ts + self.increment, wall_ms)
            return True
        return False
