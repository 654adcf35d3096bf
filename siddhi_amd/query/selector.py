"""Host-side selection of matched state events (the L5 boundary of SURVEY.md §1).

The engine returns match records: partition key, match timestamp, event type and,
per state slot, the chain of matched event sequence numbers snapshotted at
emission time.  This module rebuilds the selector output the reference's
``QuerySelector.processInBatchNoGroupBy`` (``core/query/selector/QuerySelector.java:271-313``)
would produce from those slots, following ``StateEvent.getStreamEvent(int[])``
(``core/event/state/StateEvent.java:138-189``) for chain indexes and
``AvgAttributeAggregatorExecutor`` (``core/query/selector/attribute/aggregator/
AvgAttributeAggregatorExecutor.java:143-260``) for avg (double sum / long count).
"""
from __future__ import annotations

import math
from typing import Any, Dict, List, Optional

import numpy as np

from ..flow import get_partition_flow_id

NUM_RANK = {"int": 0, "long": 1, "float": 2, "double": 3}


def f32(x) -> float:
    return float(np.float32(x))


def pick_chain(chain: List[int], index: int) -> Optional[int]:
    if not chain:
        return None
    n = len(chain)
    if index >= 0:
        return chain[index] if index < n else None
    if index == -1:
        return chain[-1]
    if index == -2:
        return chain[-2] if n >= 2 else None
    i = n + index
    return chain[i] if i >= 0 else None


def _jtype(v):
    if isinstance(v, bool):
        return "bool"
    if isinstance(v, str):
        return "string"
    return None


class Aggregator:
    def __init__(self, name: str, arg_type: Optional[str]):
        self.name = name
        self.arg_type = arg_type
        self.value = 0.0 if name in ("avg",) else 0
        self.count = 0
        self.items: List[Any] = []

    def add(self, x, remove=False):
        n = self.name
        if n == "count":
            self.count += -1 if remove else 1
            return self.count
        if x is None:
            return self.current()
        if n == "avg":
            if remove:
                self.count -= 1
                self.value -= float(x)
            else:
                self.count += 1
                self.value += float(x)
            return None if self.count == 0 else self.value / self.count
        if n == "sum":
            if self.arg_type in ("float", "double"):
                self.value = float(self.value) + (-float(x) if remove else float(x))
            else:
                self.value = int(self.value) + (-int(x) if remove else int(x))
            return self.value
        if n in ("max", "min"):
            if remove:  # sliding windows only (the deque of Min/MaxAttributeAggregatorExecutor)
                if x in self.items:
                    self.items.remove(x)
                if not self.items:
                    self.mm = None
                else:
                    self.mm = max(self.items) if n == "max" else min(self.items)
                return self.mm
            self.items.append(x)
            # MinAttributeAggregatorExecutor.processAdd: `if (minValue == null || minValue > value)`
            # (max: `<`): a NaN first value stays, a later NaN never replaces
            m = getattr(self, "mm", None)
            if m is None or (m > x if n == "min" else m < x):
                self.mm = x
            return self.mm
        raise ValueError(f"unsupported aggregate {n}")

    def current(self):
        if self.name == "avg":
            return None if self.count == 0 else self.value / self.count
        if self.name == "count":
            return self.count
        if self.name == "sum":
            return self.value
        return getattr(self, "mm", None)


class Selector:
    """Evaluates compiled select items for one query over match records."""

    def __init__(self, compiled, event_store, strings):
        self.cq = compiled
        self.events = event_store  # seq -> (stream_idx, ts, data tuple)
        self.strings = strings
        self.partitioned = compiled.partition_keys is not None
        self.aggs: Dict[Any, List[Aggregator]] = {}

    def _aggs_for(self):
        """The aggregators of the current partition flow (PartitionStateHolder.getState,
        core/util/snapshot/state/PartitionStateHolder.java:43-48): the host delivers each match
        inside its key's flow (siddhi_amd.flow), the selector is never handed a key."""
        k = get_partition_flow_id() if self.partitioned else 0
        if k not in self.aggs:
            lst = []
            self._collect_aggs(self.cq.select, lst)
            self.aggs[k] = lst
        return self.aggs[k]

    def _collect_aggs(self, items, lst):
        for it in items:
            if it["op"] == "func":
                lst.append(Aggregator(it["name"], it["args"][0].get("type") if it["args"] else None))
            elif it["op"] not in ("var", "const"):
                self._collect_aggs(it["args"], lst)

    def _val(self, seq, attr_idx, ty):
        if seq is None or seq < 0:
            return None
        stream, ts, data = self.events[seq]
        v = data[attr_idx]
        if v is None:
            return None
        if ty == "float":
            return f32(v)
        if ty == "double":
            return float(v)
        if ty in ("int", "long"):
            return int(v)
        return v

    def _eval(self, it, slots, aggs, agg_i, remove):
        op = it["op"]
        if op == "const":
            v = it["v"]
            return f32(v) if it["type"] == "float" else v
        if op == "var":
            chain = slots[it["state"]]
            if it.get("multi"):
                if not chain:
                    return None
                return [self._val(s, it["attr"], it["type"]) for s in chain]
            return self._val(pick_chain(chain, it["index"]), it["attr"], it["type"])
        if op == "func":
            arg = self._eval(it["args"][0], slots, aggs, agg_i, remove) if it["args"] else None
            a = aggs[agg_i[0]]
            agg_i[0] += 1
            return a.add(arg, remove)
        args = [self._eval(a, slots, aggs, agg_i, remove) for a in it["args"]]
        if op in ("add", "sub", "mul", "div", "mod"):
            x, y = args
            if x is None or y is None:
                return None
            if isinstance(x, float) or isinstance(y, float):
                if op == "div":
                    return None if y == 0 else x / y
                if op == "mod":
                    return None if y == 0 else math.fmod(x, y)
            return {"add": lambda: x + y, "sub": lambda: x - y, "mul": lambda: x * y,
                    "div": lambda: None if y == 0 else int(x / y),
                    "mod": lambda: None if y == 0 else int(math.fmod(x, y))}[op]()
        if op == "cmp":
            x, y = args
            if x is None or y is None:
                return False
            return {"gt": x > y, "ge": x >= y, "lt": x < y, "le": x <= y,
                    "eq": x == y, "ne": x != y}[it["cmp"]]
        if op == "and":
            return bool(args[0]) and bool(args[1])
        if op == "or":
            return bool(args[0]) or bool(args[1])
        if op == "not":
            return not (args[0] is True)
        if op == "isnull":
            return args[0] is None
        raise ValueError(op)

    def select(self, ts, etype, slots):
        """Return the output row, or None when the event is not emitted (expired)."""
        aggs = self._aggs_for()
        agg_i = [0]
        remove = etype == 1
        row = [self._eval(it, slots, aggs, agg_i, remove) for it in self.cq.select]
        if etype != 0:
            return None
        return row
