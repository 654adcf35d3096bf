"""Lower a parsed SiddhiQL state query to the NFA program consumed by the engine.

The rules reproduced here are the reference's build-time wiring rules:

* state ids follow ``MetaStateEvent`` insertion order, i.e. the recursive
  parse order of ``StateInputStreamParser.parse``
  (``core/util/parser/StateInputStreamParser.java:148-408``); a logical
  element parses its *second* operand first (``:339-352``);
* variable chain indexes follow ``ExpressionParser.parseVariable``
  (``core/util/parser/ExpressionParser.java:1253-1416``): filters default to
  CURRENT (-1), selectors to 0; an explicit ``[last-k]`` becomes ``-1-k``
  unless the variable refers to the filter's own state, where it stays
  ``-2-k``; an index-less selector reference to a count state is multi-valued;
* compare/arithmetic typing follows Java binary numeric promotion
  (``ExpressionParser.java:1425-1446``).

The output program is plain JSON (``dict``) so it can cross the C-ABI as text
(``shp_engine_create`` in ``include/siddhi_hip.h``).
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from .siddhiql import App, Expr, Query, SiddhiParserException, StateNode, parse_app

NUM_RANK = {"int": 0, "long": 1, "float": 2, "double": 3}
CURRENT = -1
LAST = -2


class SiddhiAppCreationException(ValueError):
    """Mirrors io.siddhi.core.exception.SiddhiAppCreationException."""


@dataclass
class LeafState:
    id: int
    ref: Optional[str]
    stream: str
    absent: bool
    waiting: int
    multi_value: bool
    filters: List[Expr]
    filter_json: Optional[dict] = None


@dataclass
class CompiledQuery:
    name: str
    program: dict
    query: Query
    leaves: List[LeafState]
    stream_index: Dict[str, int]
    columns: List[tuple]  # (stream_idx, attr_idx, type)
    select: List[dict]  # compiled selector items
    select_names: List[str]
    partition_keys: Optional[Dict[str, str]]

    def program_json(self) -> str:
        return json.dumps(self.program, sort_keys=True)


class QueryCompiler:
    def __init__(self, app: App, query: Query, dictionary):
        self.app = app
        self.q = query
        self.dictionary = dictionary  # callable str -> int id
        self.leaves: List[LeafState] = []
        self.stream_names = list(app.streams.keys())
        self.stream_index = {n: i for i, n in enumerate(self.stream_names)}
        self.columns: List[tuple] = []
        self.col_index: Dict[tuple, int] = {}

    # ---------------------------------------------------------------- states
    def _leaf(self, node: StateNode, absent: bool, multi_value: bool) -> LeafState:
        src = node.src
        if src.stream not in self.app.streams:
            raise SiddhiAppCreationException(f"Stream {src.stream} is not defined")
        leaf = LeafState(
            id=len(self.leaves), ref=src.ref, stream=src.stream, absent=absent,
            waiting=node.waiting if node.waiting is not None else -1,
            multi_value=multi_value, filters=src.filters)
        self.leaves.append(leaf)
        return leaf

    def _tree(self, node: StateNode, multi_value=False) -> dict:
        k = node.kind
        if k == "stream":
            return {"t": "stream", "state": self._leaf(node, False, multi_value).id}
        if k == "absent":
            return {"t": "absent", "state": self._leaf(node, True, multi_value).id}
        if k == "next":
            a = self._tree(node.a, multi_value)
            b = self._tree(node.b, multi_value)
            return {"t": "next", "a": a, "b": b}
        if k == "every":
            return {"t": "every", "x": self._tree(node.a, multi_value)}
        if k == "count":
            if node.a.kind != "stream":
                raise SiddhiAppCreationException("count state must wrap a stream state")
            leaf = self._leaf(node.a, False, True)
            mn = 0 if node.min == -1 else node.min
            mx = -1 if node.max == -1 else node.max
            return {"t": "count", "state": leaf.id, "min": mn, "max": mx}
        if k == "logical":
            # element2 parsed before element1 (StateInputStreamParser.java:339-352)
            s2 = self._tree(node.b, multi_value)
            s1 = self._tree(node.a, multi_value)
            return {"t": "logical", "op": node.logical, "s1": s1, "s2": s2}
        raise SiddhiAppCreationException(f"unsupported state element {k}")

    # ----------------------------------------------------------- expressions
    def _attr_type(self, stream: str, attr: str) -> Optional[str]:
        for an, at in self.app.streams[stream].attrs:
            if an == attr:
                return at
        return None

    def _attr_idx(self, stream: str, attr: str) -> int:
        for i, (an, _) in enumerate(self.app.streams[stream].attrs):
            if an == attr:
                return i
        raise SiddhiAppCreationException(f"{attr} not defined in {stream}")

    def _find_state(self, ref: str) -> Optional[LeafState]:
        for lf in self.leaves:
            if lf.ref is not None and lf.ref == ref:
                return lf
        for lf in self.leaves:
            if lf.ref is None and lf.stream == ref:
                return lf
        return None

    def _column(self, stream: str, attr: str) -> int:
        key = (self.stream_index[stream], self._attr_idx(stream, attr))
        if key not in self.col_index:
            self.col_index[key] = len(self.columns)
            self.columns.append((key[0], key[1], self._attr_type(stream, attr)))
        return self.col_index[key]

    def resolve_var(self, e: Expr, current: Optional[LeafState], default_index: int):
        """Return (leaf, chain_index, type, multi_value) per ExpressionParser.parseVariable."""
        if e.stream_ref is None:
            if current is not None:
                t = self._attr_type(current.stream, e.attr)
                if t is None:
                    raise SiddhiAppCreationException(
                        f"{e.attr} not defined in Input Stream: {current.stream}")
                leaf = current
            else:
                found = [lf for lf in self.leaves if self._attr_type(lf.stream, e.attr) is not None]
                if not found:
                    raise SiddhiAppCreationException(f"attribute {e.attr} not found")
                if len(found) > 1:
                    raise SiddhiAppCreationException(
                        f"attribute {e.attr} is ambiguous across input streams")
                leaf = found[0]
                t = self._attr_type(leaf.stream, e.attr)
            index = default_index if e.index is None else (e.index + 1 if e.index <= LAST else e.index)
            return leaf, index, t, False
        leaf = self._find_state(e.stream_ref)
        if leaf is None:
            raise SiddhiAppCreationException(f"Stream with reference : {e.stream_ref} not found")
        t = self._attr_type(leaf.stream, e.attr) if e.attr is not None else None
        if e.attr is not None and t is None:
            raise SiddhiAppCreationException(f"{e.attr} not defined in {leaf.stream}")
        if e.index is None:
            index = default_index
        elif e.index <= LAST:
            index = e.index + 1
            if (current is not None and current.ref is not None and leaf.ref is not None
                    and e.stream_ref == current.ref):
                index = e.index
        else:
            index = e.index
        multi = current is None and e.index is None and leaf.multi_value and leaf.ref is not None
        return leaf, index, t, multi

    def compile_filter_expr(self, e: Expr, current: LeafState) -> dict:
        ex, ty = self._cexpr(e, current)
        if ty != "bool":
            raise SiddhiAppCreationException("filter expression must be of type BOOL")
        return ex

    def _cexpr(self, e: Expr, current: LeafState):
        op = e.op
        if op == "const":
            if e.vtype == "string":
                return {"op": "const", "type": "string", "v": int(self.dictionary(e.value))}, "string"
            if e.vtype == "null":
                return {"op": "const", "type": "null", "v": 0}, "null"
            if e.vtype == "bool":
                return {"op": "const", "type": "bool", "v": 1 if e.value else 0}, "bool"
            return {"op": "const", "type": e.vtype, "v": e.value}, e.vtype
        if op == "var":
            if e.stream_ref is None and self._find_state(e.attr) is not None and \
                    self._attr_type(current.stream, e.attr) is None:
                raise SiddhiAppCreationException("state reference used as a value")
            leaf, index, t, _ = self.resolve_var(e, current, CURRENT)
            col = self._column(leaf.stream, e.attr)
            return {"op": "var", "state": leaf.id, "col": col, "index": index, "type": t}, t
        if op == "stateref":
            raise SiddhiAppCreationException("state reference used as a value")
        if op in ("and", "or"):
            a, ta = self._cexpr(e.args[0], current)
            b, tb = self._cexpr(e.args[1], current)
            if ta != "bool" or tb != "bool":
                raise SiddhiAppCreationException(f"{op} operands must be BOOL")
            return {"op": op, "a": a, "b": b}, "bool"
        if op == "not":
            a, ta = self._cexpr(e.args[0], current)
            if ta != "bool":
                raise SiddhiAppCreationException("not operand must be BOOL")
            return {"op": "not", "a": a}, "bool"
        if op == "isnull":
            inner = e.args[0]
            if inner.op == "stateref" or (inner.op == "var" and inner.stream_ref is None
                                           and self._find_state(inner.attr) is not None
                                           and self._attr_type(current.stream, inner.attr) is None):
                ref = inner.stream_ref if inner.op == "stateref" else inner.attr
                leaf = self._find_state(ref)
                idx = CURRENT if inner.index is None else (
                    inner.index + 1 if inner.index <= LAST else inner.index)
                return {"op": "isnullstate", "state": leaf.id, "index": idx}, "bool"
            a, _ = self._cexpr(inner, current)
            return {"op": "isnull", "a": a}, "bool"
        if op == "cmp":
            a, ta = self._cexpr(e.args[0], current)
            b, tb = self._cexpr(e.args[1], current)
            cmp = e.value
            if ta in NUM_RANK and tb in NUM_RANK:
                pass
            elif ta == tb and ta in ("string", "bool") and cmp in ("eq", "ne"):
                pass
            elif "null" in (ta, tb):
                pass
            else:
                raise SiddhiAppCreationException(f"cannot compare {ta} with {tb} using {cmp}")
            return {"op": "cmp", "cmp": cmp, "a": a, "b": b}, "bool"
        if op in ("add", "sub", "mul", "div", "mod"):
            a, ta = self._cexpr(e.args[0], current)
            b, tb = self._cexpr(e.args[1], current)
            if ta not in NUM_RANK or tb not in NUM_RANK:
                raise SiddhiAppCreationException(f"arithmetic on {ta}/{tb}")
            rt = ta if NUM_RANK[ta] >= NUM_RANK[tb] else tb
            return {"op": op, "type": rt, "a": a, "b": b}, rt
        if op == "func":
            return self._cfunc(e, current)
        raise SiddhiAppCreationException(f"unsupported expression {op} in a state filter")

    INSTANCE_OF = {"instanceofboolean": "bool", "instanceofdouble": "double", "instanceoffloat": "float",
                   "instanceofinteger": "int", "instanceoflong": "long", "instanceofstring": "string"}

    def _cfunc(self, e: Expr, current: LeafState):
        """Scalar functions in filters (core/executor/function/*; FunctionExecutor.execute evaluates
        every argument before the function body), with the reference's validation rules."""
        name = e.value
        args = [self._cexpr(a, current) for a in e.args]
        if name == "ifthenelse":  # IfThenElseFunctionExecutor.java
            if len(args) != 3:
                raise SiddhiAppCreationException(
                    f"Invalid no of arguments passed to ifThenElse() function, required only 3, but found {len(args)}")
            if args[0][1] != "bool":
                raise SiddhiAppCreationException("Input type of if in ifThenElse function should be of type BOOL")
            if args[1][1] != args[2][1]:
                raise SiddhiAppCreationException("Input type of then in ifThenElse function and else in "
                                                 "ifThenElse function should be of equivalent type")
            t = args[1][1]
            return {"op": "ifthenelse", "type": t, "args": [a for a, _ in args]}, t
        if name == "coalesce":  # CoalesceFunctionExecutor.java
            if not args:
                raise SiddhiAppCreationException("Coalesce must have at least one parameter")
            t = args[0][1]
            if any(ta != t for _, ta in args):
                raise SiddhiAppCreationException("Coalesce cannot have parameters with different type")
            return {"op": "coalesce", "type": t, "args": [a for a, _ in args]}, t
        if name in self.INSTANCE_OF:  # InstanceOf*FunctionExecutor.java: data instanceof <Type>
            if len(args) != 1:
                raise SiddhiAppCreationException(f"Invalid no of arguments passed to {name}")
            return {"op": "instanceof", "tag": self.INSTANCE_OF[name], "a": args[0][0]}, "bool"
        raise SiddhiAppCreationException(f"function {name} is not supported in a state filter")

    # --------------------------------------------------------------- select
    def compile_select(self):
        items = []
        names = []
        q = self.q
        if q.select_all:
            raise SiddhiAppCreationException("select * is not supported on the state path")
        for it in q.select:
            items.append(self._csel(it.expr))
            names.append(it.name)
        return items, names

    def _csel(self, e: Expr) -> dict:
        if e.op == "const":
            return {"op": "const", "type": e.vtype, "v": e.value}
        if e.op == "var":
            leaf, index, t, multi = self.resolve_var(e, None, 0)
            return {"op": "var", "state": leaf.id, "attr": self._attr_idx(leaf.stream, e.attr),
                    "index": index, "type": t, "multi": multi}
        if e.op == "func":
            name = e.value
            args = [self._csel(a) for a in e.args]
            return {"op": "func", "name": name, "args": args}
        if e.op in ("add", "sub", "mul", "div", "mod", "cmp", "and", "or", "not", "isnull"):
            return {"op": e.op, "cmp": e.value if e.op == "cmp" else None,
                    "args": [self._csel(a) for a in e.args]}
        raise SiddhiAppCreationException(f"unsupported select expression {e.op}")

    # --------------------------------------------------------------- driver
    def compile(self) -> CompiledQuery:
        q = self.q
        tree = self._tree(q.root)
        # filters are parsed per leaf, with the states known so far (parse order)
        for leaf in self.leaves:
            if leaf.filters:
                ex = None
                for f in leaf.filters:
                    fe = self.compile_filter_expr(f, leaf)
                    ex = fe if ex is None else {"op": "and", "a": ex, "b": fe}
                leaf.filter_json = ex
        sel, names = self.compile_select()
        states = []
        for lf in self.leaves:
            states.append({
                "id": lf.id, "ref": lf.ref, "stream": self.stream_index[lf.stream],
                "absent": lf.absent, "waiting": lf.waiting, "filter": lf.filter_json,
            })
        partitioned = q.partition is not None
        if partitioned:
            for lf in self.leaves:
                if lf.stream not in q.partition:
                    raise SiddhiAppCreationException(
                        f"stream {lf.stream} used in a partition without a partition key")
        program = {
            "version": 1,
            "name": q.name,
            "type": q.seq_type,
            "within": q.within if q.within is not None else -1,
            "playback": bool(self.app.playback),
            "partitioned": partitioned,
            "streams": [{"name": n, "attrs": [list(a) for a in self.app.streams[n].attrs]}
                        for n in self.stream_names],
            "columns": [{"stream": s, "attr": a, "type": t} for (s, a, t) in self.columns],
            "states": states,
            "tree": tree,
        }
        agg = self._device_aggregate(sel)
        if agg is not None:
            program["aggregate"] = agg
        return CompiledQuery(q.name, program, q, self.leaves, self.stream_index, self.columns,
                             sel, names, q.partition)

    def _device_aggregate(self, sel):
        """The select's aggregate, when the engine can run it (SHP_LAYOUT_AGG): exactly one
        avg/sum/count/min/max whose argument is a filter column of one state; the other items
        must not aggregate.  Mirrors the selector's aggregator (QuerySelector.java:271-313)."""
        funcs = [it for it in sel if it["op"] == "func"]
        if len(funcs) != 1 or funcs[0]["name"] not in ("avg", "sum", "count", "min", "max"):
            return None
        f = funcs[0]
        if f["name"] == "count":
            return {"fn": "count"} if not f["args"] else None
        if len(f["args"]) != 1 or f["args"][0]["op"] != "var" or f["args"][0].get("multi"):
            return None
        a = f["args"][0]
        leaf = self.leaves[a["state"]]
        key = (self.stream_index[leaf.stream], a["attr"])
        for ci, (s, at, _t) in enumerate(self.columns):
            if (s, at) == key:
                return {"fn": f["name"], "state": a["state"], "column": ci}
        return None


class Dictionary:
    """String dictionary shared by key columns and string constants (host-owned strings)."""

    def __init__(self):
        self.ids: Dict[str, int] = {}
        self.strings: List[str] = []

    def __call__(self, s: str) -> int:
        i = self.ids.get(s)
        if i is None:
            i = len(self.strings)
            self.ids[s] = i
            self.strings.append(s)
        return i


def compile_app(text: str, dictionary: Optional[Dictionary] = None):
    app = parse_app(text)
    dictionary = dictionary or Dictionary()
    out = []
    for q in app.queries:
        out.append(QueryCompiler(app, q, dictionary).compile())
    return app, out, dictionary
