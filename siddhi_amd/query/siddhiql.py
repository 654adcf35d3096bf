"""SiddhiQL subset parser for the pattern/sequence path.

Host-side mirror of what the Java host already holds: the reference parses
SiddhiQL with ANTLR (``SiddhiQL.g4:200-345`` pattern/sequence rules,
``SiddhiQLBaseVisitorImpl.java:760-1120`` tree building) into a
``StateInputStream`` (``api/execution/query/input/stream/StateInputStream.java``).
This module parses the same text for the subset the state path needs:

* ``define stream``; ``@app:playback``; ``@info(name=...)``
* ``partition with (attr of Stream, ...) begin ... end;``
* ``from <pattern | sequence> [within T] select ... insert into Out;``

and produces a small AST that :mod:`siddhi_amd.query.compiler` lowers to the
NFA program JSON consumed by ``libsiddhi_hip.so`` (and by the test oracle).

Tree shapes follow the visitor: ``a -> b -> c`` is left-associative
``Next(Next(a, b), c)``; ``every x`` wraps the following pattern_source only;
``A and not B`` becomes ``Logical(absent B, AND, A)`` (``State.logicalNotAnd``,
``api/execution/query/input/state/State.java:52-69``); ``A or not B for t``
becomes ``Logical(absent B, OR, A)`` (visitor ``:1005-1013``).
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import Any, List, Optional

# --------------------------------------------------------------------------
# tokens
# --------------------------------------------------------------------------

_TOKEN_RE = re.compile(
    r"""
    (?P<ws>\s+|--[^\n]*|/\*.*?\*/)
  | (?P<str>'[^']*'|"[^"]*")
  | (?P<num>(?:\d+\.\d*|\.\d+|\d+)(?:[eE][-+]?\d+)?[lLfFdD]?)
  | (?P<id>[A-Za-z_][A-Za-z0-9_]*)
  | (?P<op>->|==|!=|>=|<=|[-+*/%<>=(),;\[\]:.@#!?])
    """,
    re.VERBOSE | re.DOTALL,
)

KEYWORDS = {
    "define", "stream", "from", "select", "insert", "into", "every", "within",
    "and", "or", "not", "for", "partition", "with", "of", "begin", "end", "as",
    "is", "null", "true", "false", "last", "group", "by", "having", "current",
    "expired", "all", "events", "output", "return",
}

TIME_UNITS = {
    "millisecond": 1, "milliseconds": 1, "millisec": 1, "millis": 1, "ms": 1,
    "sec": 1000, "second": 1000, "seconds": 1000, "secs": 1000,
    "min": 60000, "minute": 60000, "minutes": 60000, "mins": 60000,
    "hour": 3600000, "hours": 3600000,
    "day": 86400000, "days": 86400000,
    "week": 604800000, "weeks": 604800000,
    "month": 2630000000, "months": 2630000000,
    "year": 31556900000, "years": 31556900000,
}


class SiddhiParserException(ValueError):
    """Raised for text outside the supported subset (mirrors SiddhiParserException)."""


@dataclass
class Tok:
    kind: str
    text: str
    pos: int


def tokenize(text: str) -> List[Tok]:
    out: List[Tok] = []
    pos = 0
    while pos < len(text):
        m = _TOKEN_RE.match(text, pos)
        if not m:
            raise SiddhiParserException(f"unexpected character {text[pos]!r} at {pos}")
        kind = m.lastgroup
        if kind != "ws":
            out.append(Tok(kind, m.group(kind), pos))
        pos = m.end()
    out.append(Tok("eof", "", pos))
    return out


# --------------------------------------------------------------------------
# AST
# --------------------------------------------------------------------------

@dataclass
class StreamDef:
    name: str
    attrs: List[tuple]  # (name, type)


@dataclass
class Expr:
    op: str
    args: List[Any] = field(default_factory=list)
    value: Any = None
    vtype: Optional[str] = None
    # variables
    stream_ref: Optional[str] = None
    attr: Optional[str] = None
    index: Optional[int] = None  # explicit chain index (LAST=-2, last-k=-2-k)


@dataclass
class BasicSource:
    ref: Optional[str]
    stream: str
    filters: List[Expr]


@dataclass
class StateNode:
    kind: str  # stream | absent | next | every | count | logical
    src: Optional[BasicSource] = None
    waiting: Optional[int] = None  # absent: ms or None (no 'for')
    a: Optional["StateNode"] = None
    b: Optional["StateNode"] = None
    min: int = -1
    max: int = -1
    logical: Optional[str] = None


@dataclass
class SelectItem:
    expr: Expr
    name: str


@dataclass
class Query:
    name: str
    seq_type: str  # pattern | sequence
    root: StateNode
    within: Optional[int]
    select: List[SelectItem]
    select_all: bool
    out_stream: str
    partition: Optional[dict]  # stream -> key attr
    output_events: str = "current"


@dataclass
class App:
    streams: dict
    queries: List[Query]
    playback: bool
    idle_time: int = -1   # @app:playback(idle.time = '...'): the heartbeat's idle time (ms), -1 = none
    increment: int = 0    # @app:playback(increment = '...'): the heartbeat's clock step (ms)


def playback_time(text: str) -> int:
    """'10 milliseconds' / '1 sec' of an @app:playback property, in ms (SiddhiAppParser reads them with
    the time grammar: core/util/parser/SiddhiAppParser.java)."""
    parts = text.split()
    total, i = 0, 0
    while i + 1 < len(parts):
        unit = parts[i + 1].lower()
        if unit not in TIME_UNITS:
            raise SiddhiParserException(f"bad time {text!r}")
        total += int(float(parts[i]) * TIME_UNITS[unit])
        i += 2
    if i != len(parts):
        raise SiddhiParserException(f"bad time {text!r}")
    return total


# --------------------------------------------------------------------------
# parser
# --------------------------------------------------------------------------

class Parser:
    def __init__(self, text: str):
        self.toks = tokenize(text)
        self.i = 0

    # -- helpers
    def peek(self, k=0) -> Tok:
        return self.toks[min(self.i + k, len(self.toks) - 1)]

    def at(self, text, k=0) -> bool:
        t = self.peek(k)
        if t.kind == "id":
            return t.text.lower() == text
        return t.text == text

    def eat(self, text=None) -> Tok:
        t = self.peek()
        if text is not None and not self.at(text):
            raise SiddhiParserException(f"expected {text!r} at {t.pos}, found {t.text!r}")
        self.i += 1
        return t

    def accept(self, text) -> bool:
        if self.at(text):
            self.i += 1
            return True
        return False

    def ident(self) -> str:
        t = self.peek()
        if t.kind != "id":
            raise SiddhiParserException(f"expected identifier at {t.pos}, found {t.text!r}")
        self.i += 1
        return t.text

    # -- top level
    def parse_app(self) -> App:
        streams = {}
        queries: List[Query] = []
        playback = False
        idle_time, increment = -1, 0
        pending_info = None
        while self.peek().kind != "eof":
            if self.at("@"):
                name, props = self.annotation()
                lname = name.lower()
                if lname in ("app:playback",):
                    playback = True
                    if props.get("idle.time") is not None:
                        idle_time = playback_time(props["idle.time"])
                        increment = playback_time(props.get("increment") or "0 ms")
                elif lname == "info":
                    pending_info = props.get("name")
                continue
            if self.at(";"):
                self.eat()
                continue
            if self.at("define"):
                sd = self.define_stream()
                streams[sd.name] = sd
                continue
            if self.at("partition"):
                queries.extend(self.partition(streams, len(queries)))
                pending_info = None
                continue
            if self.at("from"):
                q = self.query(pending_info or f"query{len(queries) + 1}", None)
                queries.append(q)
                pending_info = None
                continue
            raise SiddhiParserException(f"unsupported construct at {self.peek().pos}: {self.peek().text!r}")
        return App(streams, queries, playback, idle_time, increment)

    def annotation(self):
        self.eat("@")
        name = self.ident()
        while self.at(":") or self.at("."):
            self.eat()
            name += ":" + self.ident()
        props = {}
        if self.accept("("):
            while not self.at(")"):
                if self.peek().kind == "str":
                    props.setdefault("_", self.eat().text[1:-1])
                else:
                    key = self.ident()
                    while self.at("."):
                        self.eat()
                        key += "." + self.ident()
                    self.eat("=")
                    props[key] = self.eat().text.strip("'\"")
                self.accept(",")
            self.eat(")")
        return name, props

    def define_stream(self) -> StreamDef:
        self.eat("define")
        self.eat("stream")
        name = self.ident()
        self.eat("(")
        attrs = []
        while True:
            an = self.ident()
            at = self.ident().lower()
            if at not in ("int", "long", "float", "double", "bool", "string", "object"):
                raise SiddhiParserException(f"unknown type {at}")
            attrs.append((an, at))
            if not self.accept(","):
                break
        self.eat(")")
        return StreamDef(name, attrs)

    def partition(self, streams, nq):
        self.eat("partition")
        self.eat("with")
        self.eat("(")
        keys = {}
        while True:
            attr = self.ident()
            self.eat("of")
            stream = self.ident()
            keys[stream] = attr
            if not self.accept(","):
                break
        self.eat(")")
        self.eat("begin")
        out = []
        pending_info = None
        while not self.at("end"):
            if self.at("@"):
                name, props = self.annotation()
                if name.lower() == "info":
                    pending_info = props.get("name")
                continue
            if self.accept(";"):
                continue
            out.append(self.query(pending_info or f"query{nq + len(out) + 1}", keys))
            pending_info = None
        self.eat("end")
        return out

    def query(self, name, partition) -> Query:
        self.eat("from")
        root, seq_type = self.state_input()
        within = None
        if self.accept("within"):
            within = self.time_value()
        self.eat("select")
        select_all = False
        items: List[SelectItem] = []
        if self.accept("*"):
            select_all = True
        else:
            while True:
                e = self.expr()
                if self.accept("as"):
                    nm = self.ident()
                else:
                    nm = e.attr if e.op == "var" else f"_c{len(items)}"
                items.append(SelectItem(e, nm))
                if not self.accept(","):
                    break
        if self.at("group") or self.at("having") or self.at("output"):
            raise SiddhiParserException("group by / having / output rate limiting are outside the state path")
        output_events = "current"
        if self.accept("insert"):
            if self.accept("all"):
                self.eat("events")
                output_events = "all"
            elif self.accept("expired"):
                self.eat("events")
                output_events = "expired"
            elif self.accept("current"):
                self.eat("events")
            self.eat("into")
            out = self.ident()
        elif self.accept("return"):
            out = "__return__"
        else:
            raise SiddhiParserException("expected insert into")
        self.accept(";")
        return Query(name, seq_type, root, within, items, select_all, out, partition, output_events)

    def time_value(self) -> int:
        total = 0
        got = False
        while self.peek().kind == "num":
            num = self.eat().text
            unit = self.ident().lower()
            if unit not in TIME_UNITS:
                raise SiddhiParserException(f"unknown time unit {unit}")
            total += int(float(num.rstrip("lLfFdD")) * TIME_UNITS[unit])
            got = True
        if not got:
            raise SiddhiParserException("expected time value")
        return total

    # -- state input: decide pattern vs sequence by scanning for top-level ',' vs '->'
    def state_input(self):
        depth = 0
        j = self.i
        saw_comma = saw_arrow = False
        while True:
            t = self.toks[j]
            if t.kind == "eof":
                break
            if t.text in ("(", "["):
                depth += 1
            elif t.text in (")", "]"):
                depth -= 1
            elif depth == 0 and t.kind == "id" and t.text.lower() in ("select", "within"):
                break
            elif t.text == "->":
                saw_arrow = True
            elif t.text == "," and depth == 0:
                saw_comma = True
            j += 1
        if saw_comma and saw_arrow:
            raise SiddhiParserException("cannot mix '->' and ',' in one query")
        if saw_comma:
            return self.sequence_chain(), "sequence"
        return self.pattern_chain(), "pattern"

    # pattern:  chain := item ('->' item)*   (left assoc Next)
    def pattern_chain(self) -> StateNode:
        node = self.pattern_item()
        while self.accept("->"):
            node = StateNode("next", a=node, b=self.pattern_item())
        return node

    def pattern_item(self) -> StateNode:
        if self.at("every"):
            self.eat()
            if self.at("("):
                self.eat("(")
                inner = self.pattern_chain()
                self.eat(")")
                return StateNode("every", a=inner)
            return StateNode("every", a=self.pattern_source(allow_count_seq=False))
        if self.at("(") and not self._paren_is_logical_group():
            self.eat("(")
            inner = self.pattern_chain()
            self.eat(")")
            return inner
        return self.pattern_source(allow_count_seq=False)

    def _paren_is_logical_group(self):
        return False

    # sequence: [every] source (',' source)*  -> Next(first, chain(rest)) with left-assoc rest
    def sequence_chain(self) -> StateNode:
        first = self.sequence_item(top=True)
        rest = []
        while self.accept(","):
            rest.append(self.sequence_item(top=False))
        if not rest:
            return first
        chain = rest[0]
        for r in rest[1:]:
            chain = StateNode("next", a=chain, b=r)
        return StateNode("next", a=first, b=chain)

    def sequence_item(self, top) -> StateNode:
        if self.at("every"):
            if not top:
                raise SiddhiParserException("'every' only allowed at the start of a sequence")
            self.eat()
            if self.at("(") and not self._is_logical_paren():
                self.eat("(")
                inner = self.sequence_chain()
                self.eat(")")
                return StateNode("every", a=inner)
            return StateNode("every", a=self.pattern_source(allow_count_seq=True))
        if self.at("(") and not self._is_logical_paren():
            self.eat("(")
            inner = self.sequence_chain()
            self.eat(")")
            return inner
        return self.pattern_source(allow_count_seq=True)

    def _is_logical_paren(self):
        return False

    def pattern_source(self, allow_count_seq) -> StateNode:
        # logical / absent / count / plain stream
        if self.at("("):
            # parenthesised logical absent source
            self.eat("(")
            n = self.pattern_source(allow_count_seq)
            self.eat(")")
            return n
        left = self.stateful_or_absent()
        if self.at("and") or self.at("or"):
            op = self.eat().text.lower()
            right = self.stateful_or_absent()
            return self._make_logical(op, left, right)
        if left.kind == "absent":
            if left.waiting is None:
                raise SiddhiParserException("'not' without 'for' is only valid inside 'and'")
            return left
        # count
        if self.at("<"):
            self.eat("<")
            mn, mx = self.collect()
            self.eat(">")
            return StateNode("count", a=left, min=mn, max=mx)
        if allow_count_seq:
            if self.accept("*"):
                return StateNode("count", a=left, min=0, max=-1)
            if self.accept("+"):
                return StateNode("count", a=left, min=1, max=-1)
            if self.accept("?"):
                return StateNode("count", a=left, min=0, max=1)
        return left

    def collect(self):
        if self.at(":"):
            self.eat()
            return -1, int(self.eat().text)
        a = int(self.eat().text)
        if self.accept(":"):
            if self.peek().kind == "num":
                return a, int(self.eat().text)
            return a, -1
        return a, a

    def _make_logical(self, op, left, right) -> StateNode:
        la, ra = left.kind == "absent", right.kind == "absent"
        if op == "and":
            if la and ra:
                return StateNode("logical", a=left, b=right, logical="and")
            if la:  # not A [for t] and B
                return StateNode("logical", a=left, b=right, logical="and")
            if ra:  # A and not B [for t]
                return StateNode("logical", a=right, b=left, logical="and")
            return StateNode("logical", a=left, b=right, logical="and")
        # or
        for n in (left, right):
            if n.kind == "absent" and n.waiting is None:
                raise SiddhiParserException("'not' in 'or' requires 'for'")
        if la and ra:
            return StateNode("logical", a=left, b=right, logical="or")
        if la:
            return StateNode("logical", a=left, b=right, logical="or")
        if ra:  # A or not B for t -> logicalOr(absent B, A)
            return StateNode("logical", a=right, b=left, logical="or")
        return StateNode("logical", a=left, b=right, logical="or")

    def stateful_or_absent(self) -> StateNode:
        if self.accept("not"):
            src = self.basic_source(ref=None)
            waiting = None
            if self.accept("for"):
                waiting = self.time_value()
            return StateNode("absent", src=src, waiting=waiting)
        ref = None
        if self.peek().kind == "id" and self.at("=", 1):
            ref = self.ident()
            self.eat("=")
        return StateNode("stream", src=self.basic_source(ref))

    def basic_source(self, ref) -> BasicSource:
        self.accept("#")
        stream = self.ident()
        filters = []
        while self.at("["):
            self.eat("[")
            filters.append(self.expr())
            self.eat("]")
        if self.at("#"):
            raise SiddhiParserException("stream functions/windows inside states are outside the state path")
        return BasicSource(ref, stream, filters)

    # -- expressions (precedence: or < and < not < compare < +- < */% < unary)
    def expr(self) -> Expr:
        e = self.and_expr()
        while self.accept("or"):
            e = Expr("or", [e, self.and_expr()])
        return e

    def and_expr(self) -> Expr:
        e = self.not_expr()
        while self.accept("and"):
            e = Expr("and", [e, self.not_expr()])
        return e

    def not_expr(self) -> Expr:
        if self.accept("not"):
            return Expr("not", [self.not_expr()])
        return self.cmp_expr()

    def cmp_expr(self) -> Expr:
        e = self.add_expr()
        ops = {">": "gt", "<": "lt", ">=": "ge", "<=": "le", "==": "eq", "!=": "ne"}
        t = self.peek()
        if t.kind == "op" and t.text in ops:
            self.eat()
            return Expr("cmp", [e, self.add_expr()], value=ops[t.text])
        if self.at("is"):
            self.eat()
            self.eat("null")
            return Expr("isnull", [e])
        return e

    def add_expr(self) -> Expr:
        e = self.mul_expr()
        while self.at("+") or self.at("-"):
            op = "add" if self.eat().text == "+" else "sub"
            e = Expr(op, [e, self.mul_expr()])
        return e

    def mul_expr(self) -> Expr:
        e = self.unary()
        while self.at("*") or self.at("/") or self.at("%"):
            op = {"*": "mul", "/": "div", "%": "mod"}[self.eat().text]
            e = Expr(op, [e, self.unary()])
        return e

    def unary(self) -> Expr:
        if self.at("-") and self.peek(1).kind == "num":
            self.eat()
            return self._number(negate=True)
        if self.accept("("):
            e = self.expr()
            self.eat(")")
            return e
        t = self.peek()
        if t.kind == "num":
            return self._number()
        if t.kind == "str":
            self.eat()
            return Expr("const", value=t.text[1:-1], vtype="string")
        if self.at("true") or self.at("false"):
            self.eat()
            return Expr("const", value=t.text.lower() == "true", vtype="bool")
        if self.at("null"):
            self.eat()
            return Expr("const", value=None, vtype="null")
        if t.kind == "id":
            name = self.ident()
            if self.at("(") and not self.at("["):
                # function call (aggregates in select)
                self.eat("(")
                args = []
                if not self.at(")"):
                    while True:
                        args.append(self.expr())
                        if not self.accept(","):
                            break
                self.eat(")")
                return Expr("func", args, value=name.lower())
            index = None
            if self.at("["):
                self.eat("[")
                index = self.attribute_index()
                self.eat("]")
            if self.accept("."):
                attr = self.ident()
                return Expr("var", stream_ref=name, attr=attr, index=index)
            if index is not None:
                # e1[0] alone (null check on a state): treat as stream ref
                return Expr("stateref", stream_ref=name, index=index)
            return Expr("var", attr=name)
        raise SiddhiParserException(f"unexpected token {t.text!r} at {t.pos}")

    def attribute_index(self) -> int:
        if self.accept("last"):
            idx = -2  # SiddhiConstants.LAST (visitAttribute_index, visitor:2340-2346)
            if self.accept("-"):
                idx -= int(self.eat().text)
            return idx
        return int(self.eat().text)

    def _number(self, negate=False) -> Expr:
        txt = self.eat().text
        sfx = txt[-1].lower()
        if sfx == "l":
            v, ty = int(txt[:-1]), "long"
        elif sfx == "f":
            v, ty = float(txt[:-1]), "float"
        elif sfx == "d":
            v, ty = float(txt[:-1]), "double"
        elif "." in txt or "e" in txt.lower():
            v, ty = float(txt), "double"
        else:
            v, ty = int(txt), "int"
            if v > 2**31 - 1:
                raise SiddhiParserException(f"int literal out of range: {txt}")
        if negate:
            v = -v
        return Expr("const", value=v, vtype=ty)


def parse_app(text: str) -> App:
    return Parser(text).parse_app()
