#!/usr/bin/env python3
"""Transcribe the reference's known-answer tests into JSON fixtures (data only).

Reads the reference's TestNG sources *as text* (study; nothing is executed or
copied) and extracts, per straight-line ``@Test`` method: the SiddhiQL app
string, the ordered ``InputHandler.send`` calls with their timestamps (explicit
in playback tests; a simulated wall clock advanced by ``Thread.sleep`` for
wall-clock tests), the rows asserted with ``assertArrayEquals`` inside the
callback, and the asserted in-event count.  Tests that need Java control flow
(loops, helper threads, random data) are skipped.  Output: one JSON file per
reference test class under tests/golden/, each entry carrying the reference
``file:line`` it came from.

Usage: python tests/golden/extract_golden.py [REFERENCE_ROOT]
"""
from __future__ import annotations

import json
import os
import re
import sys

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
TEST_ROOT = os.path.join(REF, "modules/siddhi-core/src/test/java/io/siddhi/core/query")
SUITES = [
    "pattern/EveryPatternTestCase.java",
    "pattern/CountPatternTestCase.java",
    "pattern/LogicalPatternTestCase.java",
    "pattern/WithinPatternTestCase.java",
    "pattern/ComplexPatternTestCase.java",
    "pattern/absent/AbsentPatternTestCase.java",
    "pattern/absent/EveryAbsentPatternTestCase.java",
    "pattern/absent/LogicalAbsentPatternTestCase.java",
    "pattern/absent/AbsentWithEveryPatternTestCase.java",
    "sequence/SequenceTestCase.java",
    "sequence/absent/AbsentSequenceTestCase.java",
    "sequence/absent/EveryAbsentSequenceTestCase.java",
    "sequence/absent/LogicalAbsentSequenceTestCase.java",
    "sequence/absent/AbsentWithEverySequenceTestCase.java",
    "partition/PatternPartitionTestCase.java",
    "partition/SequencePartitionTestCase.java",
]
OUT = os.path.dirname(os.path.abspath(__file__))
WALL_T0 = 1_700_000_000_000  # simulated System.currentTimeMillis() at app start


class Skip(Exception):
    pass


def java_string_literals(expr: str) -> str:
    """Concatenate the string literals of a Java `"a" + "b"` expression."""
    out = []
    for m in re.finditer(r'"((?:[^"\\]|\\.)*)"', expr):
        s = m.group(1)
        s = s.replace('\\n', '\n').replace('\\t', '\t').replace('\\"', '"').replace("\\'", "'")
        out.append(s)
    return "".join(out)


def split_top(s: str, sep=","):
    parts, depth, cur, q = [], 0, [], None
    for ch in s:
        if q:
            cur.append(ch)
            if ch == q:
                q = None
            continue
        if ch in "\"'":
            q = ch
            cur.append(ch)
            continue
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == sep and depth == 0:
            parts.append("".join(cur).strip())
            cur = []
        else:
            cur.append(ch)
    if "".join(cur).strip():
        parts.append("".join(cur).strip())
    return parts


def java_value(tok: str):
    t = tok.strip()
    t = re.sub(r"^\((?:Object|Float|Double|Integer|Long|String)\)\s*", "", t)
    if t == "null":
        return None
    if t in ("true", "false"):
        return t == "true"
    if t.startswith('"'):
        return {"s": java_string_literals(t)}
    m = re.fullmatch(r"([-+]?\d+(?:\.\d*)?(?:[eE][-+]?\d+)?)([fFdDlL]?)", t)
    if m:
        num, sfx = m.group(1), m.group(2).lower()
        if sfx == "f":
            return {"f": float(num)}
        if sfx == "d" or "." in num or "e" in num.lower():
            return {"d": float(num)}
        if sfx == "l":
            return {"l": int(num)}
        return {"i": int(num)}
    raise Skip(f"value {t!r}")


def object_array(s: str):
    m = re.search(r"new\s+Object\s*\[\s*\]\s*\{(.*)\}\s*$", s.strip(), re.S)
    if not m:
        raise Skip(f"object array {s[:60]!r}")
    return [java_value(x) for x in split_top(m.group(1))]


def balanced(body: str, start: int) -> int:
    """Index just past the ')' matching the '(' at body[start]."""
    depth, q, i = 0, None, start
    while i < len(body):
        ch = body[i]
        if q:
            if ch == "\\":
                i += 2
                continue
            if ch == q:
                q = None
        elif ch in "\"'":
            q = ch
        elif ch == "(":
            depth += 1
        elif ch == ")":
            depth -= 1
            if depth == 0:
                return i + 1
        i += 1
    raise Skip("unbalanced")


def extract_method(name, body, line, relpath):
    if re.search(r"new Thread|Random|executorService|persist\(|restore|setPurge|getTimestampGenerator|"
                 r"@app:async|debug|@async|snapshot|enablePlayBack|setStatisticsLevel", body, re.S):
        raise Skip("unsupported helper")
    strings = {}
    for m in re.finditer(r"String\s+(\w+)\s*=\s*(.*?);\s*\n", body, re.S):
        strings[m.group(1)] = java_string_literals(m.group(2))
    m = re.search(r"createSiddhiAppRuntime\((.*?)\);", body, re.S)
    if not m:
        raise Skip("no app")
    app = ""
    for part in m.group(1).split("+"):
        part = part.strip()
        if part.startswith('"'):
            app += java_string_literals(part)
        elif part in strings:
            app += strings[part]
        else:
            raise Skip(f"app part {part}")
    playback = "@app:playback" in app.lower() or "@app:playback" in app
    if re.search(r"@app:playback\s*\(", app, re.I):
        raise Skip("playback heartbeat")
    # callback
    cbm = re.search(r'addCallback\(\s*"(\w+)"\s*,\s*new\s+(QueryCallback|StreamCallback)', body)
    tum = re.search(r'TestUtil\.add(Query|Stream)Callback\(', body)
    rows = []
    if cbm:
        cb_name, cb_kind = cbm.group(1), cbm.group(2)
        cb_start = body.index("(", cbm.start())
        cb_end = balanced(body, cb_start)
        cb_body = body[cb_start:cb_end]
        if re.search(r"assertArrayEquals\([^;]*removeEvents", cb_body):
            raise Skip("asserts on remove events")
        for am in re.finditer(r"assertArrayEquals\(", cb_body):
            end = balanced(cb_body, am.end() - 1)
            args = split_top(cb_body[am.end():end - 1])
            if len(args) != 2 or "getData" not in args[1]:
                raise Skip("assertArrayEquals form")
            rows.append(object_array(args[0]))
        if re.search(r"\bif\s*\(\s*(?:inEventCount|count)\b[^)]*%", cb_body):
            raise Skip("modular callback asserts")
    elif tum:
        cb_kind = "QueryCallback" if tum.group(1) == "Query" else "StreamCallback"
        cb_start = tum.end() - 1
        cb_end = balanced(body, cb_start)
        args = split_top(body[cb_start + 1:cb_end - 1])
        cb_name = java_string_literals(args[1])
        rows = [object_array(a) for a in args[2:]]
    else:
        raise Skip("no callback")
    pre = body[:cb_start]
    if re.search(r"\bfor\s*\(|\bwhile\s*\(", body[cb_end:]):
        raise Skip("control flow")
    # handlers
    handlers = {}
    for hm in re.finditer(r'InputHandler\s+(\w+)\s*=\s*\w+\.getInputHandler\("(\w+)"\)', body):
        handlers[hm.group(1)] = hm.group(2)
    rest = body[cb_end:]
    sd = re.search(r"\w+\.shutdown\(\)", rest)
    if sd:
        rest = rest[:sd.start()]  # nothing after shutdown() reaches the callback
    ops = []
    now = WALL_T0
    started = False
    if re.search(r"\.start\(\)", pre):
        started = True
    for sm in re.finditer(r"(\w+)\.send\(|Thread\.sleep\((\d+)\)|(\w+)\.start\(\)|"
                          r"assertEquals\(|waitForInEvents\(\s*(\d+)\s*,\s*\w+\s*,\s*(\d+)\s*\)|"
                          r"waitForEvents\(\s*(\d+)\s*,\s*(\d+)\s*,\s*\w+\s*,\s*(\d+)\s*\)", rest):
        if sm.group(3) is not None:
            started = True
            continue
        if sm.group(4) is not None:
            if not playback:
                ops.append({"wait_in_events": {"sleep": int(sm.group(4)), "retry": int(sm.group(5))}})
            continue
        if sm.group(6) is not None:
            if not playback:
                ops.append({"wait_events": {"sleep": int(sm.group(6)), "expected": int(sm.group(7)),
                                            "timeout": int(sm.group(8))}})
            continue
        if sm.group(2) is not None:
            if not playback:
                now += int(sm.group(2))
                ops.append({"advance": now})
            continue
        if sm.group(0).startswith("assertEquals"):
            continue
        var = sm.group(1)
        if var not in handlers:
            raise Skip(f"send on {var}")
        end = balanced(rest, sm.end() - 1)
        args = rest[sm.end():end - 1]
        parts = split_top(args)
        if len(parts) == 1 and parts[0].startswith("new Object"):
            if playback:
                raise Skip("playback send without timestamp")
            ops.append({"send": handlers[var], "ts": now, "data": object_array(parts[0])})
        elif len(parts) == 2 and parts[1].startswith("new Object"):
            tsm = re.fullmatch(r"(\d+)[lL]?", parts[0].strip())
            if not tsm:
                raise Skip("non-literal timestamp")
            ops.append({"send": handlers[var], "ts": int(tsm.group(1)), "data": object_array(parts[1])})
        elif len(parts) == 1 and parts[0].startswith("new Event("):
            inner = parts[0][len("new Event("):-1]
            ip = split_top(inner)
            tsm = re.fullmatch(r"(\d+)[lL]?", ip[0].strip())
            if not tsm:
                raise Skip("non-literal Event timestamp")
            ops.append({"send": handlers[var], "ts": int(tsm.group(1)), "data": object_array(ip[1])})
        else:
            raise Skip("send form")
    if not started:
        raise Skip("no start")
    cnt = None
    for cm in re.finditer(r"assertEquals\(\s*(?:\"[^\"]*\"\s*,\s*)?(\d+)\s*,\s*"
                          r"(?:inEventCount(?:\.get\(\))?|\w+\.getInEventCount\(\))\s*\)", rest):
        cnt = int(cm.group(1))
    if re.search(r"assertEquals\(\s*(?:\"[^\"]*\"\s*,\s*)?false\s*,\s*eventArrived\s*\)", rest):
        cnt = 0 if cnt is None else cnt
    if cnt is None:
        raise Skip("no count assertion")
    rcnt = None
    for cm in re.finditer(r"assertEquals\(\s*(?:\"[^\"]*\"\s*,\s*)?(\d+)\s*,\s*"
                          r"(?:removeEventCount(?:\.get\(\))?|\w+\.getRemoveEventCount\(\))\s*\)", rest):
        rcnt = int(cm.group(1))
    if cbm is None:
        mode = "prefix"  # TestUtil callbacks assert expected[i] for the i-th event, in order
    elif cnt == len(rows):
        mode = "ordered"
    elif len(rows) == 1:
        mode = "each"
    elif len(rows) == 0:
        mode = "count"
    else:
        mode = "contains"
    return {
        "name": f"{os.path.basename(relpath)[:-5]}.{name}",
        "source": f"modules/siddhi-core/src/test/java/io/siddhi/core/query/{relpath}:{line}",
        "app": app,
        "playback": playback,
        "start_clock": 0 if playback else WALL_T0,
        "callback": {"name": cb_name, "kind": cb_kind},
        "ops": ops,
        "expected": {"count": cnt, "remove_count": rcnt, "rows": rows, "mode": mode},
    }


def main():
    summary = {}
    for rel in SUITES:
        path = os.path.join(TEST_ROOT, rel)
        src = open(path).read()
        fixtures, skipped = [], {}
        for m in re.finditer(r"@Test[^\n]*\n\s*public void (\w+)\(\)[^{]*\{", src):
            start = m.end()
            nxt = src.find("@Test", start)
            body = src[start: nxt if nxt > 0 else len(src)]
            line = src[:m.start()].count("\n") + 1
            try:
                fixtures.append(extract_method(m.group(1), body, line, rel))
            except Skip as e:
                skipped[m.group(1)] = str(e)
        out = os.path.join(OUT, os.path.basename(rel).replace(".java", ".json"))
        with open(out, "w") as f:
            json.dump({"suite": rel, "fixtures": fixtures, "skipped": skipped}, f, indent=1)
        summary[rel] = (len(fixtures), len(skipped))
    for k, v in summary.items():
        print(f"{k}: {v[0]} extracted, {v[1]} skipped")


if __name__ == "__main__":
    main()
