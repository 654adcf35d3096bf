#!/usr/bin/env python3
"""Hand transcription (data only) of the deterministic playback known-answer tests that
extract_golden.py refuses mechanically (``++now`` timestamps, loops, clock-only sends on a
stream no query reads, stream callbacks on an inner partition's output).  SURVEY.md §8c names
them as the pins of the absent / playback semantics behind config 4.

Each fixture follows the reference test statement by statement: the timestamps are what the
test's ``++now`` / ``now += ...`` arithmetic produces from a base (the test's
``System.currentTimeMillis()``, here T0; the result does not depend on it), a send on a stream no
query reads is a clock advance (InputHandler.send in playback sets the clock first,
InputHandler.java:59-64), and the test's intermediate count asserts become ``expect_count`` ops.

Output: tests/golden/PlaybackTranscribed.json.  Usage: python tests/golden/transcribe_playback.py
"""
import json
import os

T0 = 1_700_000_000_000
P = "modules/siddhi-core/src/test/java/io/siddhi/core/query/"


def S(x):
    return {"s": x}


def F(x):
    return {"f": x}


def I(x):
    return {"i": x}


def stock(sym, price, vol=100):
    return [S(sym), F(price), I(vol)]


fixtures = []

# pattern/absent/EveryAbsentPatternTestCase.java:113-160 testQueryAbsent3
fixtures.append({
    "name": "EveryAbsentPatternTestCase.testQueryAbsent3",
    "source": P + "pattern/absent/EveryAbsentPatternTestCase.java:113",
    "app": "@app:playback define stream Stream1 (symbol string, price float, volume int); "
           "define stream Stream2 (symbol string, price float, volume int); "
           "define stream TimerStream (symbol string); "
           "@info(name = 'query1') "
           "from (e1=Stream1[price>20] -> every not Stream2[price>e1.price] for 900 milliseconds) within 2 sec "
           "select e1.symbol as symbol1 insert into OutputStream ;",
    "playback": True, "start_clock": 0,
    "callback": {"name": "query1", "kind": "QueryCallback"},
    "ops": [
        {"send": "Stream1", "ts": T0, "data": stock("WSO2", 55.6)},
        {"send": "TimerStream", "ts": T0 + 1000, "data": [S("UPDATE-TIME")]},
        {"expect_count": 1},
        {"send": "TimerStream", "ts": T0 + 2000, "data": [S("UPDATE-TIME")]},
        {"expect_count": 2},
        {"send": "TimerStream", "ts": T0 + 3000, "data": [S("UPDATE-TIME")]},
    ],
    "expected": {"count": 2, "remove_count": 0, "rows": [[S("WSO2")], [S("WSO2")]], "mode": "ordered"},
})

# pattern/absent/AbsentWithEveryPatternTestCase.java:277-310 testQuery7 (the idle.time heartbeat
# never fires: the four sends are back to back and the asserts follow at once)
fixtures.append({
    "name": "AbsentWithEveryPatternTestCase.testQuery7",
    "source": P + "pattern/absent/AbsentWithEveryPatternTestCase.java:277",
    "app": "@app:playback(idle.time = '10 milliseconds', increment = '10 milliseconds') "
           "define stream Stream1 (symbol string, price float, volume int); "
           "@info(name = 'query1') "
           "from every e1=Stream1[price>20] -> not Stream1[symbol==e1.symbol and price>e1.price] for 1sec "
           "select e1.symbol as symbol insert into OutputStream ;",
    "playback": True, "start_clock": 0,
    "callback": {"name": "query1", "kind": "QueryCallback"},
    "ops": [
        {"send": "Stream1", "ts": 1544512385000, "data": stock("WSO2", 55.6)},
        {"send": "Stream1", "ts": 1544512385100, "data": stock("GOOG", 55.6)},
        {"send": "Stream1", "ts": 1544512385800, "data": stock("WSO2", 55.7)},
        {"send": "Stream1", "ts": 1544512386200, "data": stock("GOOG", 55.6)},
    ],
    "expected": {"count": 1, "remove_count": 0, "rows": [[S("GOOG")]], "mode": "ordered"},
})

# pattern/LogicalPatternTestCase.java:1180-1247 testQuery21 and :1250-1317 testQuery22
LOGICAL_APP = ("@app:playback define stream Stream1 (symbol string, price float, volume int); "
               "define stream Stream2 (symbol string, price float, volume int); "
               "define stream Stream3 (symbol string, price float, volume int); "
               "@info(name = 'query1') "
               "from every (e1=Stream1[price>10] and e2=Stream2[price>20] -> e3=Stream3[price>30]) within 1 sec "
               "select e1.symbol as symbol1, e2.symbol as symbol2, e3.symbol as symbol3 "
               "insert into OutputStream ;")
LOGICAL_ROWS = [[S("IBM"), S("WSO2"), S("GOOGLE")], [S("IBM1"), S("WSO21"), S("GOOGLE1")]]
for name, line, head in (("testQuery21", 1180, [("Stream1", "ORACLE", 15.0), ("Stream2", "MICROSOFT", 45.0)]),
                         ("testQuery22", 1250, [("Stream1", "ORACLE", 15.0)])):
    now = T0
    ops = []
    for st, sym, pr in head:
        now += 1
        ops.append({"send": st, "ts": now, "data": stock(sym, pr)})
    now += 5000
    for st, sym, pr in (("Stream1", "IBM", 55.0), ("Stream2", "WSO2", 65.0), ("Stream3", "GOOGLE", 75.0),
                        ("Stream1", "IBM1", 55.0), ("Stream2", "WSO21", 65.0), ("Stream3", "GOOGLE1", 75.0)):
        now += 1
        ops.append({"send": st, "ts": now, "data": stock(sym, pr)})
    fixtures.append({
        "name": "LogicalPatternTestCase." + name,
        "source": P + f"pattern/LogicalPatternTestCase.java:{line}",
        "app": LOGICAL_APP, "playback": True, "start_clock": 0,
        "callback": {"name": "query1", "kind": "QueryCallback"},
        "ops": ops,
        "expected": {"count": 2, "remove_count": 0, "rows": LOGICAL_ROWS, "mode": "ordered"},
    })

# pattern/EveryPatternTestCase.java:602-690 testQuery10 (stream callback on the partition's output)
now = T0
ops = []


def login(stream, i, user, typ):
    global now
    now += 1
    ops.append({"send": stream, "ts": now, "data": [S(f"id_{i}"), S(user), S(typ)]})


for i in range(1, 7):
    login("LoginFailure", i, "hans", "failure")
login("LoginSuccess", 7, "hans", "success")
for i in range(8, 16):
    login("LoginFailure", i, "werner", "failure")
login("LoginSuccess", 16, "werner", "success")
now += 3 * 1000
for i in range(17, 23):
    login("LoginFailure", i, "hans", "failure")
login("LoginSuccess", 23, "hans", "success")
fixtures.append({
    "name": "EveryPatternTestCase.testQuery10",
    "source": P + "pattern/EveryPatternTestCase.java:602",
    "app": "@app:playback\ndefine stream LoginFailure (id string, user string, type string);\n"
           "define stream LoginSuccess (id string, user string, type string);\n\n"
           "partition with (user of LoginFailure, user of LoginSuccess)\nbegin\n\n"
           "  from every (e0=LoginFailure-> e1=LoginFailure<3:> -> e2=LoginSuccess) \n"
           "  select e0.id as id, e2.user as user\n  insert into BreakIn\n\nend;",
    "playback": True, "start_clock": 0,
    "callback": {"name": "BreakIn", "kind": "StreamCallback"},
    "ops": ops,
    "expected": {"count": 3, "remove_count": 0,
                 "rows": [[S("id_1"), S("hans")], [S("id_8"), S("werner")], [S("id_17"), S("hans")]],
                 "mode": "ordered"},
})

# pattern/CountPatternTestCase.java:935-1003 testQuery16: Java evaluates send(++now, {++now, ...})
# left to right, so each send stamps ts = now + 1 and puts now + 2 in the (unselected, string-typed)
# id attribute; 400 rounds of 8 sends then now += 100; the test asserts the count only
now = 1
ops = []
for i in range(1, 401):
    for sym, pr in (("WSO2", 25.6), ("WSO2", 23.6), ("WSO2", 23.6), ("WSO2", 23.6), ("WSO2", 23.6),
                    ("GOOG", 27.6), ("GOOG", 28.6), ("GOOG", 28.6)):
        now += 1
        ts = now
        now += 1
        ops.append({"send": "Stream1", "ts": ts, "data": [S(str(now)), S(sym), F(pr), I(100)]})
    now += 100
fixtures.append({
    "name": "CountPatternTestCase.testQuery16",
    "source": P + "pattern/CountPatternTestCase.java:935",
    "app": "@app:playback\n define stream Stream1 (id string, symbol string, price float, volume int); "
           " @info(name = 'query1')  from every e1=Stream1[symbol=='WSO2']   -> e2=Stream1[symbol=='WSO2']<2:> "
           "-> e3=Stream1[symbol=='GOOG']  within 10 milliseconds  select e1.price as price1, e2.price as price2, "
           "e3.price as price3  insert into OutputStream;",
    "playback": True, "start_clock": 0,
    "callback": {"name": "OutputStream", "kind": "StreamCallback"},
    "ops": ops,
    "expected": {"count": 1200, "remove_count": 0, "rows": [], "mode": "ordered"},
})

out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "PlaybackTranscribed.json")
with open(out, "w") as f:
    json.dump({"suite": "hand-transcribed playback tests (transcribe_playback.py)", "fixtures": fixtures}, f,
              indent=None, separators=(",", ":"))
print(out, len(fixtures))
