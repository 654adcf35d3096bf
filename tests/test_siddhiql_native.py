"""The library's SiddhiQL lowering (shp_compile_siddhiql, siddhi_amd/csrc/siddhiql.cpp) against
siddhi_amd/query/compiler.py: byte-identical program JSON for every query of every transcribed
reference fixture (tests/golden/*.json), the §8d configs and the test apps, the same string
dictionary afterwards, and an error exactly where the Python lowering raises.

Pure host code: runs on the CPU (the library loads without a GPU; nothing here touches HIP)."""
import ctypes
import json
import random

import pytest

from golden_runner import load_fixtures
from siddhi_amd import native, synth
from siddhi_amd.query.compiler import Dictionary, QueryCompiler
from siddhi_amd.query.siddhiql import parse_app


def _lib():
    L = native.lib()
    L.shp_dict_create.restype = ctypes.c_void_p
    L.shp_dict_create.argtypes = [ctypes.c_int32]
    L.shp_dict_intern.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int64]
    L.shp_dict_intern.restype = ctypes.c_int32
    L.shp_dict_size.argtypes = [ctypes.c_void_p]
    L.shp_dict_size.restype = ctypes.c_int32
    L.shp_dict_string.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_char_p, ctypes.c_size_t]
    L.shp_dict_string.restype = ctypes.c_int64
    L.shp_dict_destroy.argtypes = [ctypes.c_void_p]
    L.shp_compile_siddhiql.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_char_p,
                                       ctypes.c_size_t]
    L.shp_compile_siddhiql.restype = ctypes.c_int64
    L.shp_siddhiql_queries.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t]
    L.shp_siddhiql_queries.restype = ctypes.c_int64
    L.shp_compile_last_error.restype = ctypes.c_char_p
    return L


def native_compile(L, app, name, d):
    n = L.shp_compile_siddhiql(app.encode(), name.encode() if name else None, d, None, 0)
    if n < 0:
        return None, L.shp_compile_last_error().decode()
    buf = ctypes.create_string_buffer(n + 1)
    assert L.shp_compile_siddhiql(app.encode(), name.encode() if name else None, d, buf, n + 1) == n
    return buf.raw[:n].decode(), None


def dict_strings(L, d):
    out = []
    for i in range(L.shp_dict_size(d)):
        n = L.shp_dict_string(d, i, None, 0)
        b = ctypes.create_string_buffer(n + 1)
        L.shp_dict_string(d, i, b, n + 1)
        out.append(b.raw[:n].decode())
    return out


def python_programs(app_text):
    """compile_app's per-query outcome in order: (name, json) until the first query that raises."""
    app = parse_app(app_text)
    d = Dictionary()
    out = []
    for q in app.queries:
        try:
            out.append((q.name, QueryCompiler(app, q, d).compile().program_json()))
        except Exception as e:  # noqa: BLE001 (any error of the Python lowering)
            out.append((q.name, e))
            break
    return out, d


def check_app(L, app_text):
    try:
        want, pyd = python_programs(app_text)
    except Exception:  # noqa: BLE001 the Python parser rejects the app: so must the library
        d = L.shp_dict_create(0)
        try:
            got, err = native_compile(L, app_text, None, d)
            assert got is None, f"native accepted an app the Python parser rejects:\n{app_text}"
        finally:
            L.shp_dict_destroy(d)
        return "parse-error"
    d = L.shp_dict_create(0)
    try:
        for name, prog in want:
            got, err = native_compile(L, app_text, name, d)
            if isinstance(prog, Exception):
                assert got is None, f"native accepted query {name} that Python rejects ({prog}):\n{app_text}"
                return "error"
            assert err is None, f"native rejected query {name}: {err}\n{app_text}"
            assert got == prog, f"query {name}:\nnative {got}\npython {prog}"
        assert dict_strings(L, d) == pyd.strings
    finally:
        L.shp_dict_destroy(d)
    return "ok"


FIXTURES = load_fixtures()


def test_every_fixture_lowers_identically():
    L = _lib()
    outcomes = {}
    seen = set()
    for fx in FIXTURES:
        if fx["app"] in seen:
            continue
        seen.add(fx["app"])
        outcomes[fx["name"]] = check_app(L, fx["app"])
    # 449 fixtures share 230 distinct app texts; every in-scope one lowers identically, and the
    # out-of-scope ones (test_oracle_golden.OUT_OF_SCOPE) are rejected by both lowerings
    from test_oracle_golden import OUT_OF_SCOPE
    assert len(outcomes) >= 200
    bad = {k: v for k, v in outcomes.items() if (v == "ok") == (k in OUT_OF_SCOPE)}
    assert not bad, bad


def test_config_queries_lower_identically():
    L = _lib()
    for key, text in synth.QUERIES.items():
        assert check_app(L, text) == "ok", key


APPS = [
    # comparison grid, functions, nulls, strings, arithmetic promotion
    "define stream S (a int, b long, c float, d double, s string, f bool); "
    "from every e1=S[a > 3 and c <= 2.5f or not (d != 1e-7)] -> e2=S[b * 2 + a / 3 > e1.b % 5L and s == 'x\\u'] "
    "within 10 min select e1.a, e2.s insert into O;",
    "define stream S (a int, c float); from every e1=S[ifThenElse(a > 2, c, 1.0f) > 1.5f and "
    "coalesce(c, 2.0f) < 100f and instanceOfFloat(c)] -> e2=S[c is null or e1.c is null] select e1.c insert into O;",
    "@app:playback define stream A (k string, p float); define stream B (k string, p float); "
    "define stream C (k string, p float); partition with (k of A, k of B, k of C) begin "
    "@info(name='q') from every (e1=A[p>20] and e2=B[p>20]) -> not C[p>e1.p] for 5 sec within 10 sec "
    "select e1.k, e1.p, e2.p insert into O; end;",
    "define stream S (v float); from every e1=S[v>20]<2:5>, e2=S[v<e1[last].v] select e1[0].v, e1[last].v, e2.v "
    "insert into O;",
    "define stream S (v float, w double); from e1=S[v > 1.5e16 or w < -0.00001 or w == 123456789.125 or v > 1e-4] "
    "-> e2=S[e2[last].v > 0.1] -> e3=S[e1.v * 0.30000000000000004 < 3.14159d] select e1.v insert into O;",
    "define stream S (v float); from e1=S -> not S[v > 2] for 3 sec and e3=S select e1.v insert into O;",
    "define stream S (v float); from e1=S or not S[v > 2] for 3 sec select e1.v insert into O;",
    "define stream S (v int); from every e1=S[v > 2]+, e2=S[v == e1[last-1].v]?, e3=S*  select e1.v, e3.v "
    "insert into O;",
    "define stream S (v int); from e1=S<:4> -> e2=S<2:> select e1.v insert into O;",
    "define stream S (v int); from every e1=S[v>1] -> e2=S[v>e1.v] select count() as c, avg(e2.v) as a "
    "insert into O;",
    "define stream S (v int); partition with (v of S) begin from every e1=S[v>1] -> e2=S[v>e1.v] "
    "select max(e2.v) as m insert into O; end;",
    # errors on both sides
    "define stream S (v int); from every e1=S -> e2=T[v > 1] select e1.v insert into O;",
    "define stream S (v int); from every e1=S -> e2=S[v > 'a'] select e1.v insert into O;",
    "define stream S (v int); from every e1=S -> e2=S[q > 1] select e1.v insert into O;",
    "define stream S (v int); from every e1=S -> e2=S[v > 1] select * insert into O;",
    "define stream S (v int); from every e1=S -> e2=S[v + 1] select e1.v insert into O;",
    "define stream S (v int); from every e1=S -> e2=S[foo(v)] select e1.v insert into O;",
    "define stream S (v int); from every e1=S, e2=S -> e3=S select e1.v insert into O;",
    "define stream S (v int); from every e1=S[v > 3000000000] -> e2=S select e1.v insert into O;",
    "define stream S (v int); from e1=S[e9 is null] -> e2=S select e1.v insert into O;",
]


N_OK = 11  # APPS[:N_OK] lower; the rest are rejected (by the parser or the lowering) on both sides


@pytest.mark.parametrize("i", range(len(APPS)))
def test_handwritten_apps(i):
    r = check_app(_lib(), APPS[i])
    assert (r == "ok") == (i < N_OK), r


def test_float_constants_print_like_python():
    """Constants are printed as Python's repr(float) would (shortest round-trip digits; exponent
    form below 1e-4 and from 1e16 up) -- random magnitudes and digit counts."""
    L = _lib()
    rng = random.Random(7)
    for _ in range(300):
        mant = rng.choice(["1", "25", "3.5", "123456789.123", "0.1", "9.999999", "7"])
        ex = rng.randint(-30, 30)
        lit = f"{mant}e{ex}"
        app = f"define stream S (d double); from e1=S[d > {lit}] -> e2=S[d < -{lit}] select e1.d insert into O;"
        assert check_app(L, app) == "ok", lit


def test_queries_describe_names_and_partitions():
    L = _lib()
    text = synth.QUERIES[4]
    n = L.shp_siddhiql_queries(text.encode(), None, 0)
    b = ctypes.create_string_buffer(n + 1)
    L.shp_siddhiql_queries(text.encode(), b, n + 1)
    qs = json.loads(b.raw[:n].decode())
    app = parse_app(text)
    assert [q["name"] for q in qs] == [q.name for q in app.queries]
    assert qs[0]["partition"] == app.queries[0].partition
    assert qs[0]["playback"] is True


def test_bounded_dictionary_refuses_past_capacity():
    L = _lib()
    d = L.shp_dict_create(2)
    try:
        assert L.shp_dict_intern(d, b"a", 1) == 0
        assert L.shp_dict_intern(d, b"b", 1) == 1
        assert L.shp_dict_intern(d, b"a", 1) == 0
        assert L.shp_dict_intern(d, b"c", 1) == -6  # SHP_ERR_KEYS
        assert L.shp_dict_size(d) == 2
    finally:
        L.shp_dict_destroy(d)
