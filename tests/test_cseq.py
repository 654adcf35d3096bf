"""The count-sequence path (siddhi_amd/csrc/cseq.h): `[every] e1=S[f1]<min:M>, e2=S[f2]` (C3', C3).

CPU: the per-key automaton cseq.h implements, restated here in Python, against the oracle's
object-level restatement of CountPreStateProcessor / CountPostStateProcessor /
StreamPreStateProcessor (oracle/oracle.cpp) -- every M in 1..8, every comparison of
`e2.v OP e1[last].v`, NaN values, split batches.  This pins the rule the kernel relies on.
GPU (`-m gpu`): libsiddhi_hip.so's k_cseq against the oracle: C3' at its key counts (including
1M keys), nulls, int columns, split batches, snapshot/restore, and the general lanes on the same
stream.
"""
import operator

import numpy as np
import pytest

from diff_util import compare, per_key, program_for, run, small_stream
from oracle.oracle import OracleEngine

OPS = {"<": operator.lt, "<=": operator.le, ">": operator.gt, ">=": operator.ge, "==": operator.eq,
       "!=": operator.ne}


def _app(M, op, typ="float", f1="v > 20", every=True, mn=1):
    ev = "every " if every else ""
    return (f"define stream S (k string, v {typ}); partition with (k of S) begin @info(name='q') "
            f"from {ev}e1=S[{f1}]<{mn}:{M}>, e2=S[v {op} e1[last].v] select e1[0].v as a, e2.v as c "
            f"insert into Out; end;")


def _cq(app):
    from siddhi_amd.query.compiler import compile_app
    return compile_app(app)[1][0]


def _push(eng, ts, key, v, batch, nul=None):
    st = np.zeros(len(ts), np.int32)
    for lo in range(0, len(ts), batch):
        hi = min(len(ts), lo + batch)
        eng.push(ts[lo:hi], key[lo:hi], st[lo:hi], [v[lo:hi]], [None if nul is None else nul[lo:hi]])
    return per_key(eng.fetch())


def automaton(M, op, ts, key, v, f1=lambda x: x > 20, nul=None):
    """cseq.h's rule: per key, L = length of e1's chain (the key's last L events)."""
    cmp = OPS[op]
    out, chain = {}, {}
    for i in range(len(ts)):
        k = int(key[i])
        c = chain.get(k, [])
        x = v[i]
        xn = nul is not None and nul[i]
        prev_null = bool(c) and nul is not None and nul[c[-1]]
        f1x = (not xn) and f1(x)
        if c and not xn and not prev_null and cmp(x, v[c[-1]]):
            out.setdefault(k, []).append((int(ts[i]), 0, i, (tuple(c), (i,))))
            chain[k] = [i] if (len(c) == M and f1x) else []
        elif c and len(c) < M and f1x:
            chain[k] = c + [i]
        elif f1x:
            chain[k] = [i]
        else:
            chain[k] = []
    return out


def tables(M, every, mn):
    """cseq.h cs_tables: T0 (not f1), T10 (f1 without f2), T11 (f1 and f2) on L in 0..M+1, and
    whether the shape emits.  D = M + 1 is the dead state of a start armed once (no `every`:
    CountPreStateProcessor.init / resetState arm it once); min >= 2 never emits, since a chain
    reaches e1's new-and-every list only at min, and the sequence resets the pending one on the
    key's next event (CountPreStateProcessor.java:288-305, StreamPreStateProcessor.java:360)."""
    D = M + 1
    n = M + 2
    if mn >= 2:  # L = 1: the count-1 partial of the key's last event (alive until its next event)
        if every:
            return [0] * n, [1] * n, [1] * n, False
        return [D] * n, [1] + [D] * (n - 1), [1] + [D] * (n - 1), False
    if every:
        return [0] * n, [1] + [i + 1 for i in range(1, M)] + [1, 1], [1] + [0] * (M - 1) + [1, 1], True
    return [D] * n, [1] + [i + 1 for i in range(1, M)] + [D, D], [1] + [D] * M + [D], True


def table_automaton(M, op, every, mn, ts, key, v, f1=lambda x: x > 20, nul=None):
    """The table form the kernels run (cs_tables / co_tables): per key, L before the event and the
    key's last M events; a match closes when 1 <= L <= M and f2 holds."""
    cmp = OPS[op]
    t0, t10, t11, emit_on = tables(M, every, mn)
    out, L, hist = {}, {}, {}
    for i in range(len(ts)):
        k = int(key[i])
        Lb = L.get(k, 0)
        h = hist.setdefault(k, [])
        xn = nul is not None and nul[i]
        a = (not xn) and f1(v[i])
        b = bool(h) and not xn and not (nul is not None and nul[h[-1]]) and cmp(v[i], v[h[-1]])
        if emit_on and 1 <= Lb <= M and b:
            out.setdefault(k, []).append((int(ts[i]), 0, i, (tuple(h[len(h) - Lb:]), (i,))))
        L[k] = (t11 if b else t10)[Lb] if a else t0[Lb]
        h.append(i)
        if len(h) > M:
            h.pop(0)
    return out


def _stream(rng, n, keys, lo=15, hi=30, nan=0.01):
    ts = np.cumsum(rng.integers(0, 3, n)).astype(np.int64) + 1000
    key = rng.integers(0, keys, n).astype(np.int32)
    v = rng.integers(lo, hi, n).astype(np.float32)
    v[rng.random(n) < nan] = np.nan
    return ts, key, v


@pytest.mark.parametrize("M", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("op", list(OPS))
def test_automaton_matches_oracle(M, op):
    rng = np.random.default_rng(M * 31 + len(op))
    ts, key, v = _stream(rng, 12_000, 13)
    cq = _cq(_app(M, op))
    want = _push(OracleEngine(cq.program_json(), 0), ts, key, v, 4_999)
    got = automaton(M, op, ts, key, v)
    assert compare(want, got) is None, compare(want, got)
    assert sum(len(x) for x in want.values()) > 200


@pytest.mark.parametrize("every", [True, False], ids=["every", "once"])
@pytest.mark.parametrize("M", range(1, 9))
def test_table_automaton_matches_oracle_every_min_max(every, M):
    """Every <min:M> with min <= M <= 8, with and without `every`, against the oracle: the rule
    cs_tables encodes (C3 is `e1=S[v > 20]<2:5>` without every)."""
    ops = ["<", ">=", "!="]
    for mn in range(1, M + 1):
        op = ops[(M + mn) % 3]
        rng = np.random.default_rng(M * 100 + mn * 7 + every)
        ts, key, v = _stream(rng, 4_000, 5)
        cq = _cq(_app(M, op, every=every, mn=mn))
        want = _push(OracleEngine(cq.program_json(), 0), ts, key, v, 1_999)
        got = table_automaton(M, op, every, mn, ts, key, v)
        assert compare(want, got) is None, (mn, op, compare(want, got))
        if mn == 1:
            assert sum(len(x) for x in want.values()) >= (50 if every else 1)
    if every:  # the every / min 1 tables agree with the list form above
        rng = np.random.default_rng(3)
        ts, key, v = _stream(rng, 4_000, 7)
        assert compare(automaton(M, "<", ts, key, v), table_automaton(M, "<", True, 1, ts, key, v)) is None


@pytest.mark.parametrize("every", [True, False], ids=["every", "once"])
def test_table_automaton_live_chains_equal_oracle_oldest_live(every):
    """After every event: the oldest event the tables keep alive (the last L events of each key with
    1 <= L <= M) is the oracle's oldest live event -- including min >= 2, where L = 1 is the count-1
    partial the reference holds until the key's next event (shp_engine_oldest_live_seq, describe)."""
    for M, mn in ((5, 1), (5, 2), (3, 3), (8, 4), (2, 1)):
        rng = np.random.default_rng(M * 3 + mn + every)
        ts, key, v = _stream(rng, 500, 7, nan=0.0)
        cq = _cq(_app(M, "<", every=every, mn=mn))
        o = OracleEngine(cq.program_json(), 0)
        t0, t10, t11, _ = tables(M, every, mn)
        L, hist = {}, {}
        for i in range(len(ts)):
            o.push(ts[i:i + 1], key[i:i + 1], np.zeros(1, np.int32), [v[i:i + 1]], [None])
            o.fetch()
            k = int(key[i])
            h = hist.setdefault(k, [])
            Lb = L.get(k, 0)
            a, b = v[i] > 20, bool(h) and v[i] < v[h[-1]]
            L[k] = (t11 if b else t10)[Lb] if a else t0[Lb]
            h.append(i)
            del h[:-M]
            live = [hist[q][-L[q]] for q in L if 1 <= L[q] <= M]
            assert o.oldest_live_seq() == (min(live) if live else i + 1), (M, mn, i)


def test_table_automaton_with_nulls_once():
    rng = np.random.default_rng(19)
    ts, key, v = _stream(rng, 12_000, 400, nan=0.0)
    nul = (rng.random(len(ts)) < 0.05).astype(np.uint8)
    cq = _cq(_app(4, "<", every=False))
    want = _push(OracleEngine(cq.program_json(), 0), ts, key, v, 3_001, nul)
    got = table_automaton(4, "<", False, 1, ts, key, v, nul=nul)
    assert compare(want, got) is None, compare(want, got)
    assert sum(len(x) for x in want.values()) > 100


def test_automaton_matches_oracle_c3b_stream():
    cq = program_for("3b")
    g = small_stream(3, 150_000, 50)
    want = per_key(run(OracleEngine(cq.program_json(), 0), cq, g, 33_333))
    got = automaton(5, "<", g["ts"], g["key"], g["price"].astype(np.float32))
    assert compare(want, got) is None, compare(want, got)


def test_automaton_matches_oracle_with_nulls():
    rng = np.random.default_rng(9)
    ts, key, v = _stream(rng, 12_000, 11, nan=0.0)
    nul = (rng.random(len(ts)) < 0.05).astype(np.uint8)
    cq = _cq(_app(5, "<"))
    want = _push(OracleEngine(cq.program_json(), 0), ts, key, v, 3_001, nul)
    got = automaton(5, "<", ts, key, v, nul=nul)
    assert compare(want, got) is None, compare(want, got)


# ---------------------------------------------------------------- GPU (k_cseq)

def _hip(cq, keys, batch, force=0):
    from siddhi_amd.native import HipEngine
    return HipEngine(cq.program_json(), 0, max_keys=keys, max_batch=batch, force_general=force)


@pytest.mark.gpu
@pytest.mark.parametrize("keys,n,batch", [(1, 30_000, 7_001), (64, 200_000, 65_537), (20_000, 600_000, 200_003),
                                          (1_000_000, 3_000_000, 1_000_003)],
                         ids=["1key", "64keys", "20k", "1M"])
def test_c3b_cseq_vs_oracle(keys, n, batch):
    cq = program_for("3b")
    g = small_stream(3, n, keys)
    want = per_key(run(OracleEngine(cq.program_json(), 0), cq, g))
    eng = _hip(cq, keys, batch)
    assert eng.path == 3
    got = per_key(run(eng, cq, g, batch))
    assert compare(want, got) is None, compare(want, got)
    assert sum(len(x) for x in want.values()) > 1000


@pytest.mark.gpu
@pytest.mark.parametrize("M,op,typ", [(1, "<", "float"), (2, ">=", "float"), (3, "==", "int"), (5, "!=", "float"),
                                      (8, "<=", "int"), (5, ">", "int")])
def test_cseq_shapes_vs_oracle(M, op, typ):
    rng = np.random.default_rng(M * 7 + len(op))
    ts, key, v = _stream(rng, 150_000, 300)
    if typ == "int":
        v = np.nan_to_num(v, nan=17).astype(np.int32)
    cq = _cq(_app(M, op, typ))
    want = _push(OracleEngine(cq.program_json(), 0), ts, key, v, 40_009)
    eng = _hip(cq, 300, 1 << 16)
    assert eng.path == 3
    got = _push(eng, ts, key, v, 40_009)
    assert compare(want, got) is None, compare(want, got)
    assert sum(len(x) for x in want.values()) > 100


@pytest.mark.gpu
@pytest.mark.parametrize("every,mn,M,op,layout", [
    (False, 1, 4, "<", 0), (False, 1, 6, ">=", 4), (False, 1, 7, "<", 4), (False, 1, 8, "!=", 0),
    (False, 2, 5, "<", 0), (False, 2, 5, "<", 4), (True, 2, 5, "<", 4), (True, 3, 8, ">=", 0),
    (True, 1, 3, "!=", 4)])
def test_cseq_every_min_max_vs_oracle(every, mn, M, op, layout):
    """The count sequence's modes (cs_tables) on path 3, FULL rows and CHAIN32 words (owner path
    while M + 1 <= 7 without every, the sorted records past that)."""
    from siddhi_amd.native import HipEngine
    rng = np.random.default_rng(M * 13 + mn)
    ts, key, v = _stream(rng, 160_000, 4_000)
    cq = _cq(_app(M, op, every=every, mn=mn))
    want = _push(OracleEngine(cq.program_json(), 0), ts, key, v, 40_009)
    eng = HipEngine(cq.program_json(), 0, max_keys=4_000, max_batch=1 << 16, match_layout=layout)
    assert eng.path == 3
    got = _push(eng, ts, key, v, 40_009)
    assert compare(want, got) is None, compare(want, got)
    if mn == 1:
        assert sum(len(x) for x in want.values()) > (1000 if every else 500)


@pytest.mark.gpu
@pytest.mark.parametrize("mn,M,layout", [(2, 7, 4), (2, 7, 0), (1, 7, 4), (2, 6, 4)])
def test_cseq_once_dead_state_oldest_live_vs_oracle(mn, M, layout):
    """No `every`: a used once-armed start is the dead state D = M + 1.  At M = 7 that is past the
    owner kernel's 8-byte tables, so the engine must keep such shapes off the owner path:
    matches, the oldest live event and the described chain lengths agree with the oracle per push."""
    from siddhi_amd.native import HipEngine
    rng = np.random.default_rng(M * 31 + mn)
    ts, key, v = _stream(rng, 60_000, 500)
    cq = _cq(_app(M, "<", every=False, mn=mn))
    o = OracleEngine(cq.program_json(), 0)
    eng = HipEngine(cq.program_json(), 0, max_keys=500, max_batch=1 << 15, match_layout=layout)
    assert eng.path == 3
    st = np.zeros(len(ts), np.int32)
    for lo in range(0, len(ts), 15_013):
        hi = min(len(ts), lo + 15_013)
        args = (ts[lo:hi], key[lo:hi], st[lo:hi], [v[lo:hi]], [None])
        o.push(*args)
        eng.push(*args)
        want, got = per_key(o.fetch()), per_key(eng.fetch())
        assert compare(want, got) is None, (lo, compare(want, got))
        assert eng.oldest_live_seq() == o.oldest_live_seq(), lo
        d = eng.describe(eng.snapshot())
        assert all(0 <= s["e1"]["Count"] <= M for s in d["keys"].values())


@pytest.mark.gpu
def test_cseq_nulls_vs_oracle():
    rng = np.random.default_rng(4)
    ts, key, v = _stream(rng, 120_000, 500, nan=0.0)
    nul = (rng.random(len(ts)) < 0.04).astype(np.uint8)
    cq = _cq(_app(5, "<"))
    want = _push(OracleEngine(cq.program_json(), 0), ts, key, v, 30_011, nul)
    got = _push(_hip(cq, 500, 1 << 15), ts, key, v, 30_011, nul)
    assert compare(want, got) is None, compare(want, got)


@pytest.mark.gpu
def test_cseq_equals_general_lanes():
    """The same pushes through k_cseq and through the general NFA lanes (force_general=1)."""
    cq = program_for("3b")
    g = small_stream(3, 300_000, 3_000)
    a = _hip(cq, 3_000, 1 << 17, force=0)
    b = _hip(cq, 3_000, 1 << 17, force=1)
    assert a.path == 3 and b.path == 0
    ra, rb = per_key(run(a, cq, g, 77_777)), per_key(run(b, cq, g, 77_777))
    assert compare(ra, rb) is None, compare(ra, rb)


@pytest.mark.gpu
def test_cseq_wide_ts_span_reruns_with_16_byte_records():
    """A push whose ts span more than 2^31 ms (the 12-byte records' range): the engine re-runs it
    in the 16-byte form; the matches (ts included) equal the oracle's."""
    rng = np.random.default_rng(12)
    ts, key, v = _stream(rng, 60_000, 200)
    ts[30_000:] += 3 << 31  # a jump of ~200 days inside the first push
    cq = _cq(_app(5, "<"))
    want = _push(OracleEngine(cq.program_json(), 0), ts, key, v, 40_000)
    import os
    os.environ["SHP_CO_FULL_OFF"] = "1"  # (read at create) the sorted records, not the owner path
    try:
        eng = _hip(cq, 200, 1 << 16)
    finally:
        del os.environ["SHP_CO_FULL_OFF"]
    got = _push(eng, ts, key, v, 40_000)
    assert compare(want, got) is None, compare(want, got)
    assert eng.stat("cseq_wide_reruns") == 1  # the second push (20k events after the jump) is narrow
    assert sum(len(x) for x in want.values()) > 100
    own = _hip(cq, 200, 1 << 16)  # the owner path reads ts only per row: no re-run
    got = _push(own, ts, key, v, 40_000)
    assert compare(want, got) is None, compare(want, got)
    assert own.stat("cseq_wide_reruns") == 0
