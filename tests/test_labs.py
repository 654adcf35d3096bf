"""The logical-absent path (siddhi_amd/csrc/labs.h, the default for its shape), C4's shape:
`every (e1=S1[f] and e2=S2[f]) -> not S3[price > e1.price] for T within W` in playback.

CPU: the exact per-key rule for ANY timestamp order (tests/labs_exact.py ExactC4: the logical
partial, the absent state's pending / new-and-every lists, the key's Scheduler FIFO and
lastScheduledTime) against the oracle's object-level restatement of the Logical / AbsentStream
processors and the playback Scheduler (oracle/oracle.cpp) -- ordered C4 streams and streams whose
timestamps go back within keys and globally, keys lagging the clock, clock jumps -- on streams
with no cross-key scheduler tie (those are parity-unpinned); k_labs_w's ordered
formulation as formulas per pair (FastC4) against ExactC4, outputs AND state after every push; the
older ordered rule (`model`) and its block-at-a-time form (`wave_model`).  GPU (`-m gpu`): k_labs_w /
k_labs against the oracle, unordered streams through the default path (k_labs_w hands them to
k_labs), the two kernels' states equal after every push, split pushes, a clock advanced with no
event, snapshot/restore, the hand-back of keys with more than 64 waiting pairs.
"""
from collections import deque

import numpy as np
import pytest

from diff_util import compare, per_key, program_for, run, small_stream
from labs_exact import ExactC4, FastC4
from oracle.oracle import OracleEngine

W, WAIT = 10_000, 5_000


def model(ts, key, st, pr):
    """labs.h's rule over one playback stream (streams 0 = S1 (e1), 1 = S2 (e2), 2 = S3)."""
    out, S = {}, {}
    clock = 0
    for g in range(len(ts)):
        t, k, s, p = int(ts[g]), int(key[g]), int(st[g]), float(pr[g])
        clock = max(clock, t)
        for kk, stt in S.items():  # timers the clock reached, per key in completion order
            wq = stt["waits"]
            while wq and wq[0][0] <= clock:
                due, e1, e2 = wq.popleft()
                if abs(e1[1] - due) <= W and abs(e2[1] - due) <= W:
                    out.setdefault(kk, []).append((due, 0, g, ((e2[0],), (e1[0],), ())))
        stt = S.setdefault(k, {"pend": {"e1": None, "e2": None}, "waits": deque()})
        pend = stt["pend"]
        if any(ev is not None and abs(ev[1] - t) > W for ev in pend.values()):
            stt["pend"] = pend = {"e1": None, "e2": None}
        if s in (0, 1):
            slot, other = ("e1", "e2") if s == 0 else ("e2", "e1")
            if p > 20 and pend[slot] is None:
                pend[slot] = (g, t, p)
                if pend[other] is not None:
                    stt["waits"].append((t + WAIT, pend["e1"], pend["e2"]))
                    stt["pend"] = {"e1": None, "e2": None}
        elif s == 2:
            stt["waits"] = deque(w for w in stt["waits"] if not p > w[1][2])
    return out


def wave_model(ts, key, st, pr, block=64):
    """k_labs_w's formulation of the same rule (labs.h): per key, events taken `block` at a time;
    the partial jumps fill -> completion / reset with first-set-bit searches over the block, and
    each waiting pair fires at the first later event whose clock reaches its due time unless a Z
    event before that kills it.  Must equal `model` exactly."""
    n = len(ts)
    clock = np.maximum.accumulate(np.asarray(ts, np.int64))
    runs = {}
    for g in range(n):
        runs.setdefault(int(key[g]), []).append(g)
    out = {}
    for k, idx in runs.items():
        pend = {"e1": None, "e2": None}
        alive = []  # [due, e1, e2, c]
        lo = 0
        recs = out.setdefault(k, [])

        def settle(fires):
            nonlocal alive
            keep = []
            for w, (f, killed, flo, fhi) in zip(alive, fires):
                if f and not killed:
                    due, e1, e2, _ = w
                    if abs(e1[1] - due) <= W and abs(e2[1] - due) <= W:
                        g = next(x for x in range(flo, fhi + 1) if clock[x] >= due)
                        recs.append((due, 0, g, ((e2[0],), (e1[0],), ())))
                elif not f and not killed:
                    keep.append([w[0], w[1], w[2], -1])
            alive = keep

        for j0 in range(0, len(idx), block):
            blk = idx[j0:j0 + block]
            nv = len(blk)
            qx = [int(st[g]) == 0 and float(pr[g]) > 20 for g in blk]
            qy = [int(st[g]) == 1 and float(pr[g]) > 20 for g in blk]
            tsb = [int(ts[g]) for g in blk]
            p0 = 0
            if pend["e1"] is not None or pend["e2"] is not None:  # a half partial carried in
                slot, other, q_o = ("e1", "e2", qy) if pend["e1"] is not None else ("e2", "e1", qx)
                t0 = pend[slot][1]
                z = next((q for q in range(nv) if tsb[q] - t0 > W), 64)
                b = next((q for q in range(nv) if q_o[q]), 64)
                if b < z:
                    g = blk[b]
                    pend[other] = (g, tsb[b], float(pr[g]))
                    alive.append([tsb[b] + WAIT, pend["e1"], pend["e2"], b])
                    pend = {"e1": None, "e2": None}
                    p0 = b + 1
                elif z < 64:
                    pend = {"e1": None, "e2": None}
                    p0 = z
                else:
                    p0 = 64

            def step(p):  # from an empty partial at p: (kind, next, a, b)
                a = next((q for q in range(p, nv) if qx[q] or qy[q]), None)
                if a is None:
                    return 0, 64, None, None
                q_o = qy if qx[a] else qx
                b = next((q for q in range(a + 1, nv) if q_o[q]), None)
                if b is not None and tsb[b] - tsb[a] <= W:
                    return 1, b + 1, a, b
                z = next((q for q in range(a + 1, nv) if tsb[q] - tsb[a] > W), None)
                if z is not None:
                    return 2, z, a, b
                return 3, 64, a, b

            p = p0
            while p < nv:
                kind, nxt, a, b = step(p)
                if kind == 1:
                    ga, gb = blk[a], blk[b]
                    ea, eb = (ga, tsb[a], float(pr[ga])), (gb, tsb[b], float(pr[gb]))
                    e1, e2 = (ea, eb) if qx[a] else (eb, ea)
                    alive.append([tsb[b] + WAIT, e1, e2, b])
                    p = nxt
                elif kind == 2:
                    p = nxt
                else:
                    if kind == 3:
                        ga = blk[a]
                        pend["e1" if qx[a] else "e2"] = (ga, tsb[a], float(pr[ga]))
                    break
            fires = []
            for due, e1, e2, c in alive:
                f = next((q for q in range(c + 1, nv) if clock[blk[q]] >= due), None)
                end = nv if f is None else f
                killed = any(int(st[blk[q]]) == 2 and float(pr[blk[q]]) > e1[2] for q in range(c + 1, end))
                flo = (lo if f == 0 else blk[f - 1] + 1) if f is not None else 0
                fires.append((f is not None, killed, flo, blk[f] if f is not None else 0))
            settle(fires)
            lo = blk[-1] + 1
        settle([(due <= clock[n - 1], False, lo, n - 1) for due, *_ in alive])
        if not recs:
            del out[k]
    return out


def _oracle(cq, ts, key, st, pr, batch):
    e = OracleEngine(cq.program_json(), 0)
    for lo in range(0, len(ts), batch):
        hi = min(len(ts), lo + batch)
        e.push(ts[lo:hi], key[lo:hi], st[lo:hi], [pr[lo:hi]] * 3, [None] * 3)
    return per_key(e.fetch())


@pytest.mark.parametrize("keys,n", [(20, 100_000), (200, 200_000), (1000, 300_000)])
def test_model_matches_oracle_c4_stream(keys, n):
    cq = program_for(4)
    g = small_stream(4, n, keys)
    pr = g["price"].astype(np.float32)
    want = _oracle(cq, g["ts"], g["key"], g["stream"], pr, 65_537)
    got = model(g["ts"], g["key"], g["stream"], pr)
    assert compare(want, got) is None, compare(want, got)
    assert sum(len(x) for x in want.values()) > 0


@pytest.mark.parametrize("keys,step", [(2, 1), (5, 3), (20, 7), (100, 2)])
def test_model_matches_oracle_dense_random(keys, step):
    rng = np.random.default_rng(keys * 11 + step)
    n = 40_000
    ts = (np.arange(n) * step).astype(np.int64) + 1000
    key = rng.integers(0, keys, n).astype(np.int32)
    st = rng.integers(0, 3, n).astype(np.int32)
    pr = (rng.integers(0, 10000, n) / 100.0).astype(np.float32)
    want = _oracle(program_for(4), ts, key, st, pr, n)
    got = model(ts, key, st, pr)
    assert compare(want, got) is None, compare(want, got)
    assert sum(len(x) for x in want.values()) > 5


@pytest.mark.parametrize("block", [64, 5])
@pytest.mark.parametrize("keys,step", [(1, 400), (3, 2), (20, 7), (100, 1)])
def test_wave_formulation_matches_model(keys, step, block):
    """k_labs_w's block-at-a-time formulation (fills/completions/resets by first-set-bit searches,
    fire and kill per waiting pair) reproduces the event-by-event rule, at the kernel's 64-event
    blocks and at 5-event blocks (many block boundaries)."""
    rng = np.random.default_rng(keys * 7 + step + block)
    n = 20_000
    ts = (np.arange(n) * step).astype(np.int64) + 1000
    if keys > 1:  # runs of equal ts, and gaps beyond W (partials reset)
        ts = np.sort(ts - rng.integers(0, 3, n) + np.cumsum(rng.random(n) < 0.002) * 30_000)
    key = rng.integers(0, keys, n).astype(np.int32)
    st = rng.integers(0, 3, n).astype(np.int32)
    pr = (rng.integers(0, 10000, n) / 100.0).astype(np.float32)
    want = model(ts, key, st, pr)
    got = wave_model(ts, key, st, pr, block)
    assert compare(want, got) is None, compare(want, got)
    assert sum(len(x) for x in want.values()) > (0 if keys == 1 else 5)


def test_wave_formulation_c4_stream():
    g = small_stream(4, 60_000, 50)
    pr = g["price"].astype(np.float32)
    want = model(g["ts"], g["key"], g["stream"], pr)
    got = wave_model(g["ts"], g["key"], g["stream"], pr)
    assert compare(want, got) is None, compare(want, got)


# ---------------------------------------------------------------- GPU (k_labs)

def _hip(cq, keys, batch, **kw):
    from siddhi_amd.native import HipEngine
    return HipEngine(cq.program_json(), 0, max_keys=keys, max_batch=batch, force_general=4, **kw)


@pytest.mark.gpu
@pytest.mark.parametrize("keys,n,batch", [(1, 40_000, 9_973), (200, 300_000, 65_537), (1000, 600_000, 200_003)],
                         ids=["1key", "200keys", "1000keys"])
def test_c4_labs_vs_oracle(keys, n, batch):
    cq = program_for(4)
    g = small_stream(4, n, keys)
    want = per_key(run(OracleEngine(cq.program_json(), 0), cq, g, batch))
    eng = _hip(cq, keys, batch)
    assert eng.path == 4
    got = per_key(run(eng, cq, g, batch))
    assert compare(want, got) is None, compare(want, got)
    assert sum(len(x) for x in want.values()) > (0 if keys == 1 else 20)
    if keys > 1:  # k_labs_w ran every push (no key had more than 64 pairs waiting)
        assert eng.stat("labs_fallbacks") == 0


@pytest.mark.gpu
def test_c4_wave_kernel_equals_thread_kernel(monkeypatch):
    """k_labs_w (a wave per key) and k_labs (SHP_NO_LABS_W: a thread per key) write the same
    records on the C4 stream, split over pushes."""
    cq = program_for(4)
    g = small_stream(4, 400_000, 500)
    a = per_key(run(_hip(cq, 500, 65_537), cq, g, 65_537))
    monkeypatch.setenv("SHP_NO_LABS_W", "1")
    b = per_key(run(_hip(cq, 500, 65_537), cq, g, 65_537))
    assert compare(a, b) is None, compare(a, b)
    assert sum(len(x) for x in a.values()) > 100


@pytest.mark.gpu
def test_labs_pushes_missing_half_the_keys():
    """Pushes alternate between all keys and only the even keys: the odd keys' waiting pairs fire
    in pushes that hold none of their events (their record regions come from the key runs' would-be
    starts, k_key_bounds), exactly as the oracle."""
    cq = program_for(4)
    g = small_stream(4, 360_000, 200)
    keep = np.ones(len(g["ts"]), bool)
    blk = np.arange(len(g["ts"])) // 60_000  # odd blocks: ~30k events of even keys only
    keep[(blk % 2 == 1) & (g["key"] % 2 == 1)] = False
    g = {k: v[keep] for k, v in g.items()}
    want = per_key(run(OracleEngine(cq.program_json(), 0), cq, g, 25_000))
    eng = _hip(cq, 200, 25_000)
    got = per_key(run(eng, cq, g, 25_000))
    assert compare(want, got) is None, compare(want, got)
    assert eng.stat("labs_fallbacks") == 0


@pytest.mark.gpu
def test_labs_equals_general_lanes_and_advance():
    """Pushes, then a clock advanced with no event (shp_advance_clock fires the waiting pairs):
    the same records from k_labs and from the general lanes, and from the oracle."""
    cq = program_for(4)
    g = small_stream(4, 150_000, 300)
    end = int(g["ts"][-1]) + 60_000
    outs = []
    for mk in (lambda: OracleEngine(cq.program_json(), 0), lambda: _hip(cq, 300, 1 << 16),
               lambda: __import__("siddhi_amd.native", fromlist=["HipEngine"]).HipEngine(
                   cq.program_json(), 0, max_keys=300, max_batch=1 << 16, force_general=1)):
        e = mk()
        n = len(g["ts"])
        for lo in range(0, n, 50_000):
            hi = min(n, lo + 50_000)
            e.push(g["ts"][lo:hi], g["key"][lo:hi], g["stream"][lo:hi], [g["price"][lo:hi].astype(np.float32)] * 3,
                   [None] * 3)
        e.advance(end)
        outs.append(per_key(e.fetch()))
    assert compare(outs[0], outs[1]) is None, compare(outs[0], outs[1])
    assert compare(outs[0], outs[2]) is None, compare(outs[0], outs[2])


@pytest.mark.gpu
def test_labs_snapshot_restore_continues():
    cq = program_for(4)
    g = small_stream(4, 120_000, 200)
    want = per_key(run(OracleEngine(cq.program_json(), 0), cq, g))
    half = {k: v[:60_000] for k, v in g.items()}
    rest = {k: v[60_000:] for k, v in g.items()}
    a = _hip(cq, 200, 1 << 16)
    first = run(a, cq, half)
    blob = a.snapshot()
    assert "absent" in str(a.describe(blob))
    b = _hip(cq, 200, 1 << 16)
    b.restore(blob)
    second = run(b, cq, rest)
    from siddhi_amd.native import _concat
    got = per_key(_concat([first, second], None, a.S))
    assert compare(want, got) is None, compare(want, got)


@pytest.mark.gpu
def test_labs_unordered_push_runs_exact_and_keeps_going():
    """A push with a key going back in time: since round 6 k_labs_w runs that key's disordered blocks
    by the exact rule itself (no hand-back of the push to k_labs) and returns to its ordered
    formulation once the key's state is regular again; all against the oracle."""
    from siddhi_amd.native import _concat
    cq = program_for(4)
    g = small_stream(4, 30_000, 50)
    g["ts"] = g["ts"].copy()
    g["ts"][10_100] -= 5_000
    want = per_key(run(OracleEngine(cq.program_json(), 0), cq, g))
    eng = _hip(cq, 50, 1 << 15)
    outs = [run(eng, cq, {k: v[lo:lo + 10_000] for k, v in g.items()}) for lo in (0, 10_000, 20_000)]
    got = per_key(_concat(outs, None, eng.S))
    assert compare(want, got) is None, compare(want, got)
    assert eng.stat("labs_fallbacks") == 0


@pytest.mark.gpu
def test_labs_rings_grow_and_snapshot_carries_the_tier():
    """One key with dense events: hundreds of pairs wait on the absent state at once, beyond the
    16-entry LDS ring, so the engine moves to the HBM rings (256, 4096) and re-runs the push; a
    snapshot taken there restores into a fresh engine (tier 0) and continues exactly."""
    from siddhi_amd.native import _concat
    cq = program_for(4)
    g = small_stream(4, 80_000, 1)
    want = per_key(run(OracleEngine(cq.program_json(), 0), cq, g))
    a = _hip(cq, 1, 1 << 16)
    first = run(a, cq, {k: v[:40_000] for k, v in g.items()})
    blob = a.snapshot()
    b = _hip(cq, 1, 1 << 16)
    b.restore(blob)
    second = run(b, cq, {k: v[40_000:] for k, v in g.items()})
    got = per_key(_concat([first, second], None, a.S))
    assert compare(want, got) is None, compare(want, got)
    assert sum(len(x) for x in want.values()) > 0


@pytest.mark.gpu
def test_labs_hands_back_keys_with_many_waiting_pairs():
    """No Z event and a pair every 2 ms on one key: ~2500 pairs wait at once, beyond k_labs_w's
    64, so the pushes go to k_labs (and its rings grow to the 4096 tier); still exact."""
    cq = program_for(4)
    n = 30_000
    rng = np.random.default_rng(5)
    g = {"ts": np.arange(n, dtype=np.int64) + 10_000, "key": np.zeros(n, np.int32),
         "stream": rng.integers(0, 2, n).astype(np.int32),
         "price": (50 + rng.integers(0, 1000, n) / 100.0).astype(np.float32)}
    want = per_key(run(OracleEngine(cq.program_json(), 0), cq, g, 10_000))
    eng = _hip(cq, 1, 10_000)
    got = per_key(run(eng, cq, g, 10_000))
    assert compare(want, got) is None, compare(want, got)
    assert sum(len(x) for x in want.values()) > 5000
    assert eng.stat("labs_fallbacks") > 0


@pytest.mark.gpu
def test_labs_more_than_4096_waiting_pairs():
    """`for 20 sec`: a pair completes every ~2 ms on one key and none is killed, so ~10k pairs
    wait on the absent state at once -- past the 4096 ring -- and the rings grow to the 65536 tier
    (the reference's timer queue is unbounded).  Exact against the oracle."""
    from siddhi_amd import synth
    from siddhi_amd.query.compiler import compile_app
    app = synth.QUERIES[4].replace("for 5 sec within 10 sec", "for 20 sec within 30 sec")
    cq = compile_app(app)[1][0]
    n = 42_000
    rng = np.random.default_rng(9)
    g = {"ts": np.arange(n, dtype=np.int64) + 10_000, "key": np.zeros(n, np.int32),
         "stream": rng.integers(0, 2, n).astype(np.int32),
         "price": (50 + rng.integers(0, 1000, n) / 100.0).astype(np.float32)}
    want = per_key(run(OracleEngine(cq.program_json(), 0), cq, g, 21_000))
    eng = _hip(cq, 1, 21_000)
    got = per_key(run(eng, cq, g, 21_000))
    assert compare(want, got) is None, compare(want, got)
    assert sum(len(x) for x in want.values()) > 5_000
    assert eng.describe(eng.snapshot())["engine"]["tier"] >= 3


# ------------------------------------------------------------------ the exact rule (any order)

def unordered_c4(seed, n=30_000):
    """A C4-shaped playback stream whose timestamps misbehave in one of five ways."""
    rng = np.random.default_rng(seed)
    keys = [3, 10, 40, 5, 20, 8, 2, 60, 30, 12][seed % 10]
    ts = (np.arange(n) * int(rng.integers(1, 40))).astype(np.int64) + 100_000
    mode = seed % 5
    if mode == 0:
        ts = ts + rng.integers(-8000, 8000, n)                                 # local disorder
    elif mode == 1:
        ts = ts - (rng.random(n) < 0.05) * rng.integers(0, 30_000, n)          # occasional big decreases
    elif mode == 2:
        ts = ts + np.cumsum(rng.random(n) < 0.001) * 20_000                    # clock jumps beyond T
    elif mode == 3:
        ts = ts + (rng.integers(0, keys, n) % 3) * 7_000                       # keys lagging the clock
    else:
        ts = np.sort(ts - rng.integers(0, 3, n))                               # ordered, with ties
    key = rng.integers(0, keys, n).astype(np.int32)
    st = rng.integers(0, 3, n).astype(np.int32)
    pr = (rng.integers(0, 10000, n) / 100.0).astype(np.float32)
    return ts.astype(np.int64), key, st, pr


def _exact(ts, key, st, pr, batch):
    m = ExactC4()
    for lo in range(0, len(ts), batch):
        hi = min(len(ts), lo + batch)
        m.push(ts[lo:hi], key[lo:hi], st[lo:hi], pr[lo:hi])
    return m.fetch(), m


@pytest.mark.parametrize("seed", range(10))
def test_exact_rule_matches_oracle_any_order(seed):
    ts, key, st, pr = unordered_c4(seed)
    o = OracleEngine(program_for(4).program_json(), 0)
    for lo in range(0, len(ts), 7919):
        hi = min(len(ts), lo + 7919)
        o.push(ts[lo:hi], key[lo:hi], st[lo:hi], [pr[lo:hi]] * 3, [None] * 3)
    if o.timer_ties():
        pytest.skip("cross-key scheduler ties (TreeMultimap): parity-unpinned")
    want = per_key(o.fetch())
    got, m = _exact(ts, key, st, pr, 7919)
    assert compare(want, got) is None, compare(want, got)
    assert sum(len(x) for x in want.values()) > 10


def test_exact_rule_re_arms_and_jumps_occur():
    """The unordered streams exercise the re-arm entries and lastScheduledTime jumps that the
    ordered fast path never sees (the reason the state carries them)."""
    rearms = jumps = 0
    for seed in (0, 3, 5, 8):
        _, m = _exact(*unordered_c4(seed, 12_000), 4001)
        rearms += m.rearms
        jumps += m.jumps
    assert rearms > 0 and jumps > 0


@pytest.mark.parametrize("seed", range(24))
def test_fast_formulas_equal_exact_rule_state_and_output(seed):
    """FastC4 (k_labs_w's per-pair formulas) against ExactC4 on ordered streams: every key's state
    (partial, pending and new-and-every pairs, queue, lastScheduledTime) after every push, and the
    records; W / T / key counts / event spacing varied (T >= W included)."""
    rng = np.random.default_rng(100 + seed)
    n = 6000
    keys = int(rng.integers(1, 30))
    step = int(rng.integers(1, 600))
    Wv = int(rng.choice([3000, 6000, 10000, 20000]))
    Tv = int(rng.choice([2000, 5000, 8000]))
    ts = np.sort((np.arange(n) * step).astype(np.int64) + 10_000 - rng.integers(0, 3, n))
    key = rng.integers(0, keys, n).astype(np.int32)
    st = rng.integers(0, 3, n).astype(np.int32)
    pr = (rng.integers(0, 10000, n) / 100.0).astype(np.float32)
    a, b = ExactC4(W=Wv, T=Tv), FastC4(W=Wv, T=Tv)
    batch = int(rng.integers(100, 3000))
    for lo in range(0, n, batch):
        hi = min(n, lo + batch)
        a.push(ts[lo:hi], key[lo:hi], st[lo:hi], pr[lo:hi])
        b.push(ts[lo:hi], key[lo:hi], st[lo:hi], pr[lo:hi])
        for k in a.keys:
            assert a.keys[k].snapshot() == b.state(k), (lo, k)
    oa, ob = a.fetch(), b.fetch()
    assert compare(oa, ob) is None, compare(oa, ob)
    assert a.rearms == 0 and a.jumps == 0


# ---------------------------------------------------------------- GPU: any order, both kernels

@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(10))
def test_labs_default_path_any_order_vs_oracle(seed):
    """The default path of C4's shape (force_general = 0) is the logical-absent automaton; on the
    misbehaving streams k_labs_w runs the disordered blocks by the exact rule (clock steps beyond T
    still hand the push to k_labs), and the records equal the oracle's."""
    from siddhi_amd.native import HipEngine
    ts, key, st, pr = unordered_c4(seed)
    cq = program_for(4)
    o = OracleEngine(cq.program_json(), 0)
    e = HipEngine(cq.program_json(), 0, max_keys=64, max_batch=1 << 13)
    assert e.path == 4
    for lo in range(0, len(ts), 7919):
        hi = min(len(ts), lo + 7919)
        args = (ts[lo:hi], key[lo:hi], st[lo:hi], [pr[lo:hi]] * 3, [None] * 3)
        o.push(*args)
        e.push(*args)
    if o.timer_ties():
        # cross-key scheduler ties (TreeMultimap): parity with the reference is unpinned there (SURVEY
        # §8c); the labs engine must still equal the general lanes (force_general = 1), which model the
        # Scheduler the same way
        lanes = HipEngine(cq.program_json(), 0, max_keys=64, max_batch=1 << 13, force_general=1)
        assert lanes.path == 0
        for lo in range(0, len(ts), 7919):
            hi = min(len(ts), lo + 7919)
            lanes.push(ts[lo:hi], key[lo:hi], st[lo:hi], [pr[lo:hi]] * 3, [None] * 3)
        a, b = per_key(lanes.fetch()), per_key(e.fetch())
        assert compare(a, b) is None, compare(a, b)
        return
    want, got = per_key(o.fetch()), per_key(e.fetch())
    assert compare(want, got) is None, compare(want, got)
    if seed % 5 == 2:  # clock jumps beyond T: the push goes to k_labs
        assert e.stat("labs_fallbacks") > 0
    if seed % 5 == 0:  # local disorder: exact blocks inside k_labs_w, no hand-back
        assert e.stat("labs_fallbacks") == 0


@pytest.mark.gpu
@pytest.mark.parametrize("seed,keys", [(0, 7), (1, 30), (3, 12), (10, 200), (13, 1)])
def test_labs_exact_blocks_leave_the_thread_kernels_state(monkeypatch, seed, keys):
    """Disordered streams (events moved back past T, keys lagging the clock): k_labs_w's exact blocks
    and its return to the ordered formulation leave, after every push, the state k_labs leaves
    (SHP_NO_LABS_W) -- partial, pairs and their lists, Scheduler queue, lastScheduledTime -- and the
    same records, equal to the oracle's.  Segments (few keys) included: a cut may fall in an exact
    stretch."""
    from siddhi_amd.native import HipEngine
    ts, key, st, pr = unordered_c4(seed, 60_000)
    key = (key % keys).astype(np.int32)
    cq = program_for(4)
    o = OracleEngine(cq.program_json(), 0)
    a = HipEngine(cq.program_json(), 0, max_keys=max(keys, 8), max_batch=1 << 15)
    monkeypatch.setenv("SHP_NO_LABS_W", "1")
    b = HipEngine(cq.program_json(), 0, max_keys=max(keys, 8), max_batch=1 << 15)
    for lo in range(0, len(ts), 15_013):
        hi = min(len(ts), lo + 15_013)
        args = (ts[lo:hi], key[lo:hi], st[lo:hi], [pr[lo:hi]] * 3, [None] * 3)
        o.push(*args)
        a.push(*args)
        b.push(*args)
        assert a.describe(a.snapshot())["keys"] == b.describe(b.snapshot())["keys"], lo
    ga, gb = per_key(a.fetch()), per_key(b.fetch())
    assert compare(gb, ga) is None, compare(gb, ga)
    if not o.timer_ties():
        want = per_key(o.fetch())
        assert compare(want, ga) is None, compare(want, ga)


@pytest.mark.gpu
@pytest.mark.parametrize("keys,step", [(50, 1), (7, 300), (1, 900)])
def test_labs_wave_and_thread_kernels_leave_the_same_state(monkeypatch, keys, step):
    """k_labs_w's state (pairs and their list, the Scheduler queue, lastScheduledTime) equals
    k_labs's after every push of an ordered stream (SHP_NO_LABS_W: k_labs only)."""
    from siddhi_amd.native import HipEngine
    cq = program_for(4)
    g = small_stream(4, 60_000, keys)
    g["ts"] = (synth_t0() + np.arange(len(g["ts"])) * step).astype(np.int64)
    a = HipEngine(cq.program_json(), 0, max_keys=keys, max_batch=1 << 14)
    monkeypatch.setenv("SHP_NO_LABS_W", "1")
    b = HipEngine(cq.program_json(), 0, max_keys=keys, max_batch=1 << 14)
    cols = [g["price"].astype(np.float32)] * 3
    n = len(g["ts"])
    for lo in range(0, n, 9_001):
        hi = min(n, lo + 9_001)
        args = (g["ts"][lo:hi], g["key"][lo:hi], g["stream"][lo:hi], [c[lo:hi] for c in cols], [None] * 3)
        a.push(*args)
        b.push(*args)
        da, db = a.describe(a.snapshot()), b.describe(b.snapshot())
        assert da["keys"] == db["keys"], lo
    assert compare(per_key(a.fetch()), per_key(b.fetch())) is None
    assert a.stat("labs_fallbacks") == 0


def synth_t0():
    from siddhi_amd import synth
    return synth.T0


@pytest.mark.gpu
@pytest.mark.parametrize("step,warm", [(300, None), (40, None), (300, "0")], ids=["sparse", "denser", "no-warmup"])
def test_labs_segments_vs_oracle_and_unsegmented_state(monkeypatch, step, warm):
    """Few keys with long runs: k_labs_w cuts each key's events into segments (a wave each, the later
    ones warmed up from the empty state over the 256 events before their cut).  Sparse keys (a key
    event every 1.2 s) and denser ones (every 160 ms) converge at every cut; without a warm-up
    (SHP_LABS_WARM=0) the later segments start empty, the cut check sees the difference and the push
    re-runs unsegmented.  Either way the records equal the oracle's and the state after every push
    equals an unsegmented engine's (SHP_LABS_NOSEG)."""
    from siddhi_amd.native import HipEngine
    cq = program_for(4)
    g = small_stream(4, 200_000, 4)
    g["ts"] = (synth_t0() + np.arange(len(g["ts"])) * step).astype(np.int64)
    want = per_key(run(OracleEngine(cq.program_json(), 0), cq, g, 100_003))
    if warm is not None:
        monkeypatch.setenv("SHP_LABS_WARM", warm)
    a = HipEngine(cq.program_json(), 0, max_keys=4, max_batch=1 << 17)
    monkeypatch.delenv("SHP_LABS_WARM", raising=False)
    monkeypatch.setenv("SHP_LABS_NOSEG", "1")
    b = HipEngine(cq.program_json(), 0, max_keys=4, max_batch=1 << 17)
    cols = [g["price"].astype(np.float32)] * 3
    n, ga, gb = len(g["ts"]), [], []
    for lo in range(0, n, 100_003):
        hi = min(n, lo + 100_003)
        args = (g["ts"][lo:hi], g["key"][lo:hi], g["stream"][lo:hi], [c[lo:hi] for c in cols], [None] * 3)
        a.push(*args)
        b.push(*args)
        ga.append(a.fetch())
        gb.append(b.fetch())
        assert a.describe(a.snapshot())["keys"] == b.describe(b.snapshot())["keys"], lo
    ra = {}
    for m in ga:
        for k, v in per_key(m).items():
            ra.setdefault(k, []).extend(v)
    assert compare(want, ra) is None, compare(want, ra)
    assert sum(len(x) for x in want.values()) > 50
    assert a.stat("labs_fallbacks") == 0
    assert (a.stat("labs_segmiss") > 0) == (warm is not None)


def _sawtooth_c4(seed, n=200_000):
    """C4-shaped stream over many 16384-event multisplit segments whose clock steps back at segment
    boundaries (each segment starts below the previous one's maximum), plus the local disorder of
    unordered_c4's mode: the fused clock's carried-in value is what orders those events."""
    rng = np.random.default_rng(500 + seed)
    keys = [7, 40, 200][seed % 3]
    ts = (np.arange(n) * 3).astype(np.int64) + 1_000_000
    seg = np.arange(n) // 16384
    ts = ts - (seg % 2) * int(rng.integers(1000, 60_000))  # odd segments start below the last clock
    if seed % 2:
        ts = ts + rng.integers(-500, 500, n)
    key = rng.integers(0, keys, n).astype(np.int32)
    st = rng.integers(0, 3, n).astype(np.int32)
    pr = (rng.integers(0, 10000, n) / 100.0).astype(np.float32)
    return ts, key, st, pr


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("batch", [70_001, 1 << 16])
def test_labs_fused_clock_across_segments(seed, batch, monkeypatch):
    """The multisplit's fused clock (k_la_ms_count<true> segment-local scan, k_la_seg_clock, the
    scatter's carried-in fix-up) over pushes of several 16384-event segments whose clock steps back
    at the boundaries: records equal the device-wide scan's (SHP_LABS_SCAN_CLOCK=1) and the oracle's."""
    from siddhi_amd.native import HipEngine
    ts, key, st, pr = _sawtooth_c4(seed)
    cq = program_for(4)

    def drive(env):
        if env:
            monkeypatch.setenv("SHP_LABS_SCAN_CLOCK", "1")
        else:
            monkeypatch.delenv("SHP_LABS_SCAN_CLOCK", raising=False)
        e = HipEngine(cq.program_json(), 0, max_keys=256, max_batch=1 << 17)
        assert e.path == 4
        for lo in range(0, len(ts), batch):
            hi = min(len(ts), lo + batch)
            e.push(ts[lo:hi], key[lo:hi], st[lo:hi], [pr[lo:hi]] * 3, [None] * 3)
        return per_key(e.fetch())
    fused, scanned = drive(False), drive(True)
    assert compare(scanned, fused) is None, compare(scanned, fused)
    o = OracleEngine(cq.program_json(), 0)
    for lo in range(0, len(ts), batch):
        hi = min(len(ts), lo + batch)
        o.push(ts[lo:hi], key[lo:hi], st[lo:hi], [pr[lo:hi]] * 3, [None] * 3)
    if not o.timer_ties():
        want = per_key(o.fetch())
        assert compare(want, fused) is None, compare(want, fused)
    assert sum(len(x) for x in fused.values()) > 100
