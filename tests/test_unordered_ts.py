"""Timestamps that decrease within a key (out-of-order input) on the 2-state `every e1 -> e2
within W` shape.

The reference accepts any timestamps: StreamPreStateProcessor.expireEvents (:326-361) expires
the pending list from its head while |ts - now| > within and stops at the first live partial,
and processAndReturn (:364-403) tries every pending partial with no expiry test, so with
decreasing timestamps expired partials can stay behind a live one and still match.  The sweep
and the scan kernels replay such keys exactly (sw_seq_key / fast_seq_item) instead of failing.

CPU: the scan kernels' item bodies (host build) and the general lanes (host build) against the
oracle.  GPU (`-m gpu`): the sweep, the scan kernels and the lanes through libsiddhi_hip.so.
"""
import numpy as np
import pytest

from diff_util import compare, per_key, program_for
from hostcheck_engine import FastHostEngine, HostCheckEngine
from oracle.oracle import OracleEngine


def unordered_stream(n, keys, seed, jitter=1500, frac=0.2):
    """A C2-like stream whose timestamps jump back by up to `jitter` ms for a fraction of events."""
    rng = np.random.default_rng(seed)
    ts = 1_000_000 + np.arange(n, dtype=np.int64) * 7
    back = rng.random(n) < frac
    ts[back] -= rng.integers(1, jitter, back.sum())
    key = rng.integers(0, keys, n).astype(np.int32)
    price = (rng.integers(0, 10000, n) / 100.0).astype(np.float32)
    return ts, key, np.zeros(n, np.int32), price


def _run(eng, ts, key, st, price, batch):
    for lo in range(0, len(ts), batch):
        hi = min(len(ts), lo + batch)
        eng.push(ts[lo:hi], key[lo:hi], st[lo:hi], [price[lo:hi]], [None])
    return per_key(eng.fetch())


CASES = [(64, 1500, 0.2), (4, 3000, 0.5), (300, 900, 0.05), (16, 10, 0.3)]


@pytest.mark.parametrize("keys,jitter,frac", CASES)
@pytest.mark.parametrize("batch", [40_000, 6_151])
def test_scan_bodies_replay_unordered_keys_exactly(keys, jitter, frac, batch):
    cq = program_for(2)
    ts, key, st, price = unordered_stream(40_000, keys, seed=keys + jitter, jitter=jitter, frac=frac)
    want = _run(OracleEngine(cq.program_json(), 0), ts, key, st, price, batch)
    got = _run(FastHostEngine(cq.program_json(), max_keys=keys, max_batch=1 << 16), ts, key, st, price, batch)
    assert compare(want, got) is None, compare(want, got)
    assert sum(len(v) for v in want.values()) > 1000


@pytest.mark.parametrize("batch", [40_000, 6_151])
def test_lane_bodies_unordered_keys(batch):
    cq = program_for(2)
    ts, key, st, price = unordered_stream(40_000, 64, seed=3)
    want = _run(OracleEngine(cq.program_json(), 0), ts, key, st, price, batch)
    got = _run(HostCheckEngine(cq.program_json(), 0, max_keys=64), ts, key, st, price, batch)
    assert compare(want, got) is None, compare(want, got)


@pytest.mark.gpu
@pytest.mark.parametrize("force,keys", [(3, 4), (3, 300), (3, 2000), (2, 64), (1, 64), (0, 300), (0, 16)],
                         ids=["sweep-4", "sweep-300", "sweep-2000", "scan-64", "lanes-64", "default-300",
                              "default-16"])
@pytest.mark.parametrize("jitter,frac", [(1500, 0.2), (10, 0.5), (200_000, 0.01)])
def test_engine_replays_unordered_keys_exactly(force, keys, jitter, frac):
    from siddhi_amd.native import HipEngine
    cq = program_for(2)
    ts, key, st, price = unordered_stream(60_000, keys, seed=keys * 7 + force, jitter=jitter, frac=frac)
    want = _run(OracleEngine(cq.program_json(), 0), ts, key, st, price, 9_973)
    eng = HipEngine(cq.program_json(), 0, max_keys=keys, max_batch=1 << 14, force_general=force)
    got = _run(eng, ts, key, st, price, 9_973)
    assert compare(want, got) is None, compare(want, got)
    assert sum(len(v) for v in want.values()) > 1000


@pytest.mark.gpu
def test_sweep_timestamps_beyond_the_chunk_span():
    """Sparse keys whose consecutive events lie days apart (beyond the sweep's 2^29 ms chunk
    span) and a `within` of 5 days: replayed exactly, not refused."""
    from siddhi_amd.native import HipEngine
    from siddhi_amd.query.compiler import compile_app
    app = ("define stream S (k string, v float); partition with (k of S) begin @info(name='q') "
           "from every e1=S[v > 20] -> e2=S[v > e1.v] within 5 days select e1.v as a, e2.v as b "
           "insert into Out; end;")
    cq = compile_app(app)[1][0]
    rng = np.random.default_rng(11)
    n, keys = 30_000, 300
    ts = 1_000_000 + np.cumsum(rng.integers(0, 60_000_000, n)).astype(np.int64)  # up to ~17 h apart
    key = rng.integers(0, keys, n).astype(np.int32)
    price = (rng.integers(0, 10000, n) / 100.0).astype(np.float32)
    st = np.zeros(n, np.int32)
    want = _run(OracleEngine(cq.program_json(), 0), ts, key, st, price, 7_001)
    eng = HipEngine(cq.program_json(), 0, max_keys=keys, max_batch=1 << 14, force_general=3)
    assert eng.path == 2
    got = _run(eng, ts, key, st, price, 7_001)
    assert compare(want, got) is None, compare(want, got)
    assert sum(len(v) for v in want.values()) > 100
