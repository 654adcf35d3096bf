"""Capacity tiers of the general lanes, on the CPU (the lane code compiled for the host).

Each tier (nfa_lane.h LaneCaps: x1, x4, x16) holds exactly its list capacity of open partials
per key and matches the oracle there; one more fails that tier, which is what makes the engine
move to the next one (tests/test_capacity.py runs the growth itself on the GPU).
"""
import numpy as np
import pytest

from diff_util import compare, per_key
from hostcheck_engine import HostCheckEngine
from oracle.oracle import OracleEngine
from test_capacity import ABSENT, NEVER_CLOSES, _cq, _pending_stream, _push_all

LCAP = {0: 32, 1: 128, 2: 512}


@pytest.mark.parametrize("tier", [0, 1, 2])
def test_tier_holds_its_list_capacity(tier):
    cq = _cq(NEVER_CLOSES)
    ts, key, v = _pending_stream(2, LCAP[tier], 5)
    h = HostCheckEngine(cq.program_json(), 0, max_keys=2, tier=tier)
    o = OracleEngine(cq.program_json(), 0)
    for e in (h, o):
        _push_all(e, ts, key, v, 1 << 16)
    a, b = per_key(o.fetch()), per_key(h.fetch())
    assert compare(a, b) is None, compare(a, b)
    assert sum(len(x) for x in a.values()) == 2 * LCAP[tier]


@pytest.mark.parametrize("tier", [0, 1, 2])
def test_tier_overflows_one_past_capacity(tier):
    cq = _cq(NEVER_CLOSES)
    ts, key, v = _pending_stream(1, LCAP[tier] + 1, 6)
    h = HostCheckEngine(cq.program_json(), 0, max_keys=1, tier=tier)
    with pytest.raises(RuntimeError, match="lane error"):
        _push_all(h, ts, key, v, 1 << 16)


@pytest.mark.parametrize("tier", [1, 2])
def test_absent_timers_at_grown_tier(tier):
    """100 open absent partials of one key (100 queued timers, past tier 0's 64) fire as the oracle's."""
    cq = _cq(ABSENT)
    n1 = 100
    rng = np.random.default_rng(2)
    key = np.zeros(n1 + 1, np.int32)
    v = np.concatenate([rng.integers(1, 100, n1), [50]]).astype(np.float32)
    ts = np.concatenate([10_000 + 5 * np.arange(n1), [40_000]]).astype(np.int64)
    st = np.zeros(n1 + 1, np.int32)
    h = HostCheckEngine(cq.program_json(), 0, max_keys=1, tier=tier)
    o = OracleEngine(cq.program_json(), 0)
    for e in (h, o):
        _push_all(e, ts, key, v, 1 << 16, st, ncol=2)
    a, b = per_key(o.fetch()), per_key(h.fetch())
    assert compare(a, b) is None, compare(a, b)
    assert sum(len(x) for x in a.values()) == n1
