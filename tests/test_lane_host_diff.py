"""CPU check of the lane interpreter (host-compiled nfa_lane.h) against the oracle on synthetic streams.

These exercise the same per-key semantics the GPU lanes run (tests/hostcheck/); the GPU
itself is exercised by tests/test_gpu_parity.py.
"""
import pytest

from diff_util import compare, per_key, program_for, run, small_stream
from hostcheck_engine import HostCheckEngine
from oracle.oracle import OracleEngine

CASES = [
    ("c1", 1, dict(n=20000)),
    ("c2", 2, dict(n=30000, keys=64)),
    ("c3", 3, dict(n=30000, keys=64)),
    ("c3b", "3b", dict(n=30000, keys=64)),
    ("c4", 4, dict(n=60000, keys=200)),
    ("c5", 5, dict(n=30000, keys=64)),
]


@pytest.mark.parametrize("name,q,kw", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("batch", [None, 7777])
def test_lane_matches_oracle(name, q, kw, batch):
    cq = program_for(q)
    g = small_stream(q, kw["n"], kw.get("keys"))
    start = 0
    a = per_key(run(OracleEngine(cq.program_json(), start), cq, g))
    b = per_key(run(HostCheckEngine(cq.program_json(), start, max_keys=kw.get("keys", 1)), cq, g, batch))
    msg = compare(a, b)
    assert msg is None, msg
    if q != 3:
        assert sum(len(v) for v in a.values()) > 0
