"""C3 at its configured key count (1M keys) on the HIP path, against the oracle.

* C3 as specified -- `from e1=S[v>20]<2:5>, e2=S[v<e1[last].v]`, a *sequence* whose Kleene count
  has min 2 -- emits no match in the reference: a count partial below minCount is not re-added to
  its own list (CountPostStateProcessor.java:49-57) and the sequence receiver resets the pending
  lists on every event (StreamPreStateProcessor.resetState :288-305 via
  SequenceMultiProcessStreamReceiver.java:45-50), so `<2:5>` never reaches 2 (SURVEY §0 finding 3).
  The count-sequence automaton (cseq.h, its "once, min >= 2" tables) and the general NFA lanes
  (HBM arena, one lane per key) must both reproduce that at 1M keys.
* C3' -- `every e1=S[v>20]<1:5>` -- at 1M keys on the general lanes (11 KB of HBM arena per key,
  two arenas) and on the count-sequence automaton (k_cseq), per key bit-exact against the oracle,
  over split pushes, with a few hot keys carrying long rising runs (chains that fill to max and
  restart) among the 1M (CountPreStateProcessor.java:53-95, CountPostStateProcessor.java:39-79).
"""
import numpy as np
import pytest

from diff_util import compare, per_key, program_for, run, small_stream
from oracle.oracle import OracleEngine

pytestmark = pytest.mark.gpu

KEYS = 1_000_000


def _hip(force_general, batch):
    from siddhi_amd.native import HipEngine

    def make(pj, start):
        return HipEngine(pj, start, max_keys=KEYS, max_batch=batch, force_general=force_general)
    return make


@pytest.mark.parametrize("force_general", [1, 0], ids=["lanes", "cseq"])
def test_c3_as_specified_at_1m_keys_emits_nothing(force_general):
    cq = program_for(3)
    g = small_stream(3, 3_000_000, KEYS)
    want = run(OracleEngine(cq.program_json(), 0), cq, g)
    eng = _hip(force_general, 1 << 20)(cq.program_json(), 0)
    assert eng.path == (0 if force_general == 1 else 3)
    got = run(eng, cq, g, 1_000_003)
    assert len(want["key"]) == 0
    assert len(got["key"]) == 0
    assert eng.stat("pushes") == 3


def _with_hot_keys(g, hot=(7, 123_457, 999_999), run_len=400, every=3):
    """Splice rising runs of a few keys into the stream (one hot event every `every` events):
    their count chains fill to max (5) and restart."""
    n = len(g["ts"])
    idx = np.arange(0, n, every)[: run_len * len(hot)]
    out = {k: v.copy() for k, v in g.items()}
    for j, i in enumerate(idx):
        k = hot[j % len(hot)]
        step = j // len(hot)
        out["key"][i] = k
        out["price"][i] = np.float32(21.0 + (step % 50) * 1.5)
    return out


@pytest.mark.parametrize("force_general", [1, 0], ids=["lanes", "cseq"])
def test_c3b_at_1m_keys_vs_oracle(force_general):
    cq = program_for("3b")
    g = _with_hot_keys(small_stream("3b", 4_000_000, KEYS))
    want = per_key(run(OracleEngine(cq.program_json(), 0), cq, g))
    eng = _hip(force_general, 1 << 21)(cq.program_json(), 0)
    assert eng.path == (0 if force_general == 1 else 3)
    got = per_key(run(eng, cq, g, 1_333_333))
    msg = compare(want, got)
    assert msg is None, msg
    assert sum(len(v) for v in want.values()) > 100_000
