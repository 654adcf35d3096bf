"""SHP_LAYOUT_CHAIN32 on the count-sequence path (C3', round 4), against the oracle (GPU).

C3' (`every e1=S[f1]<1:M>, e2=S[f2(e1[last], e2)]`, CountPreStateProcessor.java:53-95,
CountPostStateProcessor.java:39-79) emits one 4-byte word per match: e2's batch index | L << 28,
its e1 chain being the L events of e2's key just before it (include/siddhi_hip.h).  Two producers:
the owner kernels (siddhi_amd/csrc/cseq_own.h: owner multisplit + per-owner LDS pass, the default
for CHAIN32) and k_cs3's emit over the sorted records (SHP_CO_OFF=1).  Both are checked
* through shp_fetch_matches, whose expansion (CseqState::expand) materialises FULL records, per key
  bit-exact against the oracle: key counts 1 .. 1M, every M / comparison / column type shape of
  tests/test_cseq.py, nulls, split pushes, snapshot / restore mid-stream;
* on the words themselves, read from HBM after shp_push_batch_device, against the reference rule
  restated in Python (tests/test_cseq.py::automaton): the set of (e2 index, L) per key, in order.
"""
import ctypes

import numpy as np
import pytest

from diff_util import compare, per_key, program_for, run, small_stream
from oracle.oracle import OracleEngine
from test_cseq import _app, _cq, _push, _stream, automaton

pytestmark = pytest.mark.gpu

PATHS = ["owner", "sort"]


@pytest.fixture(params=PATHS)
def path(request, monkeypatch):
    if request.param == "sort":
        monkeypatch.setenv("SHP_CO_OFF", "1")
    else:
        monkeypatch.delenv("SHP_CO_OFF", raising=False)
    return request.param


def _eng(cq, keys, batch, path, owner_ok=True):
    """owner_ok: the owner kernels take the shape (M <= 7: their 8-byte transition tables)."""
    from siddhi_amd.native import LAYOUT_CHAIN32, HipEngine
    e = HipEngine(cq.program_json(), 0, max_keys=keys, max_batch=batch, match_layout=LAYOUT_CHAIN32)
    assert e.path == 3
    assert e.stat("cseq_owner") == (1 if path == "owner" and owner_ok else 0)
    return e


@pytest.mark.parametrize("keys,n,batch", [(1, 30_000, 7_001), (64, 200_000, 65_537), (20_000, 600_000, 200_003),
                                          (1_000_000, 3_000_000, 1_000_003)],
                         ids=["1key", "64keys", "20k", "1M"])
def test_chain32_c3b_vs_oracle(keys, n, batch, path):
    cq = program_for("3b")
    g = small_stream(3, n, keys)
    want = per_key(run(OracleEngine(cq.program_json(), 0), cq, g))
    eng = _eng(cq, keys, batch, path)
    got = per_key(run(eng, cq, g, batch))
    assert compare(want, got) is None, compare(want, got)
    assert sum(len(x) for x in want.values()) > 1000


@pytest.mark.parametrize("M,op,typ", [(1, "<", "float"), (2, ">=", "float"), (3, "==", "int"), (5, "!=", "float"),
                                      (8, "<=", "int"), (5, ">", "int")])
def test_chain32_shapes_vs_oracle(M, op, typ, path):
    """Every M (the owner path's ring of M batch indices per key); M = 8 runs on the sorted records."""
    rng = np.random.default_rng(M * 7 + len(op))
    ts, key, v = _stream(rng, 150_000, 3_000)
    if typ == "int":
        v = np.nan_to_num(v, nan=17).astype(np.int32)
    cq = _cq(_app(M, op, typ))
    want = _push(OracleEngine(cq.program_json(), 0), ts, key, v, 40_009)
    got = _push(_eng(cq, 3_000, 1 << 16, path, owner_ok=M <= 7), ts, key, v, 40_009)
    assert compare(want, got) is None, compare(want, got)
    assert sum(len(x) for x in want.values()) > 100


def test_chain32_nulls_vs_oracle(path):
    rng = np.random.default_rng(4)
    ts, key, v = _stream(rng, 120_000, 500, nan=0.0)
    nul = (rng.random(len(ts)) < 0.04).astype(np.uint8)
    cq = _cq(_app(5, "<"))
    want = _push(OracleEngine(cq.program_json(), 0), ts, key, v, 30_011, nul)
    got = _push(_eng(cq, 500, 1 << 15, path), ts, key, v, 30_011, nul)
    assert compare(want, got) is None, compare(want, got)


def test_chain32_long_runs_cross_chunks_and_pushes(path):
    """Few keys (long key runs: a chunk of one key, chains crossing chunk and push boundaries) and a
    slowly rising value so chains fill to M and restart."""
    n, keys = 200_000, 3
    rng = np.random.default_rng(21)
    ts = np.arange(n, dtype=np.int64) * 2 + 5_000
    key = rng.integers(0, keys, n).astype(np.int32)
    v = (21.0 + (np.arange(n) % 37) * 0.5).astype(np.float32)
    v[rng.random(n) < 0.02] = 10.0
    cq = _cq(_app(5, "<"))
    want = _push(OracleEngine(cq.program_json(), 0), ts, key, v, 9_973)
    got = _push(_eng(cq, keys, 1 << 14, path), ts, key, v, 9_973)
    assert compare(want, got) is None, compare(want, got)
    assert sum(len(x) for x in want.values()) > 5_000


def test_chain32_snapshot_restore_continues_exactly(path):
    cq = program_for("3b")
    g = small_stream(3, 400_000, 5_000)
    want = per_key(run(OracleEngine(cq.program_json(), 0), cq, g))
    half = {k: x[:200_000] for k, x in g.items()}
    rest = {k: x[200_000:] for k, x in g.items()}
    a = _eng(cq, 5_000, 1 << 16, path)
    first = per_key(run(a, cq, half, 60_001))
    b = _eng(cq, 5_000, 1 << 16, path)
    b.restore(a.snapshot())
    second = per_key(run(b, cq, rest, 60_001))
    got = {k: first.get(k, []) + second.get(k, []) for k in set(first) | set(second)}
    assert compare(want, got) is None, compare(want, got)


def test_chain32_same_state_as_full_layout(path):
    """A CHAIN32 engine and a FULL one over the same pushes leave the same key state (snapshot)."""
    from siddhi_amd.native import HipEngine
    cq = program_for("3b")
    g = small_stream(3, 300_000, 2_000)
    a = _eng(cq, 2_000, 1 << 16, path)
    b = HipEngine(cq.program_json(), 0, max_keys=2_000, max_batch=1 << 16)
    ra, rb = per_key(run(a, cq, g, 50_021)), per_key(run(b, cq, g, 50_021))
    assert compare(ra, rb) is None
    assert a.snapshot() == b.snapshot()


def test_chain32_device_words_follow_the_rule(path):
    """The words in HBM after shp_push_batch_device: per key, the (e2 index, L) sequence of the rule
    restated in Python (the chain = the key's L events before e2), two pushes (chains crossing)."""
    import torch
    from siddhi_amd import native
    cq = program_for("3b")
    keys, n = 700, 120_000
    g = small_stream(3, n, keys)
    ts, key, v = g["ts"], g["key"].astype(np.int32), g["price"].astype(np.float32)
    want = automaton(5, "<", ts, key, v)
    eng = _eng(cq, keys, 1 << 16, path)
    L = native.lib()
    got = {}
    for lo in range(0, n, 60_000):
        hi = min(n, lo + 60_000)
        t_ts = torch.from_numpy(ts[lo:hi].copy()).cuda()
        t_key = torch.from_numpy(key[lo:hi].copy()).cuda()
        t_v = torch.from_numpy(v[lo:hi].copy()).cuda()
        colp = (ctypes.c_void_p * 1)(t_v.data_ptr())
        b = native.ShpBatch(hi - lo, t_ts.data_ptr(), t_key.data_ptr(), None, ctypes.cast(colp, ctypes.c_void_p),
                            None)
        mt = native.ShpMatches()
        assert L.shp_push_batch_device(eng.h, ctypes.byref(b), ctypes.byref(mt)) == 0
        assert mt.layout == native.LAYOUT_CHAIN32
        words = np.empty(mt.m, np.uint32)
        if mt.m:
            assert L.shp_dev_to_host(words.ctypes.data, mt.refs, words.nbytes) == 0
        gi = (words & ((1 << 28) - 1)).astype(np.int64) + lo
        ln = (words >> 28).astype(np.int64)
        for i, l in zip(gi, ln):
            got.setdefault(int(key[i]), []).append((int(i), int(l)))
    exp = {k: [(m[2], len(m[3][0])) for m in ms] for k, ms in want.items()}
    assert got == exp
    assert sum(len(x) for x in exp.values()) > 5_000


def test_chain32_rejected_off_the_count_sequence_path():
    from siddhi_amd.native import LAYOUT_CHAIN32, HipEngine, ShpError
    with pytest.raises(ShpError):
        HipEngine(program_for(2).program_json(), 0, max_keys=300, max_batch=1 << 16, match_layout=LAYOUT_CHAIN32)


def test_chain32_long_chains_with_a_small_match_buffer(path):
    """max_matches barely above the matches of a push, every match an M = 7 chain: the push commits
    and its expansion always fits (a CHAIN32 engine's ref capacity holds M + 1 refs per match), so
    shp_fetch_matches returns every record exactly (the expansion used to fail after the
    commit and lose the matches)."""
    from siddhi_amd.native import LAYOUT_CHAIN32, HipEngine
    app = _app(7, "<", "float")
    cq = _cq(app)
    n = 20_000
    # one key, values rising then one drop: chains of 7 close at every drop
    v = np.tile(np.array([30, 31, 32, 33, 34, 35, 36, 10], np.float32), n // 8)
    g = {"ts": np.arange(n, dtype=np.int64) + 1000, "key": np.zeros(n, np.int32), "stream": np.zeros(n, np.int32),
         "price": v}
    want = per_key(run(OracleEngine(cq.program_json(), 0), cq, g))
    m = sum(len(x) for x in want.values())
    assert m >= 2000 and all(len(r[3][0]) == 7 for x in want.values() for r in x)
    e = HipEngine(cq.program_json(), 0, max_keys=1, max_batch=n, max_matches=m + 16, match_layout=LAYOUT_CHAIN32)
    got = per_key(run(e, cq, g))
    assert compare(want, got) is None, compare(want, got)
    assert e.fetch()["key"].size == 0
