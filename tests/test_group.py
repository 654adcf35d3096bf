"""Multi-GPU behind the C-ABI (shp_group_*): the library splits each rank's slice by key owner,
exchanges it and runs every rank's engine.  On the one-GPU box every rank of
an in-process group sits on cuda:0 (device-to-device copies stand in for RCCL; the split, the
counts, the global clock / sequence columns and the per-rank engines are the same code).

Parity: the union of the ranks' matches equals the single-process oracle run per key, bit-exact
(global key ids and global event sequence numbers).  For absent-state timers (C4) the emission
position of a timer match is the rank's next event rather than the global one, so `pos` is left
out of that comparison (include/siddhi_hip.h, group.hip header)."""
import numpy as np
import pytest

from diff_util import columns_for, compare, per_key, program_for, run, small_stream
from oracle.oracle import OracleEngine

pytestmark = pytest.mark.gpu


def _slices(g, cols, lo, hi, world, with_stream):
    import torch
    out = []
    for r in range(world):
        a = lo + r * (hi - lo) // world
        b = lo + (r + 1) * (hi - lo) // world
        t = lambda x: torch.from_numpy(np.ascontiguousarray(x[a:b])).to("cuda:0")  # noqa: E731
        out.append((t(g["ts"]), t(g["key"]), t(g["stream"]) if with_stream else None, [t(c) for c in cols]))
    return out


def _run_group(cq, g, world, keys, pushes, layout, max_batch=1 << 18, **kw):
    import torch
    from siddhi_amd.native import HipGroup
    grp = HipGroup(cq.program_json(), 0, max_keys=keys, max_batch=max_batch, max_matches=max_batch,
                   devices=[0] * world, match_layout=layout, **kw)
    cols = columns_for(cq, g)
    n = len(g["ts"])
    bounds = np.linspace(0, n, pushes + 1).astype(np.int64)
    parts = []
    for p in range(pushes):
        grp.push_device(_slices(g, cols, bounds[p], bounds[p + 1], world, len(cq.program["streams"]) > 1))
        parts.append(grp.fetch())
        torch.cuda.synchronize()
    grp.close()
    return parts


def _concat(parts):
    return {k: np.concatenate([p[k] for p in parts]) for k in parts[0]}


def _drop_pos(pk):
    return {k: [(t, ty, sl) for (t, ty, _, sl) in v] for k, v in pk.items()}


@pytest.mark.parametrize("world,keys", [(2, 600), (3, 900), (4, 64)])
def test_group_c2_matches_single_process(world, keys):
    """C2 through an in-process group (sweep per rank at >= 256 keys per rank, scan kernels below)."""
    from siddhi_amd.native import LAYOUT_FULL
    cq = program_for(2)
    g = small_stream(2, 150_000, keys)
    want = per_key(run(OracleEngine(cq.program_json(), 0), cq, g))
    got = per_key(_concat(_run_group(cq, g, world, keys, 3, LAYOUT_FULL)))
    assert compare(want, got) is None, compare(want, got)
    assert sum(len(v) for v in want.values()) > 10_000


@pytest.mark.parametrize("world", [2, 3])
def test_group_c4_absent_timers_with_global_clock(world):
    """C4 (logical + absent, playback timers) sharded: every rank gets the global playback clock
    column, so its timers fire as in one process."""
    from siddhi_amd.native import LAYOUT_FULL
    cq = program_for(4)
    keys = 200
    g = small_stream(4, 120_000, keys)
    want = _drop_pos(per_key(run(OracleEngine(cq.program_json(), 0), cq, g)))
    got = _drop_pos(per_key(_concat(_run_group(cq, g, world, keys, 4, LAYOUT_FULL))))
    assert compare(want, got) is None, compare(want, got)
    assert sum(len(v) for v in want.values()) > 1000


def test_group_c3b_count_lanes():
    from siddhi_amd.native import LAYOUT_FULL
    cq = program_for("3b")
    keys = 2000
    g = small_stream(3, 100_000, keys)
    want = per_key(run(OracleEngine(cq.program_json(), 0), cq, g))
    got = per_key(_concat(_run_group(cq, g, 2, keys, 2, LAYOUT_FULL)))
    assert compare(want, got) is None, compare(want, got)
    assert sum(len(v) for v in want.values()) > 1000


def test_group_c5_device_aggregate():
    """C5's running avg on the device (SHP_LAYOUT_AGG) per rank: per key the same values as the
    reference arithmetic over the single-process matches."""
    from siddhi_amd.native import LAYOUT_AGG
    from test_gpu_parity import _expected_agg
    cq = program_for(5)
    keys = 1200
    g = small_stream(5, 200_000, keys)
    want = _expected_agg(run(OracleEngine(cq.program_json(), 0), cq, g), columns_for(cq, g)[0], "avg")
    parts = _run_group(cq, g, 2, keys, 2, LAYOUT_AGG)
    got = {}
    for p in parts:
        for k, v in zip(p["key"], p["agg"]):
            got.setdefault(int(k), []).append(float(v))
    assert set(got) == set(want)
    for k in want:
        np.testing.assert_allclose(got[k], want[k], rtol=1e-9, atol=0)


def test_group_rank_overflow_is_refused():
    """A rank that would receive more than max_batch events fails the push before any engine runs."""
    from siddhi_amd.native import LAYOUT_FULL, ShpError
    cq = program_for(2)
    g = small_stream(2, 40_000, 600)
    g["key"] = (g["key"] // 2) * 2  # every key even: all events to rank 0
    with pytest.raises(ShpError, match="SHP_ERR_CAPACITY"):
        _run_group(cq, g, 2, 600, 1, LAYOUT_FULL, max_batch=30_000)


@pytest.mark.parametrize("q,keys", [(2, 600), (4, 200)], ids=["c2", "c4"])
def test_group_member_rccl_one_rank(q, keys):
    """The per-process member (shp_group_create_rank) with a one-rank RCCL communicator: the
    count all-gather and the grouped ncclSend / ncclRecv (to itself) run as they do across
    processes on an 8-GPU node."""
    import torch
    from siddhi_amd.native import LAYOUT_FULL, HipGroup, comm_id
    cq = program_for(q)
    g = small_stream(q, 80_000, keys)
    want = per_key(run(OracleEngine(cq.program_json(), 0), cq, g))
    grp = HipGroup(cq.program_json(), 0, max_keys=keys, max_batch=1 << 17, max_matches=1 << 17, world=1, rank=0,
                   comm=comm_id(), device=0, match_layout=LAYOUT_FULL)
    cols = columns_for(cq, g)
    parts = []
    for lo, hi in ((0, 30_000), (30_000, 80_000)):
        grp.push_device(_slices(g, cols, lo, hi, 1, len(cq.program["streams"]) > 1))
        parts.append(grp.fetch())
        torch.cuda.synchronize()
    grp.close()
    got = per_key(_concat(parts))
    if q == 4:
        want, got = _drop_pos(want), _drop_pos(got)
    assert compare(want, got) is None, compare(want, got)
    assert sum(len(v) for v in want.values()) > 1000


def test_group_null_values_travel_with_their_events():
    """Null values on the sharded path: each rank's slice may carry null bytes for a column (here
    only the odd ranks' slices do); the group exchanges them with the events, so a null price
    compares as null (CompareConditionExpressionExecutor: a null operand is false) exactly as in
    one engine."""
    import torch
    from siddhi_amd.native import LAYOUT_FULL, HipGroup
    cq = program_for(2)
    keys, world = 600, 3
    g = small_stream(2, 90_000, keys)
    rng = np.random.default_rng(4)
    nul = (rng.random(len(g["ts"])) < 0.2).astype(np.uint8)
    bounds = [r * len(nul) // world for r in range(world + 1)]
    for r in range(0, world, 2):  # even ranks' slices carry no null array
        nul[bounds[r]:bounds[r + 1]] = 0
    cols = columns_for(cq, g)
    ora = OracleEngine(cq.program_json(), 0)
    ora.push(g["ts"], g["key"], g["stream"], cols, [nul])
    want = per_key(ora.fetch())
    grp = HipGroup(cq.program_json(), 0, max_keys=keys, max_batch=1 << 17, max_matches=1 << 17,
                   devices=[0] * world, match_layout=LAYOUT_FULL)
    sl = []
    for r in range(world):
        a, b = bounds[r], bounds[r + 1]
        t = lambda x: torch.from_numpy(np.ascontiguousarray(x[a:b])).to("cuda:0")  # noqa: E731
        sl.append((t(g["ts"]), t(g["key"]), None, [t(c) for c in cols], [t(nul)] if r % 2 else None))
    grp.push_device(sl)
    got = per_key(grp.fetch())
    torch.cuda.synchronize()
    grp.close()
    assert compare(want, got) is None, compare(want, got)
    assert sum(len(v) for v in want.values()) > 5_000


@pytest.mark.parametrize("world,cfg,root", [(2, 2, 0), (3, 2, 1), (3, 4, 2), (2, 5, 1)], ids=["c2w2", "c2w3", "c4w3", "c5w2"])
def test_group_gather_to_root_matches_oracle(world, cfg, root):
    """shp_group_gather_matches: every rank's records move to the root in HBM (device copies here,
    RCCL send / recv between processes), with global key ids, S-stride slots and the refs in record
    order; per key they equal the oracle's (C4: timer matches compared without pos, as above)."""
    import torch
    from siddhi_amd.native import LAYOUT_AGG, LAYOUT_FULL, HipGroup
    cq = program_for(cfg)
    keys = {2: 600, 4: 200, 5: 1000}[cfg]
    g = small_stream(cfg, 90_000, keys)
    layout = LAYOUT_AGG if cfg == 5 else LAYOUT_FULL
    grp = HipGroup(cq.program_json(), 0, max_keys=keys, max_batch=1 << 17, max_matches=1 << 17,
                   devices=[0] * world, match_layout=layout)
    cols = columns_for(cq, g)
    parts = []
    bounds = np.linspace(0, len(g["ts"]), 4).astype(np.int64)
    for p in range(3):
        grp.push_device(_slices(g, cols, bounds[p], bounds[p + 1], world, len(cq.program["streams"]) > 1))
        parts.append(grp.gather(root))
        torch.cuda.synchronize()
    grp.close()
    got = _concat(parts)
    ora = run(OracleEngine(cq.program_json(), 0), cq, g)
    if cfg == 5:
        from test_gpu_parity import _expected_agg
        want = _expected_agg(ora, cols[0], "avg")
        rows = {}
        for k, v in zip(got["key"], got["agg"]):
            rows.setdefault(int(k), []).append(float(v))
        assert set(rows) == set(want)
        for k in want:
            np.testing.assert_allclose(rows[k], want[k], rtol=1e-9, atol=0)
        return
    want, have = per_key(ora), per_key(got)
    if cfg == 4:
        want, have = _drop_pos(want), _drop_pos(have)
    assert compare(want, have) is None, compare(want, have)
    assert sum(len(v) for v in want.values()) > 500


@pytest.mark.parametrize("cfg,keys,n", [(2, 4000, 240_000), (3, 4000, 160_000), ("3b", 4000, 160_000),
                                        (4, 400, 160_000), (5, 4000, 240_000)],
                         ids=["c2", "c3", "c3b", "c4", "c5"])
def test_group_world8(cfg, keys, n):
    """Every config at the configured world size: an in-process group of 8 ranks (all on cuda:0;
    device copies stand in for RCCL), three pushes, against the single-process oracle per key
    (C5: the device running avg within 1e-9 relative; C4: timer matches without pos; C3 as
    specified matches nothing -- SURVEY §0 finding 3 -- on one engine and on eight)."""
    from siddhi_amd.native import LAYOUT_AGG, LAYOUT_FULL
    cq = program_for(cfg)
    g = small_stream(3 if cfg == "3b" else cfg, n, keys)
    ora = run(OracleEngine(cq.program_json(), 0), cq, g)
    if cfg == 5:
        from test_gpu_parity import _expected_agg
        want = _expected_agg(ora, columns_for(cq, g)[0], "avg")
        parts = _run_group(cq, g, 8, keys, 3, LAYOUT_AGG)
        got = {}
        for p in parts:
            for k, v in zip(p["key"], p["agg"]):
                got.setdefault(int(k), []).append(float(v))
        assert set(got) == set(want)
        for k in want:
            np.testing.assert_allclose(got[k], want[k], rtol=1e-9, atol=0)
        return
    want = per_key(ora)
    got = per_key(_concat(_run_group(cq, g, 8, keys, 3, LAYOUT_FULL)))
    if cfg == 4:
        want, got = _drop_pos(want), _drop_pos(got)
    assert compare(want, got) is None, compare(want, got)
    if cfg != 3:
        assert sum(len(v) for v in want.values()) > 1000


@pytest.mark.parametrize("gather", [False, True], ids=["fetch", "gather"])
def test_group_world8_c3b_chain32(gather):
    """C3' with SHP_LAYOUT_CHAIN32 at world 8: every rank on the count-sequence owner kernels over its
    dense local keys with global sequence numbers; the words expand to FULL on fetch / on the
    gather to the root, per key equal to the single-process oracle."""
    import torch
    from siddhi_amd.native import LAYOUT_CHAIN32, HipGroup
    cq = program_for("3b")
    keys, n = 8000, 240_000
    g = small_stream(3, n, keys)
    grp = HipGroup(cq.program_json(), 0, max_keys=keys, max_batch=1 << 17, max_matches=1 << 17,
                   devices=[0] * 8, match_layout=LAYOUT_CHAIN32)
    for r in range(8):
        assert grp.engine_stat(r, "cseq_owner") == 1
    cols = columns_for(cq, g)
    parts = []
    bounds = np.linspace(0, n, 4).astype(np.int64)
    for p in range(3):
        grp.push_device(_slices(g, cols, bounds[p], bounds[p + 1], 8, False))
        parts.append(grp.gather(3) if gather else grp.fetch())
        torch.cuda.synchronize()
    grp.close()
    want, have = per_key(run(OracleEngine(cq.program_json(), 0), cq, g)), per_key(_concat(parts))
    assert compare(want, have) is None, compare(want, have)
    assert sum(len(v) for v in want.values()) > 5_000


@pytest.mark.parametrize("cfg,root", [(2, 5), (4, 7)], ids=["c2", "c4"])
def test_group_world8_gather_to_root(cfg, root):
    """shp_group_gather_matches at world 8: every rank's records of each push on the root."""
    import torch
    from siddhi_amd.native import LAYOUT_FULL, HipGroup
    cq = program_for(cfg)
    keys = {2: 4000, 4: 400}[cfg]
    g = small_stream(cfg, 160_000, keys)
    grp = HipGroup(cq.program_json(), 0, max_keys=keys, max_batch=1 << 17, max_matches=1 << 17,
                   devices=[0] * 8, match_layout=LAYOUT_FULL)
    cols = columns_for(cq, g)
    parts = []
    bounds = np.linspace(0, len(g["ts"]), 4).astype(np.int64)
    for p in range(3):
        grp.push_device(_slices(g, cols, bounds[p], bounds[p + 1], 8, len(cq.program["streams"]) > 1))
        parts.append(grp.gather(root))
        torch.cuda.synchronize()
    grp.close()
    want, have = per_key(run(OracleEngine(cq.program_json(), 0), cq, g)), per_key(_concat(parts))
    if cfg == 4:
        want, have = _drop_pos(want), _drop_pos(have)
    assert compare(want, have) is None, compare(want, have)


def test_group_world8_rank_overflow_is_refused_and_state_kept():
    """At world 8, a push whose keys all land on one rank beyond its max_batch fails before any
    engine runs; the group's state is untouched, so the next pushes match the oracle over the
    stream without the refused slice."""
    import torch
    from siddhi_amd.native import LAYOUT_FULL, HipGroup, ShpError
    cq = program_for(2)
    keys = 4000
    g = small_stream(2, 120_000, keys)
    bad = {k: v.copy() for k, v in g.items()}
    bad["key"] = (bad["key"] // 8) * 8  # every key on rank 0
    grp = HipGroup(cq.program_json(), 0, max_keys=keys, max_batch=20_000, max_matches=1 << 17,
                   devices=[0] * 8, match_layout=LAYOUT_FULL)
    cols = columns_for(cq, g)
    parts = []
    grp.push_device(_slices(g, cols, 0, 60_000, 8, False))
    parts.append(grp.fetch())
    with pytest.raises(ShpError, match="SHP_ERR_CAPACITY"):
        grp.push_device(_slices(bad, columns_for(cq, bad), 60_000, 120_000, 8, False))
    grp.push_device(_slices(g, cols, 60_000, 120_000, 8, False))
    parts.append(grp.fetch())
    torch.cuda.synchronize()
    grp.close()
    want = per_key(run(OracleEngine(cq.program_json(), 0), cq, g))
    got = per_key(_concat(parts))
    assert compare(want, got) is None, compare(want, got)
