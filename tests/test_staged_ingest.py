"""Pipelined host ingest (shp_stage_batch / shp_stage_batch_ts32 / shp_run_staged): the
host copy of batch i+1 runs on a copy stream while the engine runs batch i.  The records must be the
ones shp_push_batch_compact returns for the same pushes (same committed state, same layout): checked
batch by batch on C2 (PAIRS32), C3' (CHAIN32) and C4 (FULL records), int64 and narrow ts, and against
the oracle per key after expansion.
"""
import numpy as np
import pytest

from diff_util import columns_for, program_for, small_stream


def _batches(g, step):
    n = len(g["ts"])
    return [(lo, min(n, lo + step)) for lo in range(0, n, step)]


def _engine(cfg, keys, batch, layout):
    from siddhi_amd.native import HipEngine
    cq = program_for(cfg)
    return cq, HipEngine(cq.program_json(), 0, max_keys=keys, max_batch=batch, match_layout=layout)


def _canon(r):
    """The compact words in a canonical order: per key the engine's order is the reference's emission
    order, across keys it follows which workgroup reserved its output first -- so sort stably by e2's
    batch index (one key per e2), as the host's decoding does (history.decode_pairs32)."""
    w = r["words"]
    if r["layout"] == 3:  # PAIRS32: (e2 index, delta) pairs
        p = w.reshape(-1, 2)
        return p[np.argsort(p[:, 0], kind="stable")]
    return np.sort(w & 0x0FFFFFFF) if r["layout"] == 4 else w  # CHAIN32: one match per e2


def _same(a, b):
    assert a["layout"] == b["layout"] and a["m"] == b["m"]
    if "words" in a:
        assert np.array_equal(_canon(a), _canon(b))
        if a["layout"] == 4:
            assert np.array_equal(np.sort(a["words"]), np.sort(b["words"]))
    else:
        for k in ("key", "ts", "type", "slot_len", "refs"):
            assert np.array_equal(a[k], b[k]), k


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,keys,n,step,layout,narrow", [
    (2, 10_000, 2_000_000, 300_007, 5, False), (2, 10_000, 2_000_000, 300_007, 5, True),
    (2, 10_000, 2_000_000, 300_007, 5, "key16"), ("3b", 50_000, 1_500_000, 250_003, 5, True),
    ("3b", 50_000, 1_500_000, 250_003, 5, "key16"), (5, 100_000, 1_000_000, 200_003, 5, False),
    (4, 1_000, 600_000, 100_003, 5, True), (4, 1_000, 600_000, 100_003, 5, "key16")])
def test_staged_pipeline_equals_compact_push(cfg, keys, n, step, layout, narrow):
    g = small_stream(cfg if cfg != "3b" else 3, n, keys)
    cq, a = _engine(cfg, keys, step, layout)
    _, b = _engine(cfg, keys, step, layout)
    cols = columns_for(cq, g)
    parts = _batches(g, step)
    want = []
    for lo, hi in parts:
        want.append(a.push_compact(g["ts"][lo:hi], g["key"][lo:hi], g["stream"][lo:hi],
                                   [c[lo:hi] for c in cols], [None] * len(cols)))

    def stage(i):
        lo, hi = parts[i]
        args = (g["ts"][lo:hi], g["key"][lo:hi], g["stream"][lo:hi], [c[lo:hi] for c in cols], [None] * len(cols))
        if narrow:
            base = int(g["ts"][lo])
            k16 = g["key"][lo:hi].astype(np.uint16) if narrow == "key16" else None
            b.stage(None, *args[1:], ts32=(g["ts"][lo:hi] - base).astype(np.int32), ts_base=base, key16=k16)
        else:
            b.stage(*args)
    got = []
    stage(0)
    for i in range(len(parts)):
        if i + 1 < len(parts):
            stage(i + 1)  # batch i+1's copies overlap batch i's run
        got.append(b.run_staged())
    assert len(got) == len(want)
    for x, y in zip(got, want):
        _same(x, y)
    assert sum(x["m"] for x in want) > 1000 or cfg == 4


@pytest.mark.gpu
def test_staged_capacity_and_empty_run_errors():
    from siddhi_amd.native import ShpError
    g = small_stream(2, 30_000, 100)
    cq, e = _engine(2, 100, 10_000, 5)
    cols = columns_for(cq, g)
    with pytest.raises(ShpError) as ei:
        e.run_staged()
    assert ei.value.code == -1  # SHP_ERR_ARG: nothing staged
    for lo in (0, 10_000):
        e.stage(g["ts"][lo:lo + 10_000], g["key"][lo:lo + 10_000], g["stream"][lo:lo + 10_000],
                [c[lo:lo + 10_000] for c in cols], [None])
    with pytest.raises(ShpError) as ei:
        e.stage(g["ts"][:10], g["key"][:10], g["stream"][:10], [c[:10] for c in cols], [None])
    assert ei.value.code == -3  # SHP_ERR_CAPACITY: two batches staged
    r0, r1 = e.run_staged(), e.run_staged()
    _, ref = _engine(2, 100, 10_000, 5)
    for lo, r in ((0, r0), (10_000, r1)):
        _same(r, ref.push_compact(g["ts"][lo:lo + 10_000], g["key"][lo:lo + 10_000], g["stream"][lo:lo + 10_000],
                                  [c[lo:lo + 10_000] for c in cols], [None]))


@pytest.mark.gpu
def test_staged_narrow_keys_need_max_keys_16_bits():
    from siddhi_amd.native import ShpError
    g = small_stream(2, 1_000, 100_000)
    cq, e = _engine(2, 100_000, 1_000, 5)
    cols = columns_for(cq, g)
    with pytest.raises(ShpError) as ei:
        e.stage(None, g["key"], g["stream"], cols, [None], ts32=(g["ts"] - g["ts"][0]).astype(np.int32),
                ts_base=int(g["ts"][0]), key16=g["key"].astype(np.uint16))
    assert ei.value.code == -1  # SHP_ERR_ARG: 100k keys do not fit 2 bytes
