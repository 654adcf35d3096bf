"""C2, C3′ and C5 at their configured sizes (10^8 events; 10k, 1M and 100k keys) on
the HIP path, through a size-independent property: the bench's stream generated in HBM
(`shp_synth_fill`) pushed as one 10^8-event batch and as four 2.5*10^7-event batches gives the same
matches -- key, ts, type, emission event and every slot's sequence numbers (FULL records; C5's running
avg as SHP_LAYOUT_AGG values), per key in emission order.  The split run carries every key's open
partials and aggregate state across three push boundaries; sequence numbers are the engine's running
count, so both runs name the same events.  (Parity against the oracle at sizes it finishes in seconds:
test_gpu_parity.py, test_c3_scale.py, test_retention.py; C4 at scale: test_c4_scale.py.)
"""
import ctypes

import numpy as np
import pytest

from diff_util import program_for

pytestmark = pytest.mark.gpu

N = 100_000_000


def _fetch(L, native, e):
    """shp_fetch_matches: the last device push's records copied to host memory (FULL rows with
    num_states slots each, in reference emission order; AGG rows as produced)."""
    mt = native.ShpMatches()
    rc = L.shp_fetch_matches(e.h, ctypes.byref(mt))
    assert rc == 0, L.shp_last_error(e.h)
    return native.matches_to_numpy(mt)


def _device_stream(L, cfg):
    import torch
    from siddhi_amd import synth
    spec = synth.CONFIGS[3 if cfg == "3b" else cfg]
    ts = torch.empty(N, dtype=torch.int64, device="cuda")
    key = torch.empty(N, dtype=torch.int32, device="cuda")
    price = torch.empty(N, dtype=torch.float32, device="cuda")
    assert L.shp_synth_fill(spec.config, 0, N, spec.keys, spec.n_streams, int(spec.dense), ts.data_ptr(),
                            key.data_ptr(), price.data_ptr(), None, None, None) == 0
    torch.cuda.synchronize()
    return spec.keys, ts, key, price


def _run(L, native, cq, keys, dev, layout, pushes):
    ts, key, price = dev
    step = N // pushes
    e = native.HipEngine(cq.program_json(), 0, max_keys=keys, max_batch=step, max_matches=step,
                         match_layout=layout)
    ncol = max(1, len(cq.columns))
    parts = []
    for p in range(pushes):
        lo = p * step
        colp = (ctypes.c_void_p * ncol)(*([price.data_ptr() + 4 * lo] * ncol))
        b = native.ShpBatch(step, ts.data_ptr() + 8 * lo, key.data_ptr() + 4 * lo, None,
                            ctypes.cast(colp, ctypes.c_void_p), None)
        mt = native.ShpMatches()
        rc = L.shp_push_batch_device(e.h, ctypes.byref(b), ctypes.byref(mt))
        assert rc == 0, L.shp_last_error(e.h)
        parts.append(_fetch(L, native, e))  # (mt holds device pointers: the records stay in HBM)
    path = e.path
    e.close()
    return parts, path


def _per_key_full(parts):
    """FULL records of every push, concatenated and stably sorted by key (per-key emission order)."""
    key = np.concatenate([p["key"] for p in parts])
    order = np.argsort(key, kind="stable")
    out = {"key": key[order]}
    for f in ("ts", "type", "pos"):
        out[f] = np.concatenate([p[f] for p in parts])[order]
    sl = np.concatenate([p["slot_len"] for p in parts])
    out["slot_len"] = sl[order]
    # refs: per match its slots' sequence numbers, regrouped in the sorted match order
    refs = np.concatenate([p["refs"] for p in parts])
    cnt = sl.astype(np.int64).sum(axis=1)
    start = np.concatenate([[0], np.cumsum(cnt)[:-1]])
    c, s = cnt[order], start[order]
    # each match's run of refs in the new order: position j of the output reads s_i + (j - new start_i)
    idx = np.arange(int(c.sum())) + np.repeat(s - np.concatenate([[0], np.cumsum(c)[:-1]]), c)
    out["refs"] = refs[idx]
    return out


def _per_key_agg(parts):
    key = np.concatenate([p["key"] for p in parts])
    order = np.argsort(key, kind="stable")
    return {"key": key[order], "agg": np.concatenate([p["agg"] for p in parts])[order]}


@pytest.mark.parametrize("cfg,layout_name,path", [(2, "FULL", 2), ("3b", "FULL", 3), (5, "AGG", 2)])
def test_full_size_one_push_equals_four(cfg, layout_name, path):
    from siddhi_amd import native
    L = native.lib()
    cq = program_for(cfg)
    layout = getattr(native, "LAYOUT_" + layout_name)
    keys, ts, key, price = _device_stream(L, cfg)
    one, p1 = _run(L, native, cq, keys, (ts, key, price), layout, 1)
    four, p4 = _run(L, native, cq, keys, (ts, key, price), layout, 4)
    assert p1 == p4 == path
    a, b = (_per_key_agg(one), _per_key_agg(four)) if layout_name == "AGG" else (_per_key_full(one), _per_key_full(four))
    assert len(a["key"]) > 1_000_000 and len(a["key"]) == len(b["key"])
    for name in a:
        assert np.array_equal(a[name], b[name]), name
