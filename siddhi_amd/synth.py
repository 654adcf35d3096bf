"""Deterministic synthetic event streams of SURVEY.md §8d (PCG32, identical in C++/HIP and numpy).

Event i of config c uses PCG32(seed = 0x51DD1 + c, stream 1), drawing in order
  key = pcg32() % K ; price = (float)(pcg32() % 10000) / 100.0f ; vol = pcg32() % 1000
  [; stream = pcg32() % n_streams  when the config has several streams]
ts_i = T0 + floor(i / max(1, K // 100)), except configs that set dense=True (C1, C4): ts_i = T0 + i.
The HIP generator (shp_synth_fill in libsiddhi_hip.so) produces the same arrays on the device.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

T0 = 1_544_512_385_000
MULT = np.uint64(6364136223846793005)
M64 = (1 << 64) - 1


def _pcg_seed(initstate: int, initseq: int):
    inc = ((initseq << 1) | 1) & M64
    state = 0
    state = (state * 6364136223846793005 + inc) & M64
    state = (state + initstate) & M64
    state = (state * 6364136223846793005 + inc) & M64
    return state, inc


def _advance(state: int, inc: int, delta: int) -> int:
    """LCG jump-ahead (pcg32_advance): state after `delta` steps."""
    acc_mult, acc_plus = 1, 0
    cur_mult, cur_plus = 6364136223846793005, inc
    while delta > 0:
        if delta & 1:
            acc_mult = (acc_mult * cur_mult) & M64
            acc_plus = (acc_plus * cur_mult + cur_plus) & M64
        cur_plus = ((cur_mult + 1) * cur_plus) & M64
        cur_mult = (cur_mult * cur_mult) & M64
        delta >>= 1
    return (acc_mult * state + acc_plus) & M64


def _output(old: np.ndarray) -> np.ndarray:
    xorshifted = (((old >> np.uint64(18)) ^ old) >> np.uint64(27)).astype(np.uint32)
    rot = (old >> np.uint64(59)).astype(np.uint32)
    return ((xorshifted >> rot) | (xorshifted << ((-rot.astype(np.int64)) & 31).astype(np.uint32))).astype(np.uint32)


def pcg32_draws(seed: int, start: int, count: int, lanes: int = 8192) -> np.ndarray:
    """Draws start..start+count-1 of PCG32(seed, stream 1)."""
    state0, inc = _pcg_seed(seed, 1)
    lanes = max(1, min(lanes, count))
    per = -(-count // lanes)
    st = np.array([_advance(state0, inc, start + l * per) for l in range(lanes)], dtype=np.uint64)
    out = np.empty((per, lanes), np.uint32)
    incu = np.uint64(inc)
    with np.errstate(over="ignore"):
        for s in range(per):
            out[s] = _output(st)
            st = st * MULT + incu
    return out.T.reshape(-1)[:count]


@dataclass
class StreamSpec:
    config: int
    n: int
    keys: int
    n_streams: int = 1
    dense: bool = False  # ts = T0 + i


CONFIGS = {
    1: StreamSpec(1, 1_000_000, 1, 1, True),
    2: StreamSpec(2, 100_000_000, 10_000),
    3: StreamSpec(3, 100_000_000, 1_000_000),
    4: StreamSpec(4, 100_000_000, 1_000, 3, True),
    5: StreamSpec(5, 100_000_000, 100_000),
}


def generate(spec: StreamSpec, start: int = 0, count: int | None = None):
    """Return dict of numpy arrays (ts, key, price, volume, stream) for events start..start+count-1."""
    count = spec.n if count is None else count
    per = 4 if spec.n_streams > 1 else 3
    d = pcg32_draws(0x51DD1 + spec.config, start * per, count * per).reshape(count, per)
    key = (d[:, 0] % np.uint32(spec.keys)).astype(np.int32)
    price = ((d[:, 1] % np.uint32(10000)).astype(np.float32) / np.float32(100.0)).astype(np.float32)
    vol = (d[:, 2] % np.uint32(1000)).astype(np.int64)
    stream = (d[:, 3] % np.uint32(spec.n_streams)).astype(np.int32) if per == 4 else np.zeros(count, np.int32)
    i = np.arange(start, start + count, dtype=np.int64)
    if spec.dense:
        ts = T0 + i
    else:
        ts = T0 + i // max(1, spec.keys // 100)
    return {"ts": ts, "key": key, "price": price, "volume": vol, "stream": stream}


# canonical queries
QUERIES = {
    1: "define stream StockStream (symbol string, price float, volume long); "
       "@info(name='q') from every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] within 1 sec "
       "select e1.symbol as s1, e1.price as p1, e2.price as p2 insert into Out;",
    2: "define stream StockStream (symbol string, price float, volume long); "
       "partition with (symbol of StockStream) begin "
       "@info(name='q') from every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] within 1 sec "
       "select e1.symbol as s1, e1.price as p1, e2.price as p2 insert into Out; end;",
    3: "define stream S (k string, v float); partition with (k of S) begin "
       "@info(name='q') from e1=S[v>20]<2:5>, e2=S[v<e1[last].v] "
       "select e1[0].v as a, e1[last].v as b, e2.v as c insert into Out; end;",
    "3b": "define stream S (k string, v float); partition with (k of S) begin "
          "@info(name='q') from every e1=S[v>20]<1:5>, e2=S[v<e1[last].v] "
          "select e1[0].v as a, e1[last].v as b, e2.v as c insert into Out; end;",
    4: "@app:playback define stream S1 (symbol string, price float, volume long); "
       "define stream S2 (symbol string, price float, volume long); "
       "define stream S3 (symbol string, price float, volume long); "
       "partition with (symbol of S1, symbol of S2, symbol of S3) begin "
       "@info(name='q') from every (e1=S1[price>20] and e2=S2[price>20]) -> not S3[price>e1.price] for 5 sec "
       "within 10 sec select e1.symbol as s, e1.price as p1, e2.price as p2 insert into Out; end;",
    5: "define stream StockStream (symbol string, price float, volume long); "
       "partition with (symbol of StockStream) begin "
       "@info(name='q') from every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] within 1 sec "
       "select e1.symbol as symbol, avg(e2.price) as avgPrice insert into Out; end;",
}
