"""Key-owner sharding of event batches across ranks.

A partitioned query's per-key state is isolated (``PartitionStateHolder.java:43-48``), so N
GPUs split the keys: key k lives on rank ``k % N`` (the reference's own sink precedent is
``Math.abs(key.hashCode() % N)``, ``PartitionedDistributionStrategy.java:101``).  Each rank
ingests a contiguous slice of the stream; one exchange per batch (RCCL all-to-alls over xGMI with
the ``nccl`` backend, gloo on CPU) sends every event to its key's owner.  The received buffer is
ordered by source rank and, within a source, by arrival (a stable sort), so when the ranks'
slices are consecutive pieces of the stream every key sees its events in global arrival order.
Owned keys are renumbered densely (``k // N``) so each rank's engine holds a dictionary of
``ceil(K / N)`` ids.
"""
from __future__ import annotations

from typing import Dict


def owner_of(key, world: int):
    return key % world


def local_key(key, world: int):
    """Dense id of an owned key on its rank (the rank's own dictionary)."""
    return key // world


def exchange(cols: Dict[str, "torch.Tensor"], key_name: str, world: int, dist) -> Dict[str, "torch.Tensor"]:
    """All-to-all of SoA columns by key owner; returns the columns this rank owns.

    ``cols[key_name]`` holds global key ids.  Every column keeps its dtype; the order within a
    source rank is preserved (stable sort) and sources arrive in rank order.
    """
    import torch

    key = cols[key_name]
    own = owner_of(key.to(torch.int64), world)
    order = torch.argsort(own, stable=True)
    send = torch.bincount(own, minlength=world)
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send)
    sc, rc = send.tolist(), recv.tolist()
    out = {}
    for name, col in cols.items():
        src = col[order].contiguous()
        dst = torch.empty(sum(rc), dtype=col.dtype, device=col.device)
        dist.all_to_all_single(dst, src, rc, sc)
        out[name] = dst
    return out


class DeviceExchange:
    """The same exchange on HBM-resident batches with the engine's HIP kernels: one stable split
    by destination into destination-grouped SoA columns (``shp_shard_partition_soa``), then one
    all-to-all per column (RCCL), whose receive buffers are the owner's engine input as they
    stand: ts, key (the owner's dense id ``key // N``), value, and stream when present.  There is
    no unpack pass.  Send buffers are allocated once for ``capacity`` events."""

    def __init__(self, capacity: int, world: int, dist, device, with_stream: bool = False,
                 cpu_collectives: bool = False, value_dtype=None):
        import torch

        from . import native
        self.L = native.lib()
        self.G, self.dist = world, dist
        vd = value_dtype or torch.float32
        if torch.empty(0, dtype=vd).element_size() != 4:
            raise ValueError("DeviceExchange moves 4-byte value columns (int, float, string id) only")
        self.s_ts = torch.empty(capacity, dtype=torch.int64, device=device)
        self.s_key = torch.empty(capacity, dtype=torch.int32, device=device)
        self.s_val = torch.empty(capacity, dtype=vd, device=device)
        self.s_stream = torch.empty(capacity, dtype=torch.int32, device=device) if with_stream else None
        self.ws = torch.empty(int(self.L.shp_shard_workspace_bytes(capacity, world)), dtype=torch.uint8,
                              device=device)
        self.counts = (ctypes_int64 * world)()
        self.with_stream = with_stream
        self.cpu = cpu_collectives  # gloo rehearsal (all ranks on one GPU): collectives on host copies

    def start(self, ts, key, value, stream=None):
        """Partition (HIP) and launch the per-column all-to-alls asynchronously; finish() completes them."""
        import torch

        n = ts.numel()
        if n > self.s_ts.numel() or value.dtype != self.s_val.dtype:
            raise ValueError("batch larger than the exchange capacity, or a different value dtype")
        if (stream is not None) != (self.s_stream is not None):
            raise ValueError("stream column presence differs from the exchange's")
        cur = torch.cuda.current_stream().cuda_stream
        rc = self.L.shp_shard_partition_soa(n, ts.data_ptr(), key.data_ptr(), value.data_ptr(),
                                            stream.data_ptr() if stream is not None else None, self.G,
                                            self.s_ts.data_ptr(), self.s_key.data_ptr(), self.s_val.data_ptr(),
                                            self.s_stream.data_ptr() if stream is not None else None,
                                            self.counts, self.ws.data_ptr(), cur)
        if rc != 0:
            raise RuntimeError(f"shp_shard_partition_soa failed ({rc})")
        send = torch.tensor(list(self.counts), dtype=torch.int64, device="cpu" if self.cpu else ts.device)
        recv = torch.empty_like(send)
        self.dist.all_to_all_single(recv, send)
        sc, rc_ = send.tolist(), recv.tolist()
        m = sum(rc_)
        srcs = [self.s_ts[:n], self.s_key[:n], self.s_val[:n]] + ([self.s_stream[:n]] if stream is not None else [])
        outs = [torch.empty(m, dtype=c.dtype, device=ts.device) for c in srcs]
        works = []
        if self.cpu:
            host = [torch.empty(m, dtype=c.dtype) for c in srcs]
            for h, c in zip(host, srcs):
                works.append(self.dist.all_to_all_single(h, c.cpu(), rc_, sc, async_op=True))
            return works, outs, host
        for o, c in zip(outs, srcs):
            works.append(self.dist.all_to_all_single(o, c, rc_, sc, async_op=True))
        return works, outs, None

    def finish(self, pending):
        """Wait for the all-to-alls; returns (ts, key, value, stream-or-None) of the owned events."""
        works, outs, host = pending
        for w in works:
            w.wait()
        if host is not None:
            for o, h in zip(outs, host):
                o.copy_(h)
        return outs[0], outs[1], outs[2], (outs[3] if len(outs) > 3 else None)

    def __call__(self, ts, key, value, stream=None):
        return self.finish(self.start(ts, key, value, stream))


import ctypes as _ctypes  # noqa: E402

ctypes_int64 = _ctypes.c_int64
