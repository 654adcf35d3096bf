"""Key-owner sharding of event batches across ranks.

A partitioned query's per-key state is isolated (``PartitionStateHolder.java:43-48``), so N
GPUs split the keys: key k lives on rank ``k % N`` (the reference's own sink precedent is
``Math.abs(key.hashCode() % N)``, ``PartitionedDistributionStrategy.java:101``).  Each rank
ingests a contiguous slice of the stream; one all-to-all per batch (RCCL over xGMI with the
``nccl`` backend, gloo on CPU) sends every event to its key's owner.  The received buffer is
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
    by destination into packed 16-byte records (``shp_shard_partition``), ONE all-to-all of the
    packed buffer (RCCL), one unpack into SoA columns (``shp_shard_unpack``).  Keys arrive as
    the owner's dense ids (``key // N``); a stream column, when present, rides in the top byte.
    Buffers are allocated once for ``capacity`` events and reused."""

    def __init__(self, capacity: int, world: int, dist, device, with_stream: bool = False,
                 cpu_collectives: bool = False):
        import torch

        from . import native
        self.L = native.lib()
        self.G, self.dist = world, dist
        self.send = torch.empty((capacity, 2), dtype=torch.int64, device=device)
        self.recv = torch.empty((int(capacity * 1.1) + 4096, 2), dtype=torch.int64, device=device)
        self.ws = torch.empty(int(self.L.shp_shard_workspace_bytes(capacity, world)), dtype=torch.uint8,
                              device=device)
        self.counts = (ctypes_int64 * world)()
        self.with_stream = with_stream
        self.cpu = cpu_collectives  # gloo rehearsal (all ranks on one GPU): collectives on host copies

    def start(self, ts, key, value, stream=None):
        """Partition (HIP) and launch the all-to-all asynchronously; finish() completes it."""
        import torch

        n = ts.numel()
        cur = torch.cuda.current_stream().cuda_stream
        rc = self.L.shp_shard_partition(n, ts.data_ptr(), key.data_ptr(), value.data_ptr(),
                                        stream.data_ptr() if stream is not None else None, self.G,
                                        self.send.data_ptr(), self.counts, self.ws.data_ptr(), cur)
        if rc != 0:
            raise RuntimeError(f"shp_shard_partition failed ({rc})")
        send = torch.tensor(list(self.counts), dtype=torch.int64, device="cpu" if self.cpu else ts.device)
        recv = torch.empty_like(send)
        self.dist.all_to_all_single(recv, send)
        sc, rc_ = send.tolist(), recv.tolist()
        m = sum(rc_)
        if m > self.recv.shape[0]:
            raise RuntimeError("receive buffer too small for this exchange")
        if self.cpu:
            host_recv = torch.empty((m, 2), dtype=torch.int64)
            work = self.dist.all_to_all_single(host_recv, self.send[:n].cpu(), rc_, sc, async_op=True)
            return work, m, value.dtype, stream is not None, ts.device, host_recv
        work = self.dist.all_to_all_single(self.recv[:m], self.send[:n], rc_, sc, async_op=True)
        return work, m, value.dtype, stream is not None, ts.device, None

    def finish(self, pending):
        """Wait for the all-to-all and unpack the received records into SoA columns."""
        import torch

        work, m, vdtype, has_stream, dev, host_recv = pending
        work.wait()
        if host_recv is not None:
            self.recv[:m].copy_(host_recv)
        out_ts = torch.empty(m, dtype=torch.int64, device=dev)
        out_key = torch.empty(m, dtype=torch.int32, device=dev)
        out_val = torch.empty(m, dtype=vdtype, device=dev)
        out_stream = torch.empty(m, dtype=torch.int32, device=dev) if has_stream else None
        rc = self.L.shp_shard_unpack(m, self.recv.data_ptr(), out_ts.data_ptr(), out_key.data_ptr(),
                                     out_val.data_ptr(), out_stream.data_ptr() if out_stream is not None else None,
                                     torch.cuda.current_stream().cuda_stream)
        if rc != 0:
            raise RuntimeError(f"shp_shard_unpack failed ({rc})")
        return out_ts, out_key, out_val, out_stream

    def __call__(self, ts, key, value, stream=None):
        return self.finish(self.start(ts, key, value, stream))


import ctypes as _ctypes  # noqa: E402

ctypes_int64 = _ctypes.c_int64
