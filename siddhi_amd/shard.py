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
