"""Data-parallel sharding of a record batch across ranks (one process per
GPU), and the final gather of encoded shards.

The reference marshals one batch per call on one core (xdr_to_opaque,
xdrpp/marshal.h:264-272); records are independent, so a batch of
world * n records splits into contiguous shards with no exchange on the
data path: rank r owns records [r * n, (r + 1) * n) and produces the XDR
bytes of exactly those records.  The concatenation of the shards' streams
in rank order is byte-identical to the stream of the whole batch, and the
record index of the whole batch is the shards' indices rebased by the
running stream length (tests/test_shard.py proves both with gloo).

`gather_streams` is the one collective: it brings every shard's stream and
record index to rank 0 (torch.distributed.gather; RCCL on MI355X, gloo in
the CPU tests).  It is timed and reported apart from the marshal step.
"""
from __future__ import annotations

import numpy as np

from . import workloads as W


def shard_range(rank: int, world: int, n_per_rank: int) -> tuple[int, int]:
    """(first record, record count) of `rank`'s shard (weak scaling)."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world of {world}")
    return rank * n_per_rank, n_per_rank


def seed_for(schema: str, world: int) -> int:
    """rec128 on N>1 GPUs uses its own seed."""
    if schema == "rec128":
        return W.SEED_REC128 if world == 1 else W.SEED_REC128_MGPU
    return {"numerics": W.SEED_NUMERICS, "recvar": W.SEED_RECVAR, "rpc": W.SEED_RPC,
            "vecrec": W.SEED_VECREC}[schema]


def shard_inputs(schema: str, n_per_rank: int, rank: int, world: int
                 ) -> tuple[np.ndarray, np.ndarray]:
    """Native records and heap of `rank`'s shard (heap offsets shard-local)."""
    first, n = shard_range(rank, world, n_per_rank)
    return W.GENERATORS[schema](n, seed=seed_for(schema, world), first=first)


def gather_streams(dist, xdr, offsets, rank: int, world: int):
    """Gather every rank's XDR stream (uint8 tensor) and, for var-length
    plans, its record index (int64 tensor of n + 1 entries, or None) on
    rank 0.  Returns (stream, index) on rank 0 and (None, None) elsewhere;
    index is None when `offsets` is None.  Shards may differ in length:
    lengths are exchanged first and streams padded to the longest."""
    import torch

    dev = xdr.device
    ln = torch.tensor([xdr.numel()], dtype=torch.int64, device=dev)
    lens = [torch.zeros_like(ln) for _ in range(world)]
    dist.all_gather(lens, ln)
    lens = [int(x.item()) for x in lens]
    mx = max(lens)
    buf = xdr
    if xdr.numel() < mx:
        buf = torch.zeros(mx, dtype=torch.uint8, device=dev)
        buf[: xdr.numel()] = xdr
    got = [torch.empty(mx, dtype=torch.uint8, device=dev) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, got, dst=0)
    idx_parts = None
    if offsets is not None:
        idx_parts = ([torch.empty_like(offsets) for _ in range(world)] if rank == 0 else None)
        dist.gather(offsets, idx_parts, dst=0)
    if rank != 0:
        return None, None
    stream = torch.cat([g[:k] for g, k in zip(got, lens)])
    index = None
    if idx_parts is not None:
        base = 0
        parts = []
        for i, (part, k) in enumerate(zip(idx_parts, lens)):
            parts.append(part[:-1] + base if i < world - 1 else part + base)
            base += k
        index = torch.cat(parts)
    return stream, index
