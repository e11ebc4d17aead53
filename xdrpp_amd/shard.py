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
            "vecrec": W.SEED_VECREC, "containertest": W.SEED_CONTAINERTEST, "rp_list": W.SEED_RP_LIST}[schema]


def shard_inputs(schema: str, n_per_rank: int, rank: int, world: int
                 ) -> tuple[np.ndarray, np.ndarray]:
    """Native records and heap of `rank`'s shard (heap offsets shard-local)."""
    first, n = shard_range(rank, world, n_per_rank)
    return W.GENERATORS[schema](n, seed=seed_for(schema, world), first=first)


def gather_streams(dist, xdr, offsets, rank: int, world: int):
    """Gather every rank's XDR stream (uint8 tensor) and, for var-length
    plans, its record index (int64 tensor of n + 1 entries, or None) on
    rank 0.  Returns (stream, index) on rank 0 and (None, None) elsewhere;
    index is None when `offsets` is None.

    Shards may differ in length and record count: both are exchanged first
    (one all_gather of two words), then every rank sends exactly its bytes
    and rank 0 receives them straight into their place in the whole stream
    (point-to-point sends and receives issued as one batch, so the root's
    links work at once; no padding, no concatenation copy).  Each rank
    rebases its own record index by the stream bytes of the ranks before it
    and sends its entries (the last rank also the end), so rank 0 receives
    the whole batch's index in place too."""
    import torch

    dev = xdr.device
    nrec = (offsets.numel() - 1) if offsets is not None else 0
    mine = torch.tensor([xdr.numel(), nrec], dtype=torch.int64, device=dev)
    every = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(every, mine)
    lens = [int(e[0].item()) for e in every]
    recs = [int(e[1].item()) for e in every]
    base = sum(lens[:rank])
    idx = None
    if offsets is not None:
        last = rank == world - 1
        idx = (offsets if last else offsets[:-1]) + base
    ops = []
    if rank != 0:
        if lens[rank]:
            ops.append(dist.P2POp(dist.isend, xdr.contiguous(), 0))
        if idx is not None and idx.numel():
            ops.append(dist.P2POp(dist.isend, idx.contiguous(), 0))
        for r in dist.batch_isend_irecv(ops) if ops else []:
            r.wait()
        return None, None
    stream = torch.empty(sum(lens), dtype=torch.uint8, device=dev)
    stream[:lens[0]].copy_(xdr)
    index = None
    if offsets is not None:
        index = torch.empty(sum(recs) + 1, dtype=torch.int64, device=dev)
        index[:idx.numel()].copy_(idx)
    for k in range(1, world):
        b, rb = sum(lens[:k]), sum(recs[:k])
        if lens[k]:
            ops.append(dist.P2POp(dist.irecv, stream[b:b + lens[k]], k))
        if index is not None:
            cnt = recs[k] + (1 if k == world - 1 else 0)
            if cnt:
                ops.append(dist.P2POp(dist.irecv, index[rb:rb + cnt], k))
    for r in dist.batch_isend_irecv(ops) if ops else []:
        r.wait()
    return stream, index
