"""Multi-GPU sharding of the classify path (one process per GPU, torch.distributed).

Reads shard across ranks with no data-path collective: each rank owns a contiguous block
of FASTQ records, classifies it on its own GPU against its own replica of the index, and
assigns one taxon per read exactly as meta_analysis does (reference src/cly_mt.c:902-961,
dsb_batch_taxa).  The only exchange is the final per-taxon count reduction (all_reduce
SUM over RCCL / "nccl"; "gloo" in the CPU tests), i.e. the node_count table of
meta_analysis (src/cly_mt.c:1352-1362) for the whole input.
"""
from __future__ import annotations


def shard_bounds(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous block [lo, hi) of n items owned by rank (sizes differ by at most one)."""
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def fastq_records(data: bytes) -> list[int]:
    """Byte offsets of the 4-line FASTQ records of data (plus the end offset)."""
    offs, pos, n = [], 0, len(data)
    while pos < n:
        offs.append(pos)
        for _ in range(4):
            nl = data.find(b"\n", pos)
            pos = n if nl < 0 else nl + 1
    offs.append(n)
    return offs


def split_fastq(data: bytes, rank: int, world: int) -> bytes:
    """The rank's contiguous share of the FASTQ records of data."""
    offs = fastq_records(data)
    lo, hi = shard_bounds(len(offs) - 1, rank, world)
    return data[offs[lo]:offs[hi]]


def taxon_counts(tid, weight, n_tax: int):
    """Per-taxon weights of one shard (meta_analysis node_count, src/cly_mt.c:1352-1362)."""
    import numpy as np
    return np.bincount(np.asarray(tid, dtype=np.int64), weights=None if weight is None else
                       np.asarray(weight, dtype=np.float64), minlength=n_tax).astype(np.int64)


def reduce_counts(counts, device="cpu"):
    """all_reduce SUM of a rank's per-taxon counts; returns the global table (torch int64)."""
    import torch
    import torch.distributed as dist
    t = torch.as_tensor(counts, dtype=torch.int64).to(device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t)
    return t


def classify_shard(index, data: bytes, rank: int, world: int, flag: int = 0, device="cuda"):
    """Classify this rank's share of data on its GPU and return (global per-taxon counts,
    this rank's batch).  index: a pydesamba.Index resident on this rank's GPU."""
    part = split_fastq(data, rank, world)
    batch = index.batch(part)
    batch.run(max_read_l=0)
    tid, w = batch.taxa(flag)
    return reduce_counts(taxon_counts(tid, w, index.max_tid() + 1), device), batch
