"""Multi-GPU sharding of the classify path (one process per GPU, torch.distributed).

Reads shard across ranks: each rank owns a contiguous block of FASTQ records, classifies it
on its own GPU against its own replica of the index, and assigns one taxon per read exactly as
meta_analysis does (reference src/cly_mt.c:902-961, dsb_batch_taxa).  Two exchanges:

* the carried buffer-pool length (Classify_buff_pool.max_read_l, reference src/cly.c:2953):
  a whole-input run carries the longest read that reached the length filter into every later
  read.  Each rank publishes its own maximum (one int per rank, all_gather); a rank whose
  earlier ranks reached the 2G-read threshold re-runs the leading reads whose own carry was
  still below it (src/cly.c:2954 is the only place the carry is read, and only through
  "max_read_l < 510", so no other read can change);
* the final per-taxon count reduction (all_reduce SUM over RCCL / "nccl"; "gloo" in the CPU
  tests): the node_count table of meta_analysis (src/cly_mt.c:1352-1362) for the whole input.
"""
from __future__ import annotations

# delete_small_score_rst's 2G-read branch (reference src/cly.c:2954: max_read_l < 510)
CARRY_THRESHOLD = 510


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


def earlier_carry(local_carry: int, rank: int, world: int) -> int:
    """Exclusive prefix max over ranks of their out-carry (all_gather of one int per rank)."""
    import torch
    import torch.distributed as dist
    if world <= 1 or not (dist.is_available() and dist.is_initialized()):
        return 0
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.zeros(world, dtype=torch.int64, device=dev)
    t[rank] = int(local_carry)
    dist.all_reduce(t)  # each slot written by exactly one rank: the reduce is a gather
    return int(t[:rank].max().item()) if rank > 0 else 0


def carry_rerun_prefix(carry, p_earlier: int) -> int:
    """Reads to re-run once the carry of earlier ranks is known: the leading reads whose own
    carry stayed below the 2G threshold while the earlier ranks' carry reached it.  carry is
    monotone (a prefix max), so they form a prefix of the shard."""
    if p_earlier < CARRY_THRESHOLD:
        return 0  # max(p, c) < 510 exactly when c < 510: nothing the filter reads changes
    k = 0
    for c in carry:
        if c >= CARRY_THRESHOLD:
            break
        k += 1
    return k


def taxon_counts(tid, weight, n_tax: int, device=None):
    """Per-taxon weights of one shard (meta_analysis node_count, src/cly_mt.c:1352-1362).
    device=None: a numpy table; otherwise the table is counted there (torch.bincount; integer
    weights, exact)."""
    import numpy as np
    if device is None:
        return np.bincount(np.asarray(tid, dtype=np.int64), weights=None if weight is None else
                           np.asarray(weight, dtype=np.float64), minlength=n_tax).astype(np.int64)
    import torch
    t = torch.from_numpy(np.asarray(tid, dtype=np.int64)).to(device, non_blocking=False)
    if weight is None:
        return torch.bincount(t, minlength=n_tax)
    wt = torch.from_numpy(np.asarray(weight, dtype=np.int64)).to(device)
    out = torch.zeros(n_tax, dtype=torch.int64, device=device)
    return out.index_add_(0, t, wt)


def reduce_counts(counts, device="cpu"):
    """all_reduce SUM of a rank's per-taxon counts; returns the global table (torch int64)."""
    import torch
    import torch.distributed as dist
    t = torch.as_tensor(counts, dtype=torch.int64).to(device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t)
    return t


class ShardResult:
    """One rank's classified share: the batch, plus the re-run of its leading reads when the
    carry of earlier ranks changed them (prefix reads come from `head`)."""

    def __init__(self, batch, head=None, k: int = 0):
        self.batch, self.head, self.k = batch, head, k

    def taxa(self, flag: int = 0):
        tid, w = self.batch.taxa(flag)
        if self.head is not None:
            ht, hw = self.head.taxa(flag)
            tid[:self.k], w[:self.k] = ht, hw
        return tid, w

    def format(self, fmt: int = 1) -> bytes:
        if self.head is None:
            return self.batch.format(fmt)
        return self.head.format(fmt) + self.batch.format_range(self.k, self.batch.n_reads, fmt)

    def close(self):
        for b in (self.head, self.batch):
            if b is not None:
                b.close()


def classify_shard(index, data: bytes, rank: int, world: int, flag: int = 0, device="cuda", carry_in: int = 0):
    """Classify this rank's share of data on its GPU; returns (global per-taxon counts,
    ShardResult).  index: a pydesamba.Index resident on this rank's GPU.  The result equals
    one whole-input read_classify call (carry_in: that call's incoming max_read_l)."""
    part = split_fastq(data, rank, world)
    batch = index.batch(part)
    batch.run(max_read_l=carry_in)
    p = max(carry_in, earlier_carry(batch.max_read_l, rank, world))
    res = ShardResult(batch)
    k = carry_rerun_prefix(batch.carry(), p) if batch.n_reads else 0
    if k:
        offs = fastq_records(part)
        head = index.batch(part[:offs[k]])
        head.run(max_read_l=p)
        res = ShardResult(batch, head, k)
    tid, w = res.taxa(flag)
    return reduce_counts(taxon_counts(tid, w, index.max_tid() + 1), device), res
