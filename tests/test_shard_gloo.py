"""Multi-rank host logic of the sharded path (desamba-so_amd/shard.py) on CPU with gloo,
world_size 2: contiguous read shards + per-taxon count all_reduce == the whole-input
meta_analysis node_count table."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT, golden
from samutil import ana_get_tid, groups, read_parents

import sys
sys.path.insert(0, os.path.join(ROOT, "desamba-so_amd"))
import shard  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_bounds_partition():
    for n in (0, 1, 5, 600, 1001):
        for world in (1, 2, 3, 8):
            got = [shard.shard_bounds(n, r, world) for r in range(world)]
            assert got[0][0] == 0 and got[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(got, got[1:]))
            assert max(h - l for l, h in got) - min(h - l for l, h in got) <= 1


def test_split_fastq_concatenates_back():
    fq = golden("mixed.fq")
    for world in (1, 2, 3, 8):
        assert b"".join(shard.split_fastq(fq, r, world) for r in range(world)) == fq


def _worker(rank, world, port, tids, n_tax, q):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    lo, hi = shard.shard_bounds(len(tids), rank, world)
    c = shard.reduce_counts(shard.taxon_counts(tids[lo:hi], None, n_tax))
    q.put((rank, c.numpy()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_taxon_count_reduce_world2(fixture_index, world):
    parent = read_parents(os.path.join(fixture_index, "nodes.dmp"))
    max_tid = max(parent) + 1000000  # reference src/cly_mt.c:613
    tids = np.array([ana_get_tid(r, parent, max_tid) for _, r in groups(golden("mixed.herm.sam"))], dtype=np.uint32)
    n_tax = max_tid + 1
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, tids, n_tax, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = np.bincount(tids, minlength=n_tax)
    for r in range(world):
        assert (res[r] == want).all()
    assert want.sum() == len(tids) and want[0] < len(tids)


def test_carry_rerun_prefix_only_when_earlier_ranks_cross_the_2g_threshold():
    # reference src/cly.c:2954: the carried max_read_l is only read through "< 510"
    assert shard.carry_rerun_prefix([0, 150, 150, 600, 900], 509) == 0
    assert shard.carry_rerun_prefix([0, 150, 150, 600, 900], 510) == 3
    assert shard.carry_rerun_prefix([700, 900], 8000) == 0
    assert shard.carry_rerun_prefix([150] * 7, 600) == 7
    assert shard.carry_rerun_prefix([], 600) == 0


def _carry_worker(rank, world, port, carries, q):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    q.put((rank, shard.earlier_carry(carries[rank], rank, world)))
    dist.destroy_process_group()


def test_earlier_carry_is_exclusive_prefix_max_world3():
    carries = [300, 8000, 150]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_carry_worker, args=(r, 3, port, carries, q)) for r in range(3)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == {0: 0, 1: 300, 2: 8000}
