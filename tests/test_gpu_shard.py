"""Sharded classify (desamba-so_amd/shard.py) end to end on the GPU: two ranks (gloo for the
exchanges, both on cuda:0) give the same per-taxon counts and the same records as one
whole-input call — including the carried max_read_l (reference src/cly.c:2953-2963) that a
rank holding only short reads must take over from the long reads of the rank before it."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT, golden
from samutil import groups

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _records(fq: bytes):
    lines = fq.split(b"\n")
    return [b"\n".join(lines[i:i + 4]) + b"\n" for i in range(0, len(lines) - 3, 4)]


def _rank(rank, world, port, index_dir, data, q):
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(ROOT, "desamba-so_amd"))
    os.environ["DSB_DEVICE"] = "0"
    import pydesamba
    import shard
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    idx = pydesamba.Index(index_dir)
    counts, res = shard.classify_shard(idx, data, rank, world, device="cpu")
    q.put((rank, counts.numpy(), res.format(pydesamba.FMT_SAM), res.k))
    res.close()
    idx.close()
    dist.destroy_process_group()


def test_two_rank_shards_equal_one_whole_input_call(gpu_index, fixture_index, pyd):
    # long ONT reads on rank 0's side, only Illumina reads (< 510 bp) on rank 1's side
    ont = _records(golden("ont.fq"))[:300]
    ill = _records(golden("illumina.fq"))[:300]
    data = b"".join(ont + ill)
    whole, _, _ = gpu_index.classify(data, fmt=pyd.FMT_SAM)
    b = gpu_index.batch(data)
    b.run(max_read_l=0)
    tid, _ = b.taxa(0)
    b.close()
    want = np.bincount(tid.astype(np.int64), minlength=gpu_index.max_tid() + 1)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank, args=(r, 2, port, fixture_index, data, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = {}
    for _ in ps:
        r, c, sam, k = q.get(timeout=300)
        res[r] = (c, sam, k)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert res[1][2] == 300  # every short read of rank 1 re-ran with rank 0's carry
    assert res[0][1] + res[1][1] == whole
    for r in range(2):
        assert (res[r][0] == want).all()
    # how much the carry matters here: rank 1's reads classified alone (fresh carry)
    alone, _, _ = gpu_index.classify(b"".join(ill), fmt=pyd.FMT_SAM)
    ga, gw = groups(alone), groups(res[1][1])
    assert len(ga) == len(gw) == 300
    print(f"reads whose records depend on the carry: {sum(a != b for a, b in zip(ga, gw))} / 300")
