"""GPU parity on the bench workload (C1: the 56 Mbp proxy index of data/c1_index.txz, built by
the reference's own builder) and on the wave kernels' rarely taken paths.

* 1500 fresh C1 reads (lognormal mean 8 kb, 5-15 % error): every SAM record byte-identical to
  the hermetic reference (oracle/_ref/herm_classify) run on this box.
* Forced staging overflow (DSB_WAVE_DBG=32: two anchors of staging per lane), so every seed
  group of fast and slow seeding takes the in-order replay path: still byte-identical.
* Determinism: the same resident batch classified twice gives identical results.
"""
import os
import subprocess
import sys
import tarfile

import pytest

from conftest import ROOT, golden
from samutil import compare

pytestmark = pytest.mark.gpu

HERM = os.path.join(ROOT, "oracle", "_ref", "herm_classify")
C1 = os.path.join(ROOT, "data", "c1_index.txz")


@pytest.fixture(scope="module")
def c1_index(tmp_path_factory):
    if not os.path.exists(C1):
        pytest.skip("data/c1_index.txz absent (tools/make_c1_index.sh)")
    d = tmp_path_factory.mktemp("c1")
    with tarfile.open(C1) as t:
        t.extractall(d)
    return str(d)


@pytest.fixture(scope="module")
def c1_gpu(c1_index, pyd):
    idx = pyd.Index(c1_index)
    yield idx
    idx.close()


def _reads(index_dir, n, seed, tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import simulate
    genomes = simulate.read_fasta_genomes_from_index(index_dir)
    fq = tmp_path / f"c1_{seed}.fq"
    simulate.write_fastq(list(simulate.simulate_reads(genomes, n, seed, "ont", 8000)), str(fq))
    return fq


def test_c1_reads_byte_identical_to_hermetic_reference(c1_gpu, c1_index, tmp_path):
    if not os.path.exists(HERM):
        pytest.skip("oracle/_ref not built")
    seed = 4242 + int.from_bytes(os.urandom(2), "little")
    fq = _reads(c1_index, 1500, seed, tmp_path)
    ref = subprocess.run([HERM, "--sam", c1_index, str(fq)], capture_output=True, check=True, timeout=600).stdout
    out, _, _ = c1_gpu.classify(fq.read_bytes(), fmt=1)
    r = compare(ref, out)
    assert r["full_mismatch"] == 0, (seed, r)


def test_staging_overflow_replay_is_byte_identical(gpu_index):
    os.environ["DSB_WAVE_DBG"] = "32"
    try:
        for name in ("mixed", "ont", "ont_long"):
            out, _, _ = gpu_index.classify(golden(name + ".fq"), fmt=1)
            assert out == golden(name + ".herm.sam"), name
    finally:
        os.environ.pop("DSB_WAVE_DBG", None)


def test_c1_batch_runs_are_deterministic(c1_gpu, c1_index, tmp_path):
    fq = _reads(c1_index, 2000, 77, tmp_path)
    b = c1_gpu.batch(fq.read_bytes())
    try:
        b.run(max_read_l=0)
        first = b.format(1)
        b.run(max_read_l=0)
        assert b.format(1) == first
    finally:
        b.close()
