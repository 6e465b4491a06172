"""GPU parity on the bench workload (C1: the 56 Mbp proxy index of data/c1_index.txz, built by
the reference's own builder) and on the wave kernels' rarely taken paths.

* 1500 fresh C1 reads (lognormal mean 8 kb, 5-15 % error) against the reference compiled on this
  box (oracle/_ref): T1 taxid / mapped flag on every read, T2 full records on every read the
  reference itself reproduces across builds, T3 mismatches (hazard reads only) bounded.
* (The forced staging-overflow replay, DSB_WAVE_DBG=32, needs the test build of the library:
  tests/test_gpu_hooks.py.)
* Determinism: the same resident batch classified twice gives identical results.
"""
import os
import subprocess
import sys
import tarfile

import pytest

from conftest import ROOT
from samutil import compare, groups

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


def test_c1_reads_match_reference(c1_gpu, c1_index, tmp_path):
    """T1: primary taxid and mapped flag identical to the hermetic reference for every read.
    T2: full records identical for every read whose reference output does not depend on
    uninitialised memory, i.e. on which two reference builds (clang hermetic and gcc, both with
    fresh pools) agree.  T3 (every record identical to the hermetic build) holds on all but a
    few reads of that unstable kind, which are reported."""
    gcc = os.path.join(ROOT, "oracle", "_ref", "ref_classify")
    if not (os.path.exists(HERM) and os.path.exists(gcc)):
        pytest.skip("oracle/_ref not built")
    seed = int(os.environ.get("DSB_TEST_SEED", 4242 + int.from_bytes(os.urandom(2), "little")))
    fq = _reads(c1_index, 1500, seed, tmp_path)
    herm = subprocess.run([HERM, "--sam", c1_index, str(fq)], capture_output=True, check=True, timeout=600).stdout
    t1 = subprocess.run([gcc, "--sam", "--fresh", c1_index, str(fq)], capture_output=True, check=True,
                        timeout=600).stdout
    out, _, _ = c1_gpu.classify(fq.read_bytes(), fmt=1)
    r = compare(herm, out)
    assert r["taxid_mismatch"] == 0 and r["mapped_mismatch"] == 0, (seed, r)
    gh, gt, go = groups(herm), groups(t1), groups(out)
    stable = [i for i in range(len(gh)) if gh[i] == gt[i]]
    assert len(stable) >= 0.9 * len(gh), (seed, len(stable))
    bad = [gh[i][0] for i in stable if go[i] != gh[i]]
    assert not bad, (seed, bad[:5])
    unstable_diff = [gh[i][0] for i in range(len(gh)) if go[i] != gh[i]]
    assert len(unstable_diff) <= 0.005 * len(gh), (seed, unstable_diff[:5])
    print(f"seed {seed}: {len(gh)} reads, {len(stable)} stable, T3 mismatches {len(unstable_diff)} (all unstable)")


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
